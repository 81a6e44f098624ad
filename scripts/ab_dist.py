"""In-process A/B of the single-GPU C3 iteration against the row-partitioned
halo form at one rank (the code path the N > 1 bench runs), alternated over
several rounds on one operator: pass times from the handle's HIP-event
profiler, step time from events around the call, alpha compared.

  python scripts/ab_dist.py [--rounds 3] [--steps 10] [--comm] [--more]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--comm", action="store_true", help="create a one-rank RCCL communicator first")
    ap.add_argument("--more", action="store_true", help="also the single path on the halo CSR / other buffers")
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    if args.comm:
        h.comm_init(1, 0, lz.comm_unique_id())
    n, b, m, lc = args.n, 16, args.steps, 84
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    B = lz.uniform_B(n, b, 20261015)
    kw = dict(dtype=torch.float64, device="cuda")
    Bd = torch.from_numpy(B).cuda()
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Ad = lz.CsrDevice.from_host(A)
    Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
    ccol, rcnt, hrows = lz.halo_plan(A.col, np.asarray([0, n], np.int64), 0)
    h.halo_init(0, n, rcnt, hrows)
    Ah = lz.CsrDevice.from_host(lz.CsrHost(A.n, A.row_ptr, ccol, A.val), n_cols=n + int(hrows.size))
    X0, X1 = (torch.zeros(n + int(hrows.size), b, **kw) for _ in range(2))
    Q0b, Q1b, Wb = (torch.zeros(n, b, **kw) for _ in range(3))
    runs = {
        "single": lambda k: h.block_lanczos_blas(Ad, Bd, k, lc, q, alpha, beta, Q0, Q1, W),
        "halo1": lambda k: h.block_lanczos_halo(Ah, Bd, k, lc, 0, q, alpha, beta, X0, X1),
    }
    if args.more:  # which allocation matters: the CSR arrays or the blocks
        runs["single_Ah"] = lambda k: h.block_lanczos_blas(Ah, Bd, k, lc, q, alpha, beta, Q0, Q1, W)
        runs["single_newbufs"] = lambda k: h.block_lanczos_blas(Ad, Bd, k, lc, q, alpha, beta, Q0b, Q1b, Wb)
        runs["single_X0X1"] = lambda k: h.block_lanczos_blas(Ad, Bd, k, lc, q, alpha, beta, Q0, X1, X0)
    res = {c: {"p1": [], "p2": [], "it": []} for c in runs}
    ref = None
    for rnd in range(args.rounds):
        for c, run in runs.items():
            run(2)
            torch.cuda.synchronize()
            h.prof_enable(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(m)
            e1.record()
            torch.cuda.synchronize()
            p1, c1 = h.prof_read(h.PROF_SPMM_PASS)
            p2, c2 = h.prof_read(h.PROF_UPDATE_PASS)
            h.prof_enable(False)
            if h.device_error() != 0:
                raise RuntimeError(f"device error under {c}")
            a = alpha.cpu().numpy()
            if ref is None:
                ref = a
            d = float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))
            if not d < 1e-9:
                raise RuntimeError(f"alpha differs under {c}: {d}")
            r = res[c]
            r["p1"].append(p1 / c1)
            r["p2"].append(p2 / c2)
            r["it"].append(e0.elapsed_time(e1) / m)
            print(f"round {rnd} [{c}] pass1 {r['p1'][-1]:.4f} pass2 {r['p2'][-1]:.4f} step {r['it'][-1]:.4f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
