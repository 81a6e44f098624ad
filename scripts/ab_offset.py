"""Diagnostic: pass times of the C3 iteration against the distance between the
two residual buffers the passes alternate over (W and Q1 as slices of one
allocation, `gap` rows of 128 B apart), alternated over rounds in one process.

  python scripts/ab_offset.py --gaps 0,1,8,32,512,8192 [--rounds 2] [--steps 10]
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
    ap.add_argument("--gaps", default="0,1,8,32,512,8192")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=10_000_000)
    args = ap.parse_args()
    gaps = [int(g) for g in args.gaps.split(",")]
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b, m, lc = args.n, 16, args.steps, 84
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    B = lz.uniform_B(n, b, 20261015)
    kw = dict(dtype=torch.float64, device="cuda")
    Bd = torch.from_numpy(B).cuda()
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Ad = lz.CsrDevice.from_host(A)
    Q0 = torch.zeros(1, b, **kw)
    big = torch.zeros(2 * n + max(gaps), b, **kw)
    print(f"base address mod 2 MiB: {big.data_ptr() % (1 << 21)}", flush=True)
    ref = None
    for rnd in range(args.rounds):
        for g in gaps:
            W, Q1 = big[:n], big[n + g: 2 * n + g]
            run = lambda k: h.block_lanczos_blas(Ad, Bd, k, lc, q, alpha, beta, Q0, Q1, W)  # noqa: E731
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
                raise RuntimeError(f"device error at gap {g}")
            a = alpha.cpu().numpy()
            if ref is None:
                ref = a
            if not float(np.max(np.abs(a - ref)) / np.max(np.abs(ref))) < 1e-9:
                raise RuntimeError(f"alpha differs at gap {g}")
            print(f"round {rnd} gap {g:6d} rows ({g * 128 / 1024:8.1f} KiB): pass1 {p1 / c1:.4f} "
                  f"pass2 {p2 / c2:.4f} step {e0.elapsed_time(e1) / m:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
