"""In-process A/B of kernel knobs read per call (environment variables) on the
C3 operator (n=1e7, 10 nnz/row, half-width 4096, b=16 fp64): one operator
build, configurations alternated over several rounds, pass times from the
handle's HIP-event profiler, alpha checked against the first configuration.

  python scripts/ab_c3.py "LZ_WF_SHAPE=111" "LZ_WF_SHAPE=11" ... [--rounds 3] [--steps 10] [--spmm]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfgs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--nnz-per-row", type=float, default=10.0)
    ap.add_argument("--halfwidth", type=int, default=4096)
    ap.add_argument("--spmm", action="store_true", help="also time the plain SpMM (20 launches)")
    ap.add_argument("--spmm-only", action="store_true", help="time only the plain SpMM")
    ap.add_argument("--colmod", type=int, default=0, help="diagnostic: columns mod this (an L2-resident X window)")
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b = args.n, 16
    A = lz.gen_banded(n, args.nnz_per_row, args.halfwidth, 20261015)
    B = lz.uniform_B(n, b, 20261015)
    kw = dict(dtype=torch.float64, device="cuda")
    if args.colmod:
        A = lz.CsrHost(A.n, A.row_ptr, (A.col % args.colmod).astype(A.col.dtype), A.val)
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(B).cuda()
    m = args.steps
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
    Y = torch.empty(n, b, **kw)
    ref = None
    yref = None
    res = {c: {"p1": [], "p2": [], "it": [], "spmm": [], "dalpha": []} for c in args.cfgs}
    base_env = dict(os.environ)
    for rnd in range(args.rounds):
        for c in args.cfgs:
            os.environ.clear()
            os.environ.update(base_env)
            for kv in c.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            r = res[c]
            if hasattr(h.L, "lz_set_final_state"):  # (a round-3 build has no post-call state pass)
                h.set_final_state(os.environ.get("AB_FS", "1") == "1")  # AB_FS=0: skip the post-call state pass
            if not args.spmm_only:
                h.block_lanczos_blas(Ad, Bd, 2, 84, q, alpha, beta, Q0, Q1, W)  # warm-up
                torch.cuda.synchronize()
                h.prof_enable(True)
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
                ev1.record()
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
                r.setdefault("dalpha", []).append(d)
                if not d < 1e-9 and "LZ_WF_DBG" not in c:  # measurement switches
                    raise RuntimeError(f"alpha differs under {c}: {d}")
                r["p1"].append(p1 / c1)
                r["p2"].append(p2 / c2 if c2 else 0.0)
                r["it"].append(ev0.elapsed_time(ev1) / m)
            if args.spmm or args.spmm_only:
                h.spmm(Ad, Bd, Y)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    h.spmm(Ad, Bd, Y)
                e1.record()
                torch.cuda.synchronize()
                r["spmm"].append(e0.elapsed_time(e1) / 20)
                if yref is None:
                    yref = Y.clone()
                dy = float((Y - yref).abs().max().item())
                if not dy <= 1e-12 * float(yref.abs().max().item()) and "LZ_SPMM_DIAG" not in c:
                    raise RuntimeError(f"SpMM result differs under {c}: {dy}")
            line = f"round {rnd} [{c}]"
            if r["p1"]:
                line += f" pass1 {r['p1'][-1]:.4f} pass2 {r['p2'][-1]:.4f} iter {r['it'][-1]:.4f} ms"
            if r["spmm"]:
                line += f" spmm {r['spmm'][-1]:.4f} ms"
            print(line, flush=True)
    summary = {c: {k: round(float(np.median(v)), 4) for k, v in r.items() if v} for c, r in res.items()}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
