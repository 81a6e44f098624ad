"""The column-panel SpMM candidate (lz_panel.hip) against the nnz-split gather
kernel (k_spmm_seg, lz_csr_spmm) at C3 (n = 1e7, 10 nnz/row, half width 4096,
b = 16 fp64), alternating in one process; Y of both checked against each other
(64 eps bound).  Prints the plan's size and build time and both kernels' ms per
launch and HBM fraction on the SpMM's algorithmic bytes (z*12 + (n+1)*8 + 2nbs).

  python scripts/panel_ab.py [--rounds 5] [--reps 20] [--n 10000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--halfwidth", type=int, default=4096)
    ap.add_argument("--which", default="both", choices=["both", "panel", "seg"])
    args = ap.parse_args()
    lz = ge.load_package()
    n, b = args.n, 16
    A = lz.gen_banded(n, 10.0, args.halfwidth, 20261015)
    t0 = time.time()
    pl = lz.panel_plan(A)
    t_plan = time.time() - t0
    npass = int(pl.px0.size)
    h = lz.Handle(0)
    Ad = lz.CsrDevice.from_host(A)
    pd = pl.device()
    X = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
    Y1 = torch.empty(n, b, dtype=torch.float64, device="cuda")
    Y2 = torch.empty_like(Y1)
    h.spmm(Ad, X, Y1)
    h.spmm_panel(pd, n, pl.nblocks, X, Y2)
    torch.cuda.synchronize()
    d = float((Y1 - Y2).abs().max().item())
    scale = float(Y1.abs().max().item())
    alg = A.nnz * 12 + (n + 1) * 8 + 2 * n * b * 8
    stream = pl.ev.nbytes + pl.ex.nbytes + pl.goff.nbytes + pl.pe0.nbytes + pl.px0.nbytes
    res = {"seg": [], "panel": []}
    for rnd in range(args.rounds):
        for k in ("seg", "panel"):
            if args.which not in ("both", k):
                continue
            fn = (lambda: h.spmm(Ad, X, Y1)) if k == "seg" else (lambda: h.spmm_panel(pd, n, pl.nblocks, X, Y2))
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / args.reps)
        print(f"round {rnd}: " + "  ".join(f"{k} {v[-1]:.4f} ms" for k, v in res.items() if v), flush=True)
    out = {"n": n, "nnz": int(A.nnz), "halfwidth": args.halfwidth, "plan_s": round(t_plan, 1), "passes": npass,
           "plan_entries_padded": int(pl.pe0[-1]), "plan_stream_bytes": int(stream),
           "max_abs_diff_vs_seg": d, "rel": d / scale, "alg_bytes": alg}
    for k, v in res.items():
        if v:
            ms = float(np.median(v))
            out[k] = {"ms": round(ms, 4), "GBs": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / 8000, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
