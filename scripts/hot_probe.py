"""MALL-residency probe for the C5 SpMM (diagnostic build, LZ_HIP_LIB): the C5
operator (n = 1e7, power-law degrees, b = 32 fp32) with its COLUMNS relabelled
by descending degree (Y = A P^T (P X): the same products, X's rows permuted),
so that "hot" = column < K.  Configurations (environment, read per call):
  LZ_SPMM_HOT="K,a"  gathers of columns < K with the default policy, the rest
                     with a = 1: nt, 2: sc1, 3: sc1 nt
Also the operator as generated ("orig"), to see what the relabelling alone does.
Alternating, one process; 20 launches per sample; Y compared bitwise.

  LZ_HIP_LIB=.../liblz_hip_diag.so python scripts/hot_probe.py "" "LZ_SPMM_HOT=1500000,1" ... [--rounds 3]
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
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--orig", action="store_true", help="also time the operator as generated")
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b = args.n, 32
    A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
    deg = np.diff(np.asarray(A.row_ptr))
    order = np.argsort(-deg, kind="stable")          # new label -> old row
    newlab = np.empty(n, dtype=np.int64)
    newlab[order] = np.arange(n)                      # old row -> new label
    colr = newlab[np.asarray(A.col)].astype(np.asarray(A.col).dtype)
    Ar = lz.CsrHost(A.n, A.row_ptr, colr, A.val)
    B = lz.uniform_B(n, b, 20261015, dtype=np.float32)
    Br = np.ascontiguousarray(B[order])              # P X: row new = old row order[new]
    cum = np.cumsum(np.sort(deg)[::-1]) / deg.sum()
    print("gathers to the top K rows:", {k: round(float(cum[k - 1]), 3) for k in (500_000, 1_000_000, 1_500_000,
                                                                                  2_000_000, 3_000_000)}, flush=True)
    ops = {"relab": (lz.CsrDevice.from_host(Ar), torch.from_numpy(Br).cuda())}
    if args.orig:
        ops["orig"] = (lz.CsrDevice.from_host(A), torch.from_numpy(B).cuda())
    Y = torch.empty(n, b, dtype=torch.float32, device="cuda")
    runs = [(o, c) for o in ops for c in args.cfgs] if args.orig else [("relab", c) for c in args.cfgs]
    res = {f"{o}|{c}": [] for o, c in runs}
    yref = {}
    base_env = dict(os.environ)
    for rnd in range(args.rounds):
        for o, c in runs:
            os.environ.clear()
            os.environ.update(base_env)
            for kv in c.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            Ad, Xd = ops[o]
            h.spmm(Ad, Xd, Y)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                h.spmm(Ad, Xd, Y)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 20
            if h.device_error() != 0:
                raise RuntimeError(f"device error under {o} {c}")
            if o not in yref:
                yref[o] = Y.clone()
            elif not torch.equal(Y, yref[o]):
                raise RuntimeError(f"SpMM result differs under {o} {c}")
            res[f"{o}|{c}"].append(t)
            print(f"round {rnd} [{o}] [{c}] spmm {t:.4f} ms", flush=True)
    if "orig" in yref:  # the relabelled product is the same rows, same sums in the same order
        same = torch.equal(yref["orig"], yref["relab"])
        print("orig == relab bitwise:", same)
    print(json.dumps({k: round(float(np.median(v)), 4) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
