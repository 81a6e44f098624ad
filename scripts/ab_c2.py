"""In-process A/B of environment knobs on BASELINE config C2 (single-vector
Lanczos, n = 1M, ~1e7 nnz, half band 4096, fp64): us per step, alpha checked
against the first configuration.   python scripts/ab_c2.py "LZ_VL_PF=0" "LZ_VL_PF=1" [--rounds 3]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("cfgs", nargs="+")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--m", type=int, default=200)
ap.add_argument("--no-check", action="store_true", help="kernels whose sums differ in order (alpha diverges over long runs)")
args = ap.parse_args()
lz = ge.load_package()
h = lz.Handle(0)
n = 1_000_000
A = lz.gen_banded(n, 10.0, 4096, 20261015)
Ad = lz.CsrDevice.from_host(A)
b = torch.from_numpy(lz.uniform_B(n, 1, 1)[:, 0].copy()).cuda()
m = args.m
kw = dict(dtype=torch.float64, device="cuda")
q, al, be = (torch.zeros(m, **kw) for _ in range(3))
ws = [torch.zeros(n, **kw) for _ in range(3)]
base = dict(os.environ)
ref = None
res = {c: [] for c in args.cfgs}
for rnd in range(args.rounds):
    for c in args.cfgs:
        os.environ.clear()
        os.environ.update(base)
        for kv in c.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        h.vector_lanczos(Ad, b, m, 84, q, al, be, *ws)
        torch.cuda.synchronize()
        t = time.perf_counter()
        h.vector_lanczos(Ad, b, m, 84, q, al, be, *ws)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t) / m * 1e6
        a = al.cpu().numpy()
        if ref is None:
            ref = a
        d = float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))
        if not args.no_check and not d < 1e-12:
            raise RuntimeError(f"alpha differs under {c}: {d}")
        res[c].append(us)
        print(f"round {rnd} [{c}] {us:.2f} us/step", flush=True)
print({c: round(float(np.median(v)), 2) for c, v in res.items()})
