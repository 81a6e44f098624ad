"""In-process A/B of environment knobs on BASELINE config C5 (block Lanczos,
b = 32 fp32, power-law rows, n = 1e7): ms per step and the SpMM class, alpha
checked against the first configuration (the first 3 steps).
  python scripts/ab_c5.py "LZ_SEG_WIDE=0" "LZ_SEG_WIDE=1" [--rounds 3]"""
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
ap.add_argument("--m", type=int, default=10)
args = ap.parse_args()
lz = ge.load_package()
h = lz.Handle(0)
n, m = 10_000_000, args.m
A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
Ad = lz.CsrDevice.from_host(A)
B = torch.from_numpy(lz.uniform_B(n, 32, seed=3, dtype=np.float32)).cuda()
kw = dict(dtype=torch.float32, device="cuda")
q, al, be = torch.zeros(m * 32, **kw), torch.zeros(m, 32, 32, **kw), torch.zeros(m + 1, 32, 32, **kw)
Q0, Q1, W = (torch.zeros(n, 32, **kw) for _ in range(3))
base = dict(os.environ)
ref, res = None, {c: [] for c in args.cfgs}
for rnd in range(args.rounds):
    for c in args.cfgs:
        os.environ.clear()
        os.environ.update(base)
        for kv in c.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        h.block_lanczos_blas(Ad, B, 2, 5, q, al, be, Q0, Q1, W)
        torch.cuda.synchronize()
        h.prof_enable(True)
        t = time.perf_counter()
        h.block_lanczos_blas(Ad, B, m, 5, q, al, be, Q0, Q1, W)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / m * 1e3
        sp = h.prof_read(h.PROF_SPMM)[0] / m
        h.prof_enable(False)
        a = al[:3].cpu().numpy()
        if ref is None:
            ref = a
        d = float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))
        if not d < 1e-4:
            raise RuntimeError(f"alpha differs under {c}: {d}")
        res[c].append((ms, sp))
        print(f"round {rnd} [{c}] {ms:.3f} ms/step, spmm {sp:.3f} ms", flush=True)
print({c: (round(float(np.median([x[0] for x in v])), 3), round(float(np.median([x[1] for x in v])), 3))
       for c, v in res.items()})
