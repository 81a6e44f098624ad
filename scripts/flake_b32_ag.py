"""Repeat the b = 32 fp32 virtual-rank solve (test_vranks_b32_f32) in one
process and report whether its alpha is bitwise the same every run, per
configuration (environment settings), and the first step whose alpha differs
from the first run's.  Diagnoses a result that differs between runs (a race).

  python scripts/flake_b32_ag.py REPS FORM "ENV=V ..." ["ENV=V ..." ...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402
from test_gpu_vranks import run_dist  # noqa: E402

lz, orc = ge.load_package(), ge.load_oracle()
reps, form, cfgs = int(sys.argv[1]), sys.argv[2], sys.argv[3:] or [""]
A = lz.gen_banded(20_011, 10.0, 600, seed=30, dtype=np.float32)
B = lz.uniform_B(A.n, 32, seed=31, dtype=np.float32)
m, lc = 5, 15_000
qo, ao, bo = orc.block_lanczos(A, B, m, lc)
scale = max(1.0, float(np.abs(ao).max()), float(np.abs(bo[:m]).max()))
base = dict(os.environ)
for c in cfgs:
    os.environ.clear()
    os.environ.update(base)
    for kv in c.split():
        k, v = kv.split("=", 1)
        os.environ[k] = v
    first, errs, diffs = None, [], []
    for r in range(reps):
        (q, al, be), _ = run_dist(lz, torch, A, B, m, lc, 2, form)
        errs.append(float(np.max(np.abs(al - ao))) / scale)
        if first is None:
            first = (al.copy(), be.copy())
        else:
            da = [j for j in range(m) if not np.array_equal(al[j], first[0][j])]
            db = [j for j in range(m) if not np.array_equal(be[j], first[1][j])]
            if da or db:
                diffs.append(f"run {r}: alpha steps {da} beta steps {db}")
    print(f"{form} [{c}]: {reps - 1 - len(diffs)}/{reps - 1} runs bitwise equal to the first; rel |dalpha| "
          f"max {max(errs):.2e} (tol 1e-4); " + "; ".join(diffs), flush=True)
