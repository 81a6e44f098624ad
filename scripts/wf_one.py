"""One block-Lanczos solve at C3 (n=1e7, 10 nnz/row, half-width 4096, b=16
fp64) for profilers: `--steps` steps after a warm-up solve, the step form
chosen by LZ_PASS_WF in the environment.

    rocprofv3 --pmc FETCH_SIZE -- python3 scripts/wf_one.py --steps 4
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--n", type=int, default=10_000_000)
args = ap.parse_args()
lz = ge.load_package()
h = lz.Handle(0)
n, b, m = args.n, 16, args.steps
A = lz.gen_banded(n, 10.0, 4096, 20261015)
Ad = lz.CsrDevice.from_host(A)
Bd = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
kw = dict(dtype=torch.float64, device="cuda")
q = torch.zeros(m * b, **kw)
alpha = torch.zeros(m, b, b, **kw)
beta = torch.zeros(m + 1, b, b, **kw)
Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
for _ in range(2):
    t0 = time.perf_counter()
    h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
    torch.cuda.synchronize()
    print(f"{m} steps in {(time.perf_counter() - t0) * 1e3:.2f} ms, device error {h.device_error()}", flush=True)
