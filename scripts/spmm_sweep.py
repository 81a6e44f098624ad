"""GPU micro-benchmark of the SpMM kernels (hipEvent timing through the C ABI)."""
import json
import sys
import time

import numpy as np
import torch

import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge

lz = ge.load_package()
h = lz.Handle(0)
res = []


def bench_spmm(A, b, dtype=np.float64, reps=10):
    Ad = lz.CsrDevice.from_host(A if dtype == np.float64 else lz.CsrHost(A.n, A.row_ptr, A.col, A.val.astype(dtype)))
    td = torch.float64 if dtype == np.float64 else torch.float32
    X = torch.rand(A.n, b, dtype=td, device="cuda")
    Y = torch.empty(A.n, b, dtype=td, device="cuda")
    f = (lambda: h.spmm(Ad, X, Y)) if b > 1 else (lambda: h.spmv(Ad, X[:, 0].contiguous(), Y[:, 0]))
    f(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    sv = np.dtype(dtype).itemsize
    byt = A.nnz * (sv + 4) + (A.n + 1) * 8 + 2 * A.n * b * sv
    return ms, byt / ms / 1e6


n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
for hw in (64, 4096, 65536, n):
    t = time.time()
    A = lz.gen_banded(n, 10.0, hw, seed=20261015)
    for b in (1, 4, 16, 32):
        ms, gbs = bench_spmm(A, b)
        r = dict(n=n, hw=hw, b=b, dtype="f64", ms=round(ms, 4), GBs=round(gbs, 1), frac=round(gbs / 8000, 3))
        print(json.dumps(r), flush=True)
        res.append(r)
    ms, gbs = bench_spmm(A, 32, np.float32)
    print(json.dumps(dict(n=n, hw=hw, b=32, dtype="f32", ms=round(ms, 4), GBs=round(gbs, 1), frac=round(gbs / 8000, 3))), flush=True)
A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
ms, gbs = bench_spmm(A, 32, np.float32)
print(json.dumps(dict(n=n, matrix="powerlaw", nnz=A.nnz, maxdeg=int(np.diff(A.row_ptr).max()), b=32, dtype="f32", ms=round(ms, 4), GBs=round(gbs, 1))), flush=True)
