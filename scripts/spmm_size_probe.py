"""How the b = 16 fp64 SpMM's time per nonzero depends on where its CSR
stream lives: the same banded operator (10 nnz/row, half-width 4096) at
n = 0.5M .. 10M rows (CSR 64 MB .. 1.28 GB: MALL-resident when the SpMM is
replayed back to back at the small sizes, HBM at C3)."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
for n in (500_000, 1_000_000, 2_000_000, 4_000_000, 10_000_000):
    A = lz.gen_banded(n, 10.0, 4096, seed=20261015)
    Ad = lz.CsrDevice.from_host(A)
    X = torch.rand(n, 16, dtype=torch.float64, device="cuda")
    Y = torch.empty(n, 16, dtype=torch.float64, device="cuda")
    for _ in range(3):
        h.spmm(Ad, X, Y)
    torch.cuda.synchronize()
    h.prof_enable(True)
    for _ in range(20):
        h.spmm(Ad, X, Y)
    torch.cuda.synchronize()
    ms, c = h.prof_read(h.PROF_SPMM)
    h.prof_enable(False)
    t = ms / c
    byt = A.nnz * 12 + (n + 1) * 8 + 2 * n * 16 * 8
    print(json.dumps({"n": n, "nnz": A.nnz, "csr_MB": round((A.nnz * 12 + (n + 1) * 8) / 1e6, 1), "ms": round(t, 4),
                      "ns_per_knnz": round(t * 1e9 / A.nnz, 3), "GBs": round(byt / t / 1e6, 1)}), flush=True)
    del Ad, X, Y
