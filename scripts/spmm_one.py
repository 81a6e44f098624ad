"""Run one SpMM configuration a few times (for rocprofv3 counter passes)."""
import sys
import numpy as np
import torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n, hw, b = int(float(sys.argv[1])), int(float(sys.argv[2])), int(sys.argv[3])
A = lz.gen_banded(n, 10.0, hw, seed=20261015)
Ad = lz.CsrDevice.from_host(A)
X = torch.rand(n, b, dtype=torch.float64, device="cuda")
Y = torch.empty(n, b, dtype=torch.float64, device="cuda")
for _ in range(5):
    h.spmm(Ad, X, Y)
torch.cuda.synchronize()
print("done", A.nnz)
