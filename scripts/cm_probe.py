"""Column-major SpMM (the reference's Dense_matrix layout) at the reference's
harness size: Yee N=160, b=16 fp32; run under rocprofv3 --kernel-trace --stats
to split the X transpose from the SpMM with its column-major Y store."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
A64 = lz.matrix_a(160)
n, b = A64.n, 16
Ad = lz.CsrDevice.from_host(lz.CsrHost(n, A64.row_ptr, A64.col, A64.val.astype(np.float32)))
f32 = dict(dtype=torch.float32, device="cuda")
Xc, Yc = torch.rand(b, n, **f32), torch.empty(b, n, **f32)
X, Y = torch.rand(n, b, **f32), torch.empty(n, b, **f32)
for _ in range(10):
    h.spmm(Ad, Xc, Yc, layout=lz.LZ_COL_MAJOR)
    h.spmm(Ad, X, Y)
torch.cuda.synchronize()
print("ok")
