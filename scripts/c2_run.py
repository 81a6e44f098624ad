"""BASELINE config 1 (single-vector Lanczos, n=1M, nnz~1e7) for profiling."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n = 1_000_000
A = lz.gen_banded(n, 10.0, 4096, 20261015)
Ad = lz.CsrDevice.from_host(A)
b = torch.from_numpy(lz.uniform_B(n, 1, 1)[:, 0].copy()).cuda()
m = 200
kw = dict(dtype=torch.float64, device="cuda")
q, al, be = (torch.zeros(m, **kw) for _ in range(3))
ws = [torch.zeros(n, **kw) for _ in range(3)]
for _ in range(3):
    h.vector_lanczos(Ad, b, m, 84, q, al, be, *ws)
torch.cuda.synchronize()
t = time.perf_counter()
h.vector_lanczos(Ad, b, m, 84, q, al, be, *ws)
torch.cuda.synchronize()
print("us/iter", (time.perf_counter() - t) / m * 1e6)
