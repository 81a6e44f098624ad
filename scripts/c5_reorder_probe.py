"""Experiment: C5 SpMM / iteration time on the power-law operator as generated
and relabelled by descending degree (P A P^T, B permuted alike)."""
import json, os, sys, time
import numpy as np
import scipy.sparse as sp
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n = 10_000_000
A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
deg = np.diff(A.row_ptr)
t = time.time()
perm = np.argsort(-deg, kind="stable")          # new row i = old row perm[i]
M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(n, n))
Mp = M[perm][:, perm].tocsr()
Mp.sort_indices()
Ap = lz.CsrHost(n, Mp.indptr.astype(np.int64), Mp.indices.astype(np.int32), Mp.data.astype(np.float32))
print(f"permute {time.time()-t:.1f}s", file=sys.stderr)
B = lz.uniform_B(n, 32, seed=3, dtype=np.float32)
out = {}
for name, AA, BB in (("natural", A, B), ("degree_sorted", Ap, B[perm])):
    Ad = lz.CsrDevice.from_host(AA)
    Bd = torch.from_numpy(np.ascontiguousarray(BB)).cuda()
    Y = torch.empty(n, 32, dtype=torch.float32, device="cuda")
    h.spmm(Ad, Bd, Y); torch.cuda.synchronize()
    h.prof_enable(True)
    for _ in range(10): h.spmm(Ad, Bd, Y)
    torch.cuda.synchronize()
    ms, c = h.prof_read(h.PROF_SPMM); h.prof_enable(False)
    m = 10
    kw = dict(dtype=torch.float32, device="cuda")
    q, al, be = torch.zeros(m * 32, **kw), torch.zeros(m, 32, 32, **kw), torch.zeros(m + 1, 32, 32, **kw)
    P = [torch.zeros(n, 32, **kw) for _ in range(3)]
    h.block_lanczos_blas(Ad, Bd, 2, 5, q, al, be, *P); torch.cuda.synchronize()
    t0 = time.perf_counter(); h.block_lanczos_blas(Ad, Bd, m, 5, q, al, be, *P); torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[name] = {"spmm_ms": round(ms / c, 4), "iter_ms": round(dt / m * 1e3, 3), "alpha0_trace": float(al[0].trace())}
    del Ad, Bd, Y, P
    torch.cuda.empty_cache()
print(json.dumps(out))
