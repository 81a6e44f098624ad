"""BASELINE config 4 (block Lanczos b=32 fp32, power-law-degree CSR): time and
per-kernel-class split (HIP events on the handle's stream)."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 10
t = time.time()
A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
print(f"gen n={A.n} nnz={A.nnz} max_row={int(np.diff(A.row_ptr).max())} in {time.time()-t:.1f}s", file=sys.stderr)
Ad = lz.CsrDevice.from_host(A)
B = torch.from_numpy(lz.uniform_B(n, 32, seed=3, dtype=np.float32)).cuda()
kw = dict(dtype=torch.float32, device="cuda")
q, al, be = torch.zeros(m * 32, **kw), torch.zeros(m, 32, 32, **kw), torch.zeros(m + 1, 32, 32, **kw)
Q0, Q1, W = (torch.zeros(n, 32, **kw) for _ in range(3))
h.block_lanczos_blas(Ad, B, 2, 5, q, al, be, Q0, Q1, W)
torch.cuda.synchronize()
h.prof_enable(True)
t0 = time.perf_counter()
h.block_lanczos_blas(Ad, B, m, 5, q, al, be, Q0, Q1, W)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
names = ["fused_spmm_pass", "update_pass", "small", "gram", "tsmm", "spmm"]
split = {nm: round(h.prof_read(i)[0] / m, 4) for i, nm in enumerate(names)}
h.prof_enable(False)
spmm_bytes = A.nnz * 8 + (n + 1) * 8 + 2 * n * 32 * 4
print(json.dumps({"workload": f"C5 block Lanczos b=32 fp32 power-law n={n} nnz={A.nnz}", "iters_per_s": round(m / dt, 2),
                  "ms_per_iter": round(dt / m * 1e3, 3), "ms_per_iter_by_class": split,
                  "spmm_GBs": round(spmm_bytes / (split["spmm"] * 1e-3) / 1e9, 1) if split["spmm"] else None}))
