"""FDTD validation loop (methods/fdtd.hpp:33-56): time ftdt_block on the
reference driver's matrix A(N) with b=16, hipGraph replay vs eager launches
(LZ_FDTD_GRAPH=0 in the environment selects eager)."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
steps = int(float(sys.argv[2])) if len(sys.argv) > 2 else 100000
b = int(sys.argv[3]) if len(sys.argv) > 3 else 16
A = lz.matrix_a(N)
n = A.n
h = lz.Handle(0)
Ad = lz.CsrDevice.from_host(A)
kw = dict(dtype=torch.float64, device="cuda")
U0 = torch.from_numpy(lz.rand_B(n, b)).cuda()
U, D, out = torch.empty(n, b, **kw), torch.empty(n, b, **kw), torch.empty(b, **kw)
h.ftdt_block(Ad, U0, 1000, 1.0, 0, U, D, out)
torch.cuda.synchronize()
t0 = time.perf_counter()
h.ftdt_block(Ad, U0, steps, 1.0, 0, U, D, out)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"workload": f"FDTD n={n} nnz={A.nnz} b={b} steps={steps}",
                  "graph": os.environ.get("LZ_FDTD_GRAPH", "1") != "0",
                  "s_total": round(dt, 3), "us_per_step": round(dt / steps * 1e6, 3),
                  "out0": float(out[0])}))
