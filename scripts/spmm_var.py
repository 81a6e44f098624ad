"""One SpMM variant (LZ_SPMM_KERNEL, read once per process) on the C3 operator:
average kernel time from HIP events on the handle's stream, and a checksum of Y
so variants can be compared across processes (same arithmetic order -> equal)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
hw = int(float(sys.argv[2])) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
b = 16
A = lz.gen_banded(n, 10.0, hw, seed=20261015)
Ad = lz.CsrDevice.from_host(A)
X = torch.from_numpy(lz.uniform_B(n, b, 5)).cuda()
Y = torch.empty(n, b, dtype=torch.float64, device="cuda")
h.spmm(Ad, X, Y); torch.cuda.synchronize()
h.prof_enable(True)
for _ in range(reps):
    h.spmm(Ad, X, Y)
torch.cuda.synchronize()
ms, cnt = h.prof_read(h.PROF_SPMM)
h.prof_enable(False)
t = ms / cnt
byt = A.nnz * 12 + (n + 1) * 8 + 2 * n * b * 8
print(json.dumps(dict(variant=os.environ.get("LZ_SPMM_KERNEL", "default"), n=n, hw=hw, ms=round(t, 4),
                      GBs=round(byt / t / 1e6, 1), ysum=float(Y.sum()), err=h.device_error())), flush=True)
