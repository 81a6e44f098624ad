"""A/B of SpMM kernel variants on one operator (variant via LZ_SPMM_KERNEL env)."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
n, hw, b = int(float(sys.argv[1])), int(float(sys.argv[2])), int(sys.argv[3])
A = lz.gen_banded(n, 10.0, hw, seed=20261015)
Ad = lz.CsrDevice.from_host(A)
X = torch.rand(n, b, dtype=torch.float64, device="cuda")
Y = torch.empty(n, b, dtype=torch.float64, device="cuda")
h.spmm(Ad, X, Y); torch.cuda.synchronize()
ref = Y.clone()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    h.spmm(Ad, X, Y)
e.record(); torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
byt = A.nnz * 12 + (n + 1) * 8 + 2 * n * b * 8
err = h.device_error()
print(json.dumps(dict(err=err, variant=os.environ.get("LZ_SPMM_KERNEL", "buf"),
                      n=n, hw=hw, b=b, ms=round(ms, 4), GBs=round(byt / ms / 1e6, 1), same=bool(torch.equal(ref, Y)) if os.environ.get("LZ_SPMM_KERNEL","")[2:3] == "" else None)), flush=True)
