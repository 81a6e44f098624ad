"""Debug: alpha with 16- vs 32-bit columns over n; device error word."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
lz = ge.load_package()
h = lz.Handle(0)
for n in [49952, 49953, 50021, 50176, 50177, 45000, 57344, 60013, 100003]:
    A = lz.gen_banded(n, 10.0, 16, seed=21)
    B = lz.uniform_B(A.n, 16, seed=4)
    Ad = lz.CsrDevice.from_host(A)
    res = {}
    for c in ("0", "1"):
        os.environ["LZ_PASS1_C16"] = c
        q, al, be = lz.run_block_lanczos(h, Ad, torch.from_numpy(B).cuda(), 1, 0)
        torch.cuda.synchronize()
        res[c] = (al.cpu().numpy(), h.device_error())
    print(n, "nnz", A.nnz, "dalpha", float(np.abs(res["0"][0] - res["1"][0]).max()), "err", res["0"][1], res["1"][1],
          flush=True)
