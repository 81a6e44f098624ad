"""Debug: the wavefront step's first launch (m = 1): Y_0 (left in Q0) against
A @ B, and alpha_0, per block shape and column width."""
import os
import sys

import numpy as np
import scipy.sparse as sps
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
orc = ge.load_oracle()
h = lz.Handle(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
A = lz.gen_banded(n, 10.0, 16, 20261015)
B = lz.uniform_B(n, 16, 7)
S = sps.csr_matrix((A.val, A.col, A.row_ptr), shape=(n, n))
Yref = S @ B
Ad = lz.CsrDevice.from_host(A)
Bd = torch.from_numpy(B).cuda()
kw = dict(dtype=torch.float64, device="cuda")
for shape in ("10", "11", "12"):
    for c16 in ("0", "1"):
        os.environ["LZ_WF_SHAPE"], os.environ["LZ_PASS1_C16"] = shape, c16
        m = 1
        q = torch.zeros(m * 16, **kw)
        al = torch.zeros(m, 16, 16, **kw)
        be = torch.zeros(m + 1, 16, 16, **kw)
        Q0, Q1, W = (torch.zeros(n, 16, **kw) for _ in range(3))
        h.block_lanczos_blas(Ad, Bd, m, 84, q, al, be, Q0, Q1, W)
        torch.cuda.synchronize()
        Y = Q0.cpu().numpy()
        dy = np.abs(Y - Yref)
        bad = np.argwhere(dy > 1e-12 * np.abs(Yref).max())
        print(f"shape {shape} c16 {c16}: max|dY| {dy.max():.2e}, bad entries {len(bad)}, first rows "
              f"{sorted(set(bad[:, 0].tolist()))[:12]} err {h.device_error()}", flush=True)
