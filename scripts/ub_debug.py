"""Round 6 debug: the b = 32 fp32 solve under LZ_UB_DMA settings, each
compared with the first run (max |d| of q / alpha / beta / W per step)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
h = lz.Handle(0)
n, m = int(sys.argv[1]) if len(sys.argv) > 1 else 20_011, 4
A = lz.gen_powerlaw(n, 10.0, 2.1, max(2, n // 10), seed=n % 89, dtype=np.float32)
B = lz.uniform_B(A.n, 32, seed=9, dtype=np.float32)
Ad, Bd = lz.CsrDevice.from_host(A), torch.from_numpy(B).cuda()
kw = dict(dtype=torch.float32, device="cuda")
ref = None
for cfg in ["0", "0", "1", "1", "3", "0"]:
    os.environ["LZ_UB_DMA"] = cfg
    q, al, be = torch.zeros(m * 32, **kw), torch.zeros(m, 32, 32, **kw), torch.zeros(m + 1, 32, 32, **kw)
    Q0, Q1, W = (torch.full((A.n, 32), float("nan"), **kw) for _ in range(3))
    h.block_lanczos_blas(Ad, Bd, m, 84, q, al, be, Q0, Q1, W)
    torch.cuda.synchronize()
    out = [t.cpu().numpy() for t in (q, al, be, W)]
    if ref is None:
        ref = out
    d = [float(np.nanmax(np.abs(x - y))) for x, y in zip(out, ref)]
    dq = [float(np.max(np.abs(out[0][32 * j:32 * j + 32] - ref[0][32 * j:32 * j + 32]))) for j in range(m)]
    print(f"LZ_UB_DMA={cfg}: max|d| q {d[0]:.2e} alpha {d[1]:.2e} beta {d[2]:.2e} W {d[3]:.2e}  q per step {dq}",
          flush=True)
