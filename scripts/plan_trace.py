"""One C3 solve per configuration (for a rocprofv3 kernel trace): beta_0's Gram
on the side stream beside the plans or on the main stream, 2 solves each.
  python scripts/plan_trace.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

lz = ge.load_package()
h = lz.Handle(0)
n, b = 10_000_000, 16
A = lz.gen_banded(n, 10.0, 4096, 20261015)
Ad = lz.CsrDevice.from_host(A)
Bd = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
for cfg in ({"LZ_GRAM_SIDE": "0"}, {"LZ_GRAM_SIDE": "1"}) * 2:
    os.environ.update(cfg)
    lz.run_block_lanczos(h, Ad, Bd, 3, 84)
    torch.cuda.synchronize()
print("done")
