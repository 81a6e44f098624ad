"""Per-block timeline of the wavefront step launch (LZ_WF_DBG=128 stamps,
lz_debug_wf_times) on the C3 operator: when each block starts and when its
consumers and updaters finish, summarised by XCD region (block & 7) -- the
launch's tail imbalance.

  python scripts/wf_times.py [--rounds 3] [--steps 10]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=10_000_000)
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b = args.n, 16
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    B = lz.uniform_B(n, b, 20261015)
    kw = dict(dtype=torch.float64, device="cuda")
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(B).cuda()
    m = args.steps
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
    G = torch.cuda.get_device_properties(0).multi_processor_count
    os.environ["LZ_WF_DBG"] = "128"
    for r in range(args.rounds):
        h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
        torch.cuda.synchronize()
        if h.device_error() != 0:
            raise RuntimeError("device error")
        st, ce, ue = h.wf_times(G)
        end = np.maximum(ce, ue)
        print(f"round {r}: start spread {st.max():.1f} us; block end min {end.min():.1f} median "
              f"{np.median(end):.1f} max {end.max():.1f} us; consumers-end minus updaters-end median "
              f"{np.median(ce - ue):.1f} us", flush=True)
        for x in range(8):
            sel = np.arange(x, G, 8)
            print(f"   region {x}: end min {end[sel].min():.1f} median {np.median(end[sel]):.1f} "
                  f"max {end[sel].max():.1f}; updaters end median {np.median(ue[sel]):.1f}", flush=True)


if __name__ == "__main__":
    main()
