"""Where the wavefront step's sqrtm block spends the launch (LZ_WF_DBG=128
stamps, lz_debug_wf_stamps): C3 operator, one solve per round, the last step
launch's stamps in microseconds after its start.

  python scripts/wf_stamps.py [--rounds 5] [--steps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
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
    os.environ["LZ_WF_DBG"] = "128"
    names = ["wait done", "fold done", "sqrtm done", "last wavefront block end", "last G slab stored"]
    for r in range(args.rounds):
        h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
        torch.cuda.synchronize()
        st = h.wf_stamps()
        print(f"round {r}: " + ", ".join(f"{k} {v:.1f}" for k, v in zip(names, st)), flush=True)
        if h.device_error() != 0:
            raise RuntimeError("device error")


if __name__ == "__main__":
    main()
