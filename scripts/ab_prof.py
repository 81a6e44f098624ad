"""Cost of the handle's HIP-event profiler inside a timed C3 run: the same
20-step block_lanczos_blas call with lz_prof_enable off and on, alternated.

  python scripts/ab_prof.py [--rounds 3] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b, m = 10_000_000, 16, args.steps
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
    kw = dict(dtype=torch.float64, device="cuda")
    q = torch.zeros(m * b, **kw)
    alpha, beta = torch.zeros(m, b, b, **kw), torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
    h.block_lanczos_blas(Ad, Bd, 3, 84, q, alpha, beta, Q0, Q1, W)
    torch.cuda.synchronize()
    for rnd in range(args.rounds):
        for prof in (False, True):
            h.prof_enable(prof)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / m * 1e3
            h.prof_enable(False)
            print(f"round {rnd} prof={int(prof)} {dt:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
