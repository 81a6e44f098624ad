"""In-process A/B of the single-vector Lanczos step at C2 (n = 1M, 10 nnz/row,
half width 4096, fp64): configurations (environment variables read per call)
alternated over rounds, microseconds per step of an m-step solve, alpha / beta
checked against the first configuration.

  python scripts/ab_c2.py "LZ_VL_KERNEL=win1024" "LZ_VL_KERNEL=row" [--rounds 4] [--steps 200]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfgs", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", "--m", type=int, default=200)
    ap.add_argument("--no-check", action="store_true", help="skip the alpha / beta comparison")
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, m = 1_000_000, args.steps
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    Ad = lz.CsrDevice.from_host(A)
    kw = dict(dtype=torch.float64, device="cuda")
    b = torch.from_numpy(lz.uniform_B(n, 1, 20261015)[:, 0].copy()).cuda()
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m + 1, **kw)
    q0, q1, w = (torch.zeros(n, **kw) for _ in range(3))
    base = dict(os.environ)
    res = {c: [] for c in args.cfgs}
    ref = None
    for rnd in range(args.rounds):
        for c in args.cfgs:
            os.environ.clear()
            os.environ.update(base)
            for kv in c.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            h.vector_lanczos(Ad, b, 3, 84, q, al, be, q0, q1, w)  # warm-up
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.vector_lanczos(Ad, b, m, 84, q, al, be, q0, q1, w)
            e1.record()
            torch.cuda.synchronize()
            a = np.concatenate([al.cpu().numpy(), be[:m].cpu().numpy()])
            if ref is None:
                ref = a
            d = float(np.max(np.abs(a[:30] - ref[:30])) / np.max(np.abs(ref[:30])))
            if not d < 1e-9 and not args.no_check:
                raise RuntimeError(f"alpha/beta (first 15 steps) differ under {c}: {d}")
            res[c].append(e0.elapsed_time(e1) * 1e3 / m)
            print(f"round {rnd} [{c}] {res[c][-1]:.2f} us/step  d(first 15 steps) {d:.1e}", flush=True)
    print(json.dumps({c: round(float(np.median(v)), 2) for c, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
