"""The wavefront step (LZ_PASS_WF, lz_wf.hip) against the CPU oracle and the
two-pass step, over operator sizes that exercise its edge cases (fewer tiles
than regions, a last partial tile, wide and narrow bands), then an in-process
A/B at C3.

  python scripts/wf_check.py [--ab-rounds 3] [--steps 20]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
from bench import RITZ_TOL, compare_run  # noqa: E402


def run(lz, h, Ad, Bd, m, lc, wf):
    os.environ["LZ_PASS_WF"] = "1" if wf else "0"
    q, al, be = lz.run_block_lanczos(h, Ad, Bd, m, lc)
    torch.cuda.synchronize()
    err = h.device_error()
    if err:
        raise SystemExit(f"device error {err} (wf={wf})")
    return q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ab-rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    lz = ge.load_package()
    orc = ge.load_oracle()
    h = lz.Handle(0)
    cases = [(1000, 10.0, 16), (5000, 10.0, 64), (60013, 10.0, 4096), (200003, 10.0, 2048), (1_000_000, 10.0, 4096),
             (777_777, 10.0, 8192)]
    for n, npr, hw in cases:
        A = lz.gen_banded(n, npr, hw, 20261015)
        B = lz.uniform_B(n, 16, 7)
        Ad = lz.CsrDevice.from_host(A)
        Bd = torch.from_numpy(B).cuda()
        m, lc = 8, min(84, n - 1)
        t0 = time.time()
        qo, ao, bo = orc.block_lanczos(A, B, m, lc)
        got = run(lz, h, Ad, Bd, m, lc, True)
        two = run(lz, h, Ad, Bd, m, lc, False)
        par = compare_run(lz, m, 16, (got[1], got[2], got[0]), (ao, bo, qo), 1e-9, RITZ_TOL)
        d2 = float(np.abs(got[1] - two[1]).max() / np.abs(two[1]).max())
        print(f"n={n} npr={npr} hw={hw}: parity {par['ok']} max_dritz {par['max_dritz']:.1e} "
              f"alpha vs two-pass {d2:.2e} ({time.time() - t0:.1f}s)", flush=True)
        if not par["ok"] or not d2 < 1e-9:
            raise SystemExit(f"wavefront step mismatch: {par}")
    # reproducibility: the same solve twice, bitwise
    n = 1_000_000
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(lz.uniform_B(n, 16, 20261015)).cuda()
    r1, r2 = run(lz, h, Ad, Bd, 10, 84, True), run(lz, h, Ad, Bd, 10, 84, True)
    same = all(np.array_equal(x, y) for x, y in zip(r1, r2))
    print("bitwise reproducible:", same, flush=True)
    if not same:
        raise SystemExit("not reproducible")
    # C3 timing A/B (no per-launch events: whole-iteration time)
    n, b, m = 10_000_000, 16, args.steps
    A = lz.gen_banded(n, 10.0, 4096, 20261015)
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
    kw = dict(dtype=torch.float64, device="cuda")
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.zeros(n, b, **kw) for _ in range(3))
    res = {"0": [], "1": []}
    ref = None
    for rnd in range(args.ab_rounds):
        for wf in ("0", "1"):
            os.environ["LZ_PASS_WF"] = wf
            h.block_lanczos_blas(Ad, Bd, 2, 84, q, alpha, beta, Q0, Q1, W)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.block_lanczos_blas(Ad, Bd, 2, 84, q, alpha, beta, Q0, Q1, W)
            e1.record()
            torch.cuda.synchronize()
            t2 = e0.elapsed_time(e1)
            e0.record()
            h.block_lanczos_blas(Ad, Bd, m, 84, q, alpha, beta, Q0, Q1, W)
            e1.record()
            torch.cuda.synchronize()
            marg = (e0.elapsed_time(e1) - t2) / (m - 2)
            print(f"   LZ_PASS_WF={wf}: marginal {marg:.4f} ms/step, set-up + 2 steps {t2:.3f} ms", flush=True)
            if h.device_error():
                raise SystemExit(f"device error at C3 (wf={wf})")
            a = alpha.cpu().numpy()
            if ref is None:
                ref = a
            d = float(np.abs(a - ref).max() / np.abs(ref).max())
            ms = e0.elapsed_time(e1) / m
            res[wf].append(ms)
            print(f"round {rnd} LZ_PASS_WF={wf}: {ms:.4f} ms/step ({1e3 / ms:.1f} it/s), alpha vs first {d:.1e}",
                  flush=True)
            if not d < 1e-9:
                raise SystemExit("C3 alpha mismatch")
    print({k: round(float(np.median(v)), 4) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
