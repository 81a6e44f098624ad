"""In-process A/B on BASELINE config C5 (b = 32 fp32, power-law rows, n = 10M):
configurations (environment variables read per call) alternated over rounds,
ms per block step of an m-step solve and the SpMM class time, alpha checked
against the first configuration (fp32: 1e-4 relative).

  python scripts/ab_c5.py "LZ_C5_B2=1" "LZ_C5_B2=0" [--rounds 3] [--steps 10]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--banded", type=int, default=0, help="a banded operator of this half width instead (10 nnz/row)")
    args = ap.parse_args()
    lz = ge.load_package()
    h = lz.Handle(0)
    n, b, m = 10_000_000, 32, args.steps
    if args.banded:
        A = lz.gen_banded(n, 10.0, args.banded, 20261015, dtype=np.float32)
    else:
        A = lz.gen_powerlaw(n, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
    Ad = lz.CsrDevice.from_host(A)
    B = torch.from_numpy(lz.uniform_B(n, b, 20261015, dtype=np.float32)).cuda()
    kw = dict(dtype=torch.float32, device="cuda")
    q, al, be = torch.zeros(m * b, **kw), torch.zeros(m, b, b, **kw), torch.zeros(m + 1, b, b, **kw)
    P = [torch.zeros(n, b, **kw) for _ in range(3)]
    base = dict(os.environ)
    res = {c: {"it": [], "spmm": [], "el": [], "ub": []} for c in args.cfgs}
    ref = None
    for rnd in range(args.rounds):
        for c in args.cfgs:
            os.environ.clear()
            os.environ.update(base)
            for kv in c.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            h.set_final_state(os.environ.get("AB_FS", "1") == "1")  # AB_FS=0: no post-call state pass
            h.block_lanczos_blas(Ad, B, 2, 84, q, al, be, *P)
            torch.cuda.synchronize()
            h.prof_enable(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.block_lanczos_blas(Ad, B, m, 84, q, al, be, *P)
            e1.record()
            torch.cuda.synchronize()
            sp, cnt = h.prof_read(h.PROF_SPMM)
            el, cel = h.prof_read(h.PROF_SPMM_PASS)  # pass EL (beta^2 form) / pass E
            ub, cub = h.prof_read(h.PROF_UPDATE_PASS)  # pass UB / pass U
            h.prof_enable(False)
            a = al.cpu().numpy()
            if ref is None:
                ref = a
            d = float(np.max(np.abs(a[:4] - ref[:4])) / np.max(np.abs(ref[:4])))
            if not d < 1e-4 and "AB_NOCHECK" not in c:  # (AB_NOCHECK=1: a diagnostic setting, results wrong)
                raise RuntimeError(f"alpha differs under {c}: {d}")
            res[c]["it"].append(e0.elapsed_time(e1) / m)
            res[c]["spmm"].append(sp / max(cnt, 1))
            res[c]["el"].append(el / max(cel, 1))
            res[c]["ub"].append(ub / max(cub, 1))
            print(f"round {rnd} [{c}] step {res[c]['it'][-1]:.4f} ms  spmm {res[c]['spmm'][-1]:.4f} ms  "
                  f"el {res[c]['el'][-1]:.4f} ms  ub {res[c]['ub'][-1]:.4f} ms  d {d:.1e}", flush=True)
    print(json.dumps({c: {k: round(float(np.median(v)), 4) for k, v in r.items()} for c, r in res.items()}, indent=1))


if __name__ == "__main__":
    main()
