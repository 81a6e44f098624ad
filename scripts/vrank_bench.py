"""The N-rank distributed iteration at bench scale on ONE GPU (virtual ranks).

    python scripts/vrank_bench.py --ranks 4 [--config c3|c4] [--exchange halo|allgather|both]
                                  [--steps 10] [--warmup 2] [--overlap 1|0|both] [--out FILE]

Each virtual rank (lz_local_group_create / lz_comm_init_local: one host thread,
one stream, one lz handle) owns the row slab bench.py's rank would own at N
GPUs -- C3 weak scaling: 10M rows per rank of an N*10M-row banded operator;
C4: 40M rows in total, 25 nnz/row, half width 2^16 -- and runs the same entry
points (lz_halo_init + lz_block_lanczos_halo, or lz_block_lanczos_dist with the
in-place all-gather), the collectives done by device copies.  The first
--parity-steps steps are checked against the CPU oracle on the GLOBAL operator
(alpha, beta, the row probe, Ritz values), as bench.py does at N > 1.

The ranks share one GPU, so a step takes about N times a single rank's step:
the times here show that the N-rank code runs at scale and what the
interior/boundary split does on one device, not multi-GPU scaling (that is
bench.py's run over RCCL at N GPUs).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
from bench import RITZ_TOL, compare_run, log  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--config", choices=["c3", "c4"], default="c3")
    ap.add_argument("--exchange", choices=["halo", "allgather", "both"], default="both")
    ap.add_argument("--overlap", choices=["1", "0", "both"], default="1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--parity-steps", type=int, default=3)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    lz = ge.load_package()
    orc = ge.load_oracle()
    N, b, seed, lc = args.ranks, 16, 20261015, 84
    c4 = args.config == "c4"
    if c4:
        n_total = args.n or 40_000_000
        npr, hw = 25.0, 1 << 16
        bounds = np.array([n_total * g // N for g in range(N + 1)], np.int64)
    else:
        n_rank = args.n or 10_000_000
        n_total, npr, hw = n_rank * N, 10.0, 4096
        bounds = np.array([n_rank * g for g in range(N + 1)], np.int64)
    t0 = time.time()
    A = lz.gen_banded(n_total, npr, hw, seed)
    B = lz.uniform_B(n_total, b, seed)
    log(f"global operator n={n_total} nnz={A.nnz} in {time.time() - t0:.1f}s")
    K, W = args.steps, args.warmup
    m_chk = min(K, args.parity_steps)
    t0 = time.time()
    qo, ao, bo = orc.block_lanczos(A, B, m_chk, lc)
    log(f"oracle {m_chk} steps in {time.time() - t0:.1f}s")
    n_pad = int(np.max(np.diff(bounds)))
    results = []
    forms = ["halo", "allgather"] if args.exchange == "both" else [args.exchange]
    overlaps = ["1", "0"] if args.overlap == "both" else [args.overlap]
    for form in forms:
        for ov in overlaps:
            os.environ["LZ_DIST_OVERLAP"] = ov
            bar = threading.Barrier(N)

            def rank_fn(r, h):
                kw = dict(dtype=torch.float64, device="cuda")
                r0, r1 = int(bounds[r]), int(bounds[r + 1])
                nl = r1 - r0
                k0, k1 = int(A.row_ptr[r0]), int(A.row_ptr[r1])
                rp = (A.row_ptr[r0:r1 + 1] - A.row_ptr[r0]).astype(np.int64)
                col, val = A.col[k0:k1], A.val[k0:k1]
                m_max = max(K, W, 1)
                q = torch.zeros(m_max * b, **kw)
                al = torch.zeros(m_max, b, b, **kw)
                be = torch.zeros(m_max + 1, b, b, **kw)
                Bl = torch.from_numpy(np.ascontiguousarray(B[r0:r1])).cuda()
                if form == "halo":
                    ccol, cnt, rows = lz.halo_plan(col, bounds, r)
                    h.halo_init(r0, nl, cnt, rows)
                    nh = int(rows.size)
                    Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, ccol, val), n_cols=nl + nh)
                    X0, X1 = (torch.zeros(nl + nh, b, **kw) for _ in range(2))

                    def run(m):
                        h.block_lanczos_halo(Ad, Bl, m, lc, 0, q, al, be, X0, X1)
                else:
                    nh = 0
                    pcol = lz.remap_cols_padded(col, bounds, n_pad)
                    Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, pcol, val), n_cols=n_pad * N)
                    Bp = torch.zeros(n_pad, b, **kw)
                    Bp[:nl] = Bl
                    Wl = torch.zeros(n_pad, b, **kw)
                    X = torch.zeros(n_pad * N, b, **kw)

                    def run(m):
                        h.block_lanczos_dist(Ad, n_pad, n_pad * N, Bp, m, lc, 0, q, al, be, None, Wl, X)
                run(W)
                torch.cuda.current_stream().synchronize()
                bar.wait()
                t = time.perf_counter()
                run(K)
                torch.cuda.current_stream().synchronize()
                el = time.perf_counter() - t
                bar.wait()
                assert h.device_error() == 0
                return (el, al.cpu().numpy()[:K], be.cpu().numpy()[: K + 1], q.cpu().numpy()[: K * b], nh,
                        h.last_split())

            res = lz.run_virtual_ranks(N, rank_fn)
            el = max(x[0] for x in res)
            for r in range(1, N):
                assert np.array_equal(res[r][1], res[0][1]), "ranks disagree on alpha"
            par = compare_run(lz, m_chk, b, (res[0][1], res[0][2], res[0][3]), (ao, bo, qo), 1e-9, RITZ_TOL)
            ent = {"exchange": form, "overlap": ov == "1", "ms_per_step_all_ranks": round(el / K * 1e3, 3),
                   "ms_per_step_per_rank_equiv": round(el / K * 1e3 / N, 3),
                   "halo_rows": [int(x[4]) for x in res], "split": [x[5] for x in res], "parity": par}
            log(json.dumps(ent))
            if not par["ok"]:
                raise SystemExit(f"parity failed: {ent}")
            results.append(ent)
    out = {"what": "virtual ranks on ONE GPU: the N-rank distributed iteration at bench scale, checked against the "
                   "oracle on the global operator; times are of N ranks sharing one device (not scaling)",
           "config": args.config.upper(), "ranks": N, "n_total": n_total, "nnz": int(A.nnz), "b": b,
           "steps": K, "warmup": W, "results": results}
    s = json.dumps(out)
    print(s)
    if args.out:
        open(args.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
