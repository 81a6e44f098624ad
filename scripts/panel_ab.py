"""The column-panel SpMM candidate (csrc/lz_panel.hip, round 5) against the
nnz-split gather kernel (k_spmm_seg, lz_csr_spmm) at C3 (n = 1e7, 10 nnz/row,
half width 4096, b = 16 fp64), alternating in one process; Y of both checked
against each other (64 eps bound).  Prints the plan's size and build time and
both kernels' ms per launch and HBM fraction on the SpMM's algorithmic bytes
(z*12 + (n+1)*8 + 2nbs).

The candidate lost (5.16 vs 1.19 ms, DESIGN.md 4 SpMM) and lives only in the
diagnostic build: run `make -C gpu-implementation-of-signle-and-block-lanczos_amd diag`
first; this script loads lib/liblz_hip_diag.so (include/lz_diag.h).
`--check` runs the round-5 parity cases (small operators against a dense
numpy product) instead of the timing.

  python scripts/panel_ab.py [--rounds 5] [--reps 20] [--n 10000000] [--check]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG_LIB = os.path.join(ROOT, "gpu-implementation-of-signle-and-block-lanczos_amd", "lib", "liblz_hip_diag.so")
os.environ.setdefault("LZ_HIP_LIB", DIAG_LIB)
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

PANEL_ROWS, PANEL_WIDTH, PANEL_MAX_ENTRIES, PANEL_GOFF = 2048, 512, 1536, 136


@dataclass
class PanelPlan:
    """The column-panel SpMM's once-per-operator plan (lz_debug_spmm_panel in the diag
    build, host arrays): passes = (row block, 512-row X panel, up to 1536 entries)."""
    n: int
    nblocks: int
    bp0: np.ndarray    # int32 [nblocks + 1]
    px0: np.ndarray    # int32 [npass]
    pe0: np.ndarray    # int32 [npass + 1]
    goff: np.ndarray   # uint16 [npass * 136]
    ev: np.ndarray     # float64 [pe0[-1]]
    ex: np.ndarray     # uint16 [pe0[-1]]

    def device(self, device="cuda"):
        return {k: torch.from_numpy(getattr(self, k)).to(device) for k in ("bp0", "px0", "pe0", "goff", "ev", "ex")}


def panel_plan(A) -> PanelPlan:
    """For every block of 2048 rows, its entries regrouped by the 512-row X panel
    their column falls in (panels from the block's smallest column), CSR order
    kept inside a panel (so by row, then column), a panel of more than 1536
    entries split over several passes, each pass padded to 8 entries; entry
    word = (row % 16) << 9 | (column - panel start); group offsets = where each
    16-row group's entries start in the pass."""
    R, W, E, GO = PANEL_ROWS, PANEL_WIDTH, PANEL_MAX_ENTRIES, PANEL_GOFF
    n, rp, col = A.n, A.row_ptr.astype(np.int64), A.col
    nb = (n + R - 1) // R
    cnt = np.diff(rp)
    rows = np.repeat(np.arange(n, dtype=np.int64), cnt)
    blk = rows // R
    starts = rp[np.minimum(np.arange(nb, dtype=np.int64) * R, n)]
    has = np.diff(np.append(starts, rp[n])) > 0
    base = np.zeros(nb, np.int64)
    if has.any():  # (an empty block contributes no entries, so each segment ends at the next one's start)
        base[has] = np.minimum.reduceat(col, starts[has])
    rel = col.astype(np.int64) - base[blk]
    p = rel // W
    maxp = int(p.max()) + 1 if p.size else 1
    key = blk * maxp + p
    order = np.argsort(key, kind="stable")
    key_s = key[order]
    # segments (block, panel) and their split into passes of <= E entries
    seg_start = np.flatnonzero(np.r_[True, key_s[1:] != key_s[:-1]]) if key_s.size else np.zeros(0, np.int64)
    seg_len = np.diff(np.r_[seg_start, key_s.size])
    seg_pass = (seg_len + E - 1) // E
    pass_base = np.r_[0, np.cumsum(seg_pass)[:-1]]
    npass = int(seg_pass.sum())
    seg_of = np.repeat(np.arange(seg_start.size), seg_len)
    idx_in_seg = np.arange(key_s.size) - seg_start[seg_of]
    pid = pass_base[seg_of] + idx_in_seg // E
    pass_cnt = np.bincount(pid, minlength=npass)
    pad = (pass_cnt + 7) // 8 * 8
    pe0 = np.r_[0, np.cumsum(pad)].astype(np.int64)
    pass_first = np.r_[0, np.cumsum(pass_cnt)[:-1]]
    dest = pe0[pid] + (np.arange(key_s.size) - pass_first[pid])
    rows_s = rows[order]
    ev = np.zeros(int(pe0[-1]), np.float64)
    ex = np.zeros(int(pe0[-1]), np.uint16)
    ev[dest] = A.val[order]
    ex[dest] = (((rows_s % 16) << 9) | (rel[order] % W)).astype(np.uint16)
    g = (rows_s % R) // 16
    gc = np.bincount(pid * 128 + g, minlength=npass * 128).reshape(npass, 128) if npass else \
        np.zeros((0, 128), np.int64)
    goff = np.zeros((npass, GO), np.uint16)
    goff[:, 1:129] = np.cumsum(gc, axis=1)
    seg_blk = key_s[seg_start] // maxp
    seg_p = key_s[seg_start] % maxp
    pass_seg = np.repeat(np.arange(seg_start.size), seg_pass)
    px0 = (base[seg_blk[pass_seg]] + seg_p[pass_seg] * W).astype(np.int32)
    pass_blk = seg_blk[pass_seg]
    bp0 = np.searchsorted(pass_blk, np.arange(nb + 1)).astype(np.int32)
    if pe0[-1] >= 2 ** 31:
        raise RuntimeError("panel plan: more than 2^31 entries")
    return PanelPlan(n, nb, bp0, px0, pe0.astype(np.int32), goff.reshape(-1), ev, ex)




def spmm_panel(h, plan_dev, n, nblocks, X, Y):
    """Y = A X by lz_debug_spmm_panel (diag build) from a PanelPlan's device arrays."""
    L = h.L
    fn = L.lz_debug_spmm_panel
    vp = ctypes.c_void_p
    fn.restype = ctypes.c_int
    fn.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp]
    d = plan_dev
    rc = fn(h.ptr, n, X.shape[0], X.data_ptr(), Y.data_ptr(), nblocks, *(d[k].data_ptr() for k in
                                                                        ("bp0", "px0", "pe0", "goff", "ev", "ex")))
    if rc:
        raise RuntimeError(f"lz_debug_spmm_panel: {rc} {L.lz_last_error()}")
    return Y


def check(lz, h):
    """Round-5 parity cases: n not a multiple of the 2048-row block, panels split
    over several passes (30 entries per row), a band wider and narrower than the
    panel, a single short block; 64 eps bound against the dense product."""
    for n, npr, hw in ((50_021, 10.0, 4096), (20_480, 10.0, 256), (9_000, 30.0, 2000), (4_099, 5.0, 3000),
                       (300, 8.0, 100)):
        A = lz.gen_banded(n, npr, hw, seed=n % 97)
        pl = panel_plan(A)
        assert pl.pe0[-1] >= A.nnz and (np.diff(pl.pe0) <= PANEL_MAX_ENTRIES).all()
        X = np.random.default_rng(5).uniform(-1, 1, (n, 16))
        Y = torch.full((n, 16), float("nan"), dtype=torch.float64, device="cuda")
        spmm_panel(h, pl.device(), n, pl.nblocks, torch.from_numpy(X).cuda(), Y)
        torch.cuda.synchronize()
        M = np.zeros((n, n))
        rows = np.repeat(np.arange(n), np.diff(A.row_ptr))
        np.add.at(M, (rows, A.col), A.val)
        ref, bound = M @ X, np.abs(M) @ np.abs(X)
        err = np.abs(Y.cpu().numpy() - ref)
        ok = bool(np.all(err <= 64 * np.finfo(np.float64).eps * bound + 1e-300))
        print(json.dumps({"n": n, "nnz_per_row": npr, "halfwidth": hw, "max_err": float(err.max()), "ok": ok}))
        if not ok:
            raise SystemExit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--halfwidth", type=int, default=4096)
    ap.add_argument("--which", default="both", choices=["both", "panel", "seg"])
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    lz = ge.load_package()
    if args.check:
        check(lz, lz.Handle(0))
        return
    n, b = args.n, 16
    A = lz.gen_banded(n, 10.0, args.halfwidth, 20261015)
    t0 = time.time()
    pl = panel_plan(A)
    t_plan = time.time() - t0
    npass = int(pl.px0.size)
    h = lz.Handle(0)
    Ad = lz.CsrDevice.from_host(A)
    pd = pl.device()
    X = torch.from_numpy(lz.uniform_B(n, b, 20261015)).cuda()
    Y1 = torch.empty(n, b, dtype=torch.float64, device="cuda")
    Y2 = torch.empty_like(Y1)
    h.spmm(Ad, X, Y1)
    spmm_panel(h, pd, n, pl.nblocks, X, Y2)
    torch.cuda.synchronize()
    d = float((Y1 - Y2).abs().max().item())
    scale = float(Y1.abs().max().item())
    alg = A.nnz * 12 + (n + 1) * 8 + 2 * n * b * 8
    stream = pl.ev.nbytes + pl.ex.nbytes + pl.goff.nbytes + pl.pe0.nbytes + pl.px0.nbytes
    res = {"seg": [], "panel": []}
    for rnd in range(args.rounds):
        for k in ("seg", "panel"):
            if args.which not in ("both", k):
                continue
            fn = (lambda: h.spmm(Ad, X, Y1)) if k == "seg" else (lambda: spmm_panel(h, pd, n, pl.nblocks, X, Y2))
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / args.reps)
        print(f"round {rnd}: " + "  ".join(f"{k} {v[-1]:.4f} ms" for k, v in res.items() if v), flush=True)
    out = {"n": n, "nnz": int(A.nnz), "halfwidth": args.halfwidth, "plan_s": round(t_plan, 1), "passes": npass,
           "plan_entries_padded": int(pl.pe0[-1]), "plan_stream_bytes": int(stream),
           "max_abs_diff_vs_seg": d, "rel": d / scale, "alg_bytes": alg}
    for k, v in res.items():
        if v:
            ms = float(np.median(v))
            out[k] = {"ms": round(ms, 4), "GBs": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / 8000, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
