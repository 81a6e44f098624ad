"""N-rank decompositions driven natively from ONE GPU (virtual ranks).

Each virtual rank is a host thread with its own stream and its own lz handle,
attached to an in-process group (lz_local_group_create / lz_comm_init_local):
the ranks run exactly the entry points an RCCL rank runs -- lz_halo_init's
count and request exchanges, lz_block_lanczos_halo (owner-side packing, the
point-to-point round into the halo runs, the compact-column fused pass) and
lz_block_lanczos_dist (the in-place all-gather, pass 2's SWAP form, the padded
numbering, the windowed pass 1 past 2^24 gathered rows) -- with the
collectives moved by device copies instead of RCCL.  Every run is compared
with the single-process CPU oracle on the global operator
(methods/block_lanczos.hpp:104-166 op order), and every rank's alpha/beta must
be bit-identical.

Covered: nnz-balanced uneven slabs (lzh_partition_rows), lc owned by a rank
other than 0, halos reaching past the neighbours, a power-law operator, the
interior/boundary split (pass 1 of the interior rows beside the exchange) on
and off, b in {1, 4, 16} fp64 and b = 32 fp32, and a gathered block of
2^24+ rows.
"""
import os

import numpy as np
import pytest

from test_gpu_lanczos import assert_close_run

pytestmark = pytest.mark.gpu


def _slab(A, r0, r1):
    rp = A.row_ptr[r0:r1 + 1] - A.row_ptr[r0]
    k0, k1 = int(A.row_ptr[r0]), int(A.row_ptr[r1])
    return rp.astype(np.int64), A.col[k0:k1].copy(), A.val[k0:k1].copy()


def _owner(bounds, row):
    return int(np.searchsorted(bounds, row, side="right") - 1)


def run_dist(lz, torch, A, B, m, lc, nranks, form, overlap=True, bounds=None, wf_out=None):
    """Run the distributed block Lanczos over `nranks` virtual ranks; returns
    (q, alpha, beta) of lc's owner and every rank's split (interior rows) or
    None; wf_out (a list) receives every rank's (wavefront step, pass-2-first
    overlap) flags."""
    n, b = B.shape
    if bounds is None:
        bounds = lz.partition_rows(A, nranks)
    bounds = np.asarray(bounds, np.int64)
    lc_rank = _owner(bounds, lc)
    n_pad = int(np.max(np.diff(bounds)))
    dt = torch.float64 if B.dtype == np.float64 else torch.float32
    val_dt = B.dtype
    old = os.environ.get("LZ_DIST_OVERLAP")
    os.environ["LZ_DIST_OVERLAP"] = "1" if overlap else "0"

    def rank_fn(r, h):
        kw = dict(dtype=dt, device="cuda")
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        nl = r1 - r0
        rp, col, val = _slab(A, r0, r1)
        val = val.astype(val_dt)
        q = torch.zeros(m * b, **kw)
        al = torch.zeros(m, b, b, **kw)
        be = torch.zeros(m + 1, b, b, **kw)
        Bl = torch.from_numpy(np.ascontiguousarray(B[r0:r1])).cuda()
        if form == "halo":
            ccol, cnt, rows = lz.halo_plan(col, bounds, r)
            h.halo_init(r0, nl, cnt, rows)
            nh = int(rows.size)
            assert h.halo_sizes()[0] == nh
            Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, ccol, val), n_cols=nl + nh)
            X0 = torch.zeros(nl + nh, b, **kw)
            X1 = torch.zeros(nl + nh, b, **kw)
            h.block_lanczos_halo(Ad, Bl, m, lc - bounds[lc_rank], lc_rank, q, al, be, X0, X1)
        else:
            pcol = lz.remap_cols_padded(col, bounds, n_pad)
            Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, pcol, val), n_cols=n_pad * nranks)
            Bp = torch.zeros(n_pad, b, **kw)
            Bp[:nl] = Bl
            W = torch.zeros(n_pad, b, **kw)
            X = torch.zeros(n_pad * nranks, b, **kw)
            h.block_lanczos_dist(Ad, n_pad, n_pad * nranks, Bp, m, lc - bounds[lc_rank], lc_rank, q, al, be,
                                 None, W, X)
        assert h.device_error() == 0
        return q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy(), h.last_split(), h.last_wf()

    try:
        res = lz.run_virtual_ranks(nranks, rank_fn)
    finally:
        if old is None:
            os.environ.pop("LZ_DIST_OVERLAP", None)
        else:
            os.environ["LZ_DIST_OVERLAP"] = old
    for r in range(1, nranks):  # every rank holds the same alpha / beta bits
        assert np.array_equal(res[r][1], res[0][1]) and np.array_equal(res[r][2][:m], res[0][2][:m]), r
    q, al, be = res[lc_rank][:3]
    if wf_out is not None:
        wf_out.extend(x[4] for x in res)
    return (q, al, be), [x[3] for x in res]


@pytest.mark.parametrize("form", ["halo", "allgather"])
@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_vranks_b16_banded(lz, orc, torch_cuda, form, nranks):
    """Banded operator, nnz-balanced slabs, lc on a rank other than 0; the
    interior rows' pass 1 runs beside the exchange (split must be on).  The
    halo form runs the wavefront step with the requested rows' pass 2 first and
    the exchange beside the rest of the step (asserted); the all-gather form
    the two-pass step (its default at N > 1)."""
    A = lz.gen_banded(120_011, 10.0, 1500, seed=100 + nranks)
    B = lz.uniform_B(A.n, 16, seed=7)
    m, lc = 7, 120_011 * 5 // 8 + 3
    wfs = []
    got, splits = run_dist(lz, torch_cuda, A, B, m, lc, nranks, form, wf_out=wfs)
    assert all(s is not None for s in splits), splits  # every rank split its rows
    assert all(w == ((True, True) if form == "halo" else (False, False)) for w in wfs), wfs
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
def test_vranks_b16_allgather_wavefront(lz, orc, torch_cuda, monkeypatch, nranks):
    """The all-gather form on the wavefront step (LZ_AG_WF=1; the default at
    one rank): pass 2 writes V_{j+1} into the rank's slot of X_full and V_j into
    W, the in-place all-gather fills the peers' slots, then the boundary tiles."""
    monkeypatch.setenv("LZ_AG_WF", "1")
    A = lz.gen_banded(120_011, 10.0, 1500, seed=110 + nranks)
    B = lz.uniform_B(A.n, 16, seed=8)
    m, lc = 7, 120_011 // 3 + 5
    wfs = []
    got, splits = run_dist(lz, torch_cuda, A, B, m, lc, nranks, "allgather", wf_out=wfs)
    assert all(w[0] for w in wfs), wfs
    if nranks > 1:
        assert all(s is not None for s in splits), splits
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("wf", ["0", "1"])
@pytest.mark.parametrize("nranks", [1, 3, 4])
def test_vranks_b16_halo_step_forms(lz, orc, torch_cuda, monkeypatch, wf, nranks):
    """The halo form's two step forms: the wavefront step per rank (pass 2 +
    interior pass 1 in one launch, then the exchange and the boundary tiles;
    the default) and the two-pass step (LZ_PASS_WF=0), with the split on and
    off (at 4 ranks the half width exceeds a rank's rows: no interior tiles)."""
    monkeypatch.setenv("LZ_PASS_WF", wf)
    hw = 30_000 if nranks == 4 else 2048
    A = lz.gen_banded(100_003, 10.0, hw, seed=40 + nranks)
    B = lz.uniform_B(A.n, 16, seed=3)
    m, lc = 8, 77_777
    got, _ = run_dist(lz, torch_cuda, A, B, m, lc, nranks, "halo")
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("nranks", [2, 4])
def test_vranks_b16_halo_wide_rows(lz, orc, torch_cuda, nranks):
    """Config C4's density (25 entries per row) on the halo form: each rank runs
    the wavefront step's wide shape (two 4400-entry stages)."""
    A = lz.gen_banded(120_011, 25.0, 6000, seed=50 + nranks)
    B = lz.uniform_B(A.n, 16, seed=6)
    m, lc = 7, 1_234
    got, _ = run_dist(lz, torch_cuda, A, B, m, lc, nranks, "halo")
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("form", ["halo", "allgather"])
def test_vranks_b16_overlap_off_equals_on(lz, orc, torch_cuda, form):
    """LZ_DIST_OVERLAP=0 (exchange, then the whole pass) against the split run:
    both match the oracle; the halos reach past the neighbouring ranks."""
    A = lz.gen_banded(48_007, 10.0, 9000, seed=11)  # half width > rows per rank at 8 ranks
    B = lz.uniform_B(A.n, 16, seed=12)
    m, lc = 6, 47_000
    ref = orc.block_lanczos(A, B, m, lc)
    for ov in (False, True):
        got, splits = run_dist(lz, torch_cuda, A, B, m, lc, 8, form, overlap=ov)
        if not ov:
            assert all(s is None for s in splits)
        assert_close_run(lz, m, 16, got, ref)


@pytest.mark.parametrize("form", ["halo", "allgather"])
def test_vranks_b16_powerlaw(lz, orc, torch_cuda, form):
    """Power-law rows (config C5's generator, fp64): rows everywhere reach other
    ranks, so the split is off on most ranks and the halo is most of the block."""
    A = lz.gen_powerlaw(40_009, 10.0, 2.1, 5000, seed=13, dtype=np.float64)
    B = lz.uniform_B(A.n, 16, seed=14)
    m, lc = 5, 123
    got, _ = run_dist(lz, torch_cuda, A, B, m, lc, 4, form)
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("form", ["halo", "allgather"])
@pytest.mark.parametrize("b", [1, 4])
@pytest.mark.parametrize("nranks", [2, 4])
def test_vranks_generic_b(lz, orc, torch_cuda, form, b, nranks):
    """b = 1 (the single-vector recurrence, methods/vector_lanczos.hpp:8-67) and
    the reference driver's N_COL = 4 (test_lanczos.cu:5), fp64."""
    A = lz.gen_banded(30_011, 10.0, 800, seed=20 + b)
    B = lz.uniform_B(A.n, b, seed=21)
    m, lc = 8, 30_011 - 5
    got, splits = run_dist(lz, torch_cuda, A, B, m, lc, nranks, form)
    assert all(s is not None for s in splits)
    assert_close_run(lz, m, b, got, orc.block_lanczos(A, B, m, lc))
    if b == 1:  # the same numbers as the single-vector oracle
        qv, av, bv = orc.vector_lanczos(A, B[:, 0], m, lc)
        assert np.allclose(got[1].ravel(), av, rtol=1e-9, atol=1e-12)
        assert np.allclose(got[2].ravel()[:m], bv, rtol=1e-9, atol=1e-12)
        assert np.allclose(got[0], qv, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("form", ["halo", "allgather"])
def test_vranks_b32_f32(lz, orc, torch_cuda, form):
    """b = 32 fp32 (config C5's shape) at 2 ranks: MFMA pass E, VALU pass U / SWAP."""
    A = lz.gen_banded(20_011, 10.0, 600, seed=30, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=31, dtype=np.float32)
    m, lc = 5, 15_000
    got, _ = run_dist(lz, torch_cuda, A, B, m, lc, 2, form)
    qo, ao, bo = orc.block_lanczos(A, B, m, lc)
    q, al, be = got
    scale = max(1.0, float(np.abs(ao).max()), float(np.abs(bo[:m]).max()))
    assert np.max(np.abs(al - ao)) <= 1e-4 * scale
    assert np.max(np.abs(be[:m] - bo[:m])) <= 1e-4 * scale
    assert np.allclose(q, qo, rtol=1e-4, atol=1e-4 * np.abs(qo).max())


@pytest.mark.parametrize("wf", ["0", "1"])
def test_vranks_allgather_wide_window(lz, orc, torch_cuda, monkeypatch, wf):
    """8 ranks whose gathered block has 8 * n_pad >= 2^24 rows (2.2 GB at b = 16
    fp64): pass 1 gathers through its 2^24-row window, interior split on; in
    the two-pass step and (LZ_AG_WF=1) in the wavefront step."""
    monkeypatch.setenv("LZ_AG_WF", wf)
    n = 8 * ((1 << 21) + 1000)
    A = lz.gen_banded(n, 3.0, 200, seed=41)
    B = lz.uniform_B(A.n, 16, seed=42)
    m, lc = 3, n - 77
    wfs = []
    got, splits = run_dist(lz, torch_cuda, A, B, m, lc, 8, "allgather", wf_out=wfs)
    assert all(s is not None for s in splits)
    assert all(w[0] == (wf == "1") for w in wfs), wfs
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("b,dtype", [(4, np.float32), (16, np.float64), (3, np.float64)])
def test_vranks_halo_exchange_rows(lz, torch_cuda, b, dtype):
    """lz_halo_exchange alone at 3 ranks: every halo row equals its owner's row."""
    torch = torch_cuda
    A = lz.gen_banded(9_001, 6.0, 2000, seed=50)
    bounds = np.array([0, 2000, 6500, 9001], np.int64)
    G = np.arange(A.n * b, dtype=dtype).reshape(A.n, b) / 7.0
    tdt = torch.float32 if dtype == np.float32 else torch.float64

    def rank_fn(r, h):
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        _, col, _ = _slab(A, r0, r1)
        _, cnt, rows = lz.halo_plan(col, bounds, r)
        h.halo_init(r0, r1 - r0, cnt, rows)
        X = torch.zeros(r1 - r0 + rows.size, b, dtype=tdt, device="cuda")
        X[: r1 - r0] = torch.from_numpy(G[r0:r1]).cuda()
        h.halo_exchange(X)
        return X.cpu().numpy(), rows

    for r, (X, rows) in enumerate(lz.run_virtual_ranks(3, rank_fn)):
        nl = int(bounds[r + 1] - bounds[r])
        assert np.array_equal(X[nl:], G[rows.astype(np.int64)]), r


def test_vranks_failing_rank_aborts_group(lz, torch_cuda):
    """A rank that fails before a collective aborts the group: the others
    return an error (LZ_E_COMM) instead of waiting at the barrier."""
    import time
    A = lz.gen_banded(4_000, 5.0, 100, seed=60)
    bounds = np.array([0, 2000, 4000], np.int64)

    def rank_fn(r, h):
        if r == 1:
            raise RuntimeError("rank 1 fails on purpose")
        _, col, _ = _slab(A, 0, 2000)
        _, cnt, rows = lz.halo_plan(col, bounds, 0)
        h.halo_init(0, 2000, cnt, rows)  # collective: rank 1 never arrives

    t0 = time.time()
    with pytest.raises(lz.LanczosError):
        lz.run_virtual_ranks(2, rank_fn)
    assert time.time() - t0 < 60


def test_vranks_argument_error_aborts_group(lz, torch_cuda):
    """A rank whose distributed call fails its argument checks aborts the group
    inside the library (no Python-side abort involved): the rank waiting in the
    first collective returns LZ_E_COMM at once instead of at the barrier timeout."""
    import ctypes
    import time
    torch = torch_cuda
    A = lz.gen_banded(4_000, 5.0, 100, seed=61)
    bounds = np.array([0, 2000, 4000], np.int64)
    codes = [None, None]

    def rank_fn(r, h):
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        rp, col, val = _slab(A, r0, r1)
        ccol, cnt, rows = lz.halo_plan(col, bounds, r)
        h.halo_init(r0, r1 - r0, cnt, rows)
        nh = int(rows.size)
        Ad = lz.CsrDevice.from_host(lz.CsrHost(r1 - r0, rp, ccol, val), n_cols=r1 - r0 + nh)
        kw = dict(dtype=torch.float64, device="cuda")
        q, al, be = torch.zeros(4 * 16, **kw), torch.zeros(4, 16, 16, **kw), torch.zeros(5, 16, 16, **kw)
        X0, X1 = torch.zeros(r1 - r0 + nh, 16, **kw), torch.zeros(r1 - r0 + nh, 16, **kw)
        Bl = torch.ones(r1 - r0, 16, **kw)
        m = 0 if r == 1 else 4  # rank 1: m = 0 fails the argument check
        codes[r] = h.L.lz_block_lanczos_halo(h.ptr, r1 - r0, Ad.nnz, Ad.row_ptr.data_ptr(), Ad.col.data_ptr(),
                                              Ad.val.data_ptr(), lz.LZ_F64, 16, m, 0, 0, Bl.data_ptr(),
                                              q.data_ptr(), al.data_ptr(), be.data_ptr(), X0.data_ptr(),
                                              X1.data_ptr())

    t0 = time.time()
    lz.run_virtual_ranks(2, rank_fn)
    assert time.time() - t0 < 60
    assert codes[1] == -1 and codes[0] == -3, codes  # LZ_E_ARG on rank 1, LZ_E_COMM on rank 0


@pytest.mark.parametrize("form,b", [("halo", 16), ("allgather", 16), ("halo", 4)])
def test_vranks_setup_failure_votes(lz, torch_cuda, form, b):
    """A rank whose set-up fails inside the distributed solve (forced by
    lz_debug_fail_next_setup: as a failed workspace growth or plan) still joins
    the solve's first collective, the ranks' set-up vote, with ok = 0: its peer
    returns LZ_E_STATE naming the peer's failure, not the group's abort (over
    RCCL no abort is issued before a collective, so without the vote the peer
    would wait in a collective this rank never issues)."""
    import time
    torch = torch_cuda
    A = lz.gen_banded(4_000, 5.0, 100, seed=63)
    bounds = np.array([0, 2000, 4000], np.int64)
    out = [None, None]

    def rank_fn(r, h):
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        nl = r1 - r0
        rp, col, val = _slab(A, r0, r1)
        kw = dict(dtype=torch.float64, device="cuda")
        q, al, be = torch.zeros(4 * b, **kw), torch.zeros(4, b, b, **kw), torch.zeros(5, b, b, **kw)
        Bl = torch.ones(nl, b, **kw)
        if form == "halo":
            ccol, cnt, rows = lz.halo_plan(col, bounds, r)
            h.halo_init(r0, nl, cnt, rows)
            nh = int(rows.size)
            Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, ccol, val), n_cols=nl + nh)
            X0, X1 = torch.zeros(nl + nh, b, **kw), torch.zeros(nl + nh, b, **kw)
            args = (h.ptr, nl, Ad.nnz, Ad.row_ptr.data_ptr(), Ad.col.data_ptr(), Ad.val.data_ptr(), lz.LZ_F64, b, 4,
                    0, 0, Bl.data_ptr(), q.data_ptr(), al.data_ptr(), be.data_ptr(), X0.data_ptr(), X1.data_ptr())
            fn = h.L.lz_block_lanczos_halo
        else:
            n_pad = 2000
            pcol = lz.remap_cols_padded(col, bounds, n_pad)
            Ad = lz.CsrDevice.from_host(lz.CsrHost(nl, rp, pcol, val), n_cols=2 * n_pad)
            W, X = torch.zeros(n_pad, b, **kw), torch.zeros(2 * n_pad, b, **kw)
            args = (h.ptr, nl, n_pad, 2 * n_pad, Ad.nnz, Ad.row_ptr.data_ptr(), Ad.col.data_ptr(), Ad.val.data_ptr(),
                    lz.LZ_F64, b, 4, 0, 0, Bl.data_ptr(), q.data_ptr(), al.data_ptr(), be.data_ptr(), None, None,
                    W.data_ptr(), X.data_ptr())
            fn = h.L.lz_block_lanczos_dist
        if r == 1:
            h.debug_fail_next_setup(-2)  # as a failed hipMalloc
        rc = fn(*args)
        out[r] = (rc, h.L.lz_last_error().decode())

    t0 = time.time()
    lz.run_virtual_ranks(2, rank_fn)
    assert time.time() - t0 < 60
    assert out[1][0] == -2 and "lz_debug_fail_next_setup" in out[1][1], out
    assert out[0][0] == -4 and "peer rank failed its set-up" in out[0][1], out


def _with_far_entries(lz, A, pairs, v=1e-3):
    """A plus the symmetric entries (r, c), (c, r) of `pairs`, value v."""
    import scipy.sparse as sp
    M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))
    r = np.array([p[0] for p in pairs] + [p[1] for p in pairs])
    c = np.array([p[1] for p in pairs] + [p[0] for p in pairs])
    M = (M + sp.csr_matrix((np.full(r.size, v), (r, c)), shape=(A.n, A.n))).tocsr()
    M.sort_indices()
    return lz.CsrHost(A.n, M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data.astype(np.float64))


@pytest.mark.parametrize("nranks", [2, 4])
def test_vranks_b16_far_head_rows(lz, orc, torch_cuda, nranks):
    """A banded operator plus a few rows well inside each rank's first half
    that reference distant rows of the previous rank: the interior starts
    hundreds of tiles into the rank (the wavefront step's region 0 runs pass 2
    from tile 0 but pass 1 from there), so its updaters must pace from the
    pass-1 start, or the interior launch's waits form a cycle (device error 6)."""
    n = 160_000
    A = lz.gen_banded(n, 10.0, 500, seed=90 + nranks)
    bounds = np.array([n * g // nranks for g in range(nranks + 1)], np.int64)
    pairs = []
    for g in range(1, nranks):
        r0, r1 = int(bounds[g]), int(bounds[g + 1])
        for k, frac in enumerate((0.30, 0.36, 0.41)):  # first half of the rank's rows
            pairs.append((r0 + int(frac * (r1 - r0)) + k, int(bounds[g - 1]) + 100 + 37 * k))
    A = _with_far_entries(lz, A, pairs)
    B = lz.uniform_B(A.n, 16, seed=91)
    m, lc = 6, n - 1000
    got, splits = run_dist(lz, torch_cuda, A, B, m, lc, nranks, "halo", bounds=bounds)
    for g in range(1, nranks):  # the far rows moved the interior start deep into the rank
        assert splits[g] is not None and splits[g][0] > 0.25 * (bounds[g + 1] - bounds[g]), splits
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def test_vranks_halo_exchange_back_to_back(lz, torch_cuda):
    """Two lz_halo_exchange calls in a row, the second at a larger b (its send
    buffer is reallocated): each fills every halo row with its owner's row of
    that call's block (no peer reads a repacked or freed send buffer)."""
    torch = torch_cuda
    A = lz.gen_banded(9_001, 6.0, 2000, seed=52)
    bounds = np.array([0, 3000, 6000, 9001], np.int64)
    Gs = {b: np.arange(A.n * b, dtype=np.float64).reshape(A.n, b) / (3.0 + b) for b in (4, 16)}

    def rank_fn(r, h):
        r0, r1 = int(bounds[r]), int(bounds[r + 1])
        _, col, _ = _slab(A, r0, r1)
        _, cnt, rows = lz.halo_plan(col, bounds, r)
        h.halo_init(r0, r1 - r0, cnt, rows)
        out = {}
        for b in (4, 16):
            X = torch.zeros(r1 - r0 + rows.size, b, dtype=torch.float64, device="cuda")
            X[: r1 - r0] = torch.from_numpy(Gs[b][r0:r1]).cuda()
            h.halo_exchange(X)
            X[: r1 - r0] = -1.0  # overwritten at once: a late peer copy would see it
            out[b] = X
        return {b: X.cpu().numpy() for b, X in out.items()}, rows

    for r, (Xs, rows) in enumerate(lz.run_virtual_ranks(3, rank_fn)):
        nl = int(bounds[r + 1] - bounds[r])
        for b, X in Xs.items():
            assert np.array_equal(X[nl:], Gs[b][rows.astype(np.int64)]), (r, b)


def test_vranks_barrier_timeout(lz, torch_cuda, monkeypatch):
    """LZ_LOCAL_TIMEOUT_S (read when the group is created): a rank that never
    reaches a collective makes the others' barrier give up after that many
    seconds with LZ_E_COMM (no abort involved: rank 1 simply returns)."""
    import time
    monkeypatch.setenv("LZ_LOCAL_TIMEOUT_S", "2")
    A = lz.gen_banded(4_000, 5.0, 100, seed=62)
    bounds = np.array([0, 2000, 4000], np.int64)

    def rank_fn(r, h):
        if r == 1:
            return None
        _, col, _ = _slab(A, 0, 2000)
        _, cnt, rows = lz.halo_plan(col, bounds, 0)
        h.halo_init(0, 2000, cnt, rows)  # collective: rank 1 never arrives

    t0 = time.time()
    with pytest.raises(lz.LanczosError, match="timeout"):
        lz.run_virtual_ranks(2, rank_fn)
    assert 1.5 < time.time() - t0 < 60


_C4 = {}


def _c4_problem(lz, orc):
    """BASELINE config C4 (n = 4e7, ~25 entries per row, half width 2^16) and
    the oracle's first 3 steps on it, built once for the module's C4 tests."""
    import time
    if not _C4:
        n, m, lc = 40_000_000, 3, 84
        t0 = time.time()
        A = lz.gen_banded(n, 25.0, 1 << 16, seed=20261015)
        B = lz.uniform_B(n, 16, seed=20261015)
        assert 0.99e9 < A.nnz < 1.01e9
        _C4.update(A=A, B=B, m=m, lc=lc, ref=orc.block_lanczos(A, B, m, lc), t_build=time.time() - t0)
    return _C4


@pytest.mark.timeout(900)
@pytest.mark.parametrize("form", ["halo", "allgather"])
def test_vranks_c4_full_size(lz, orc, torch_cuda, form):
    """BASELINE config C4 at full size: n = 4e7 rows, ~25 entries per row
    (nnz ~ 1e9), half width 2^16, row-partitioned over 8 virtual ranks, 3 steps
    against the oracle on the GLOBAL operator (methods/block_lanczos.hpp:131-166).
    halo: the wavefront step with the requested rows' pass 2 first and the
    exchange beside the rest of each step (asserted).  allgather: the north
    star's exchange -- every step all-gathers the whole Krylov block into each
    rank's X_full (5.1 GB per rank here) -- on the two-pass step, its default at
    N > 1 (asserted).  The 8 ranks share one device here; over RCCL each is one
    MI355X (bench.py --gpus 8 --config c4)."""
    import time
    P = _c4_problem(lz, orc)
    N, n = 8, P["A"].n
    bounds = np.array([n * g // N for g in range(N + 1)], np.int64)
    wfs = []
    t1 = time.time()
    got, splits = run_dist(lz, torch_cuda, P["A"], P["B"], P["m"], P["lc"], N, form, bounds=bounds, wf_out=wfs)
    t2 = time.time()
    assert all(w == ((True, True) if form == "halo" else (False, False)) for w in wfs), wfs
    if form == "allgather":
        assert all(s is not None for s in splits), splits  # interior pass 1 beside the all-gather
    assert_close_run(lz, P["m"], 16, got, P["ref"])
    print(f"C4 8 virtual ranks ({form}): operator + oracle {P['t_build']:.1f} s, distributed solve {t2 - t1:.1f} s")


@pytest.mark.parametrize("form", ["halo", "allgather"])
@pytest.mark.parametrize("nranks", [1, 2])
def test_vranks_b32_f32_repeatable(lz, orc, torch_cuda, form, nranks):
    """The same distributed b = 32 fp32 solve, each time on fresh handles (new
    workspaces) and non-blocking rank streams, is bitwise the same run after
    run.  Before round 5 the SpMM's long-tile queue counts were zeroed by a
    null-stream hipMemset that did not order against the rank's stream: about
    one run in ten (N = 2; nearly half at N = 1) read a fresh allocation's
    garbage as the queue count -- tiles recomputed in the long-tile pass's
    summation order, alpha ~4e-4 off the oracle after 5 steps, once an illegal
    address."""
    A = lz.gen_banded(20_011, 10.0, 600, seed=30, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=31, dtype=np.float32)
    m, lc = 3, 15_000
    first = None
    for _ in range(8):
        got, _ = run_dist(lz, torch_cuda, A, B, m, lc, nranks, form)
        if first is None:
            first = got
            qo, ao, bo = orc.block_lanczos(A, B, m, lc)
            scale = max(1.0, float(np.abs(ao).max()), float(np.abs(bo[:m]).max()))
            assert np.max(np.abs(got[1] - ao)) <= 1e-4 * scale
        else:
            assert np.array_equal(got[1], first[1]) and np.array_equal(got[2][:m], first[2][:m])
