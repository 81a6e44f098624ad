"""GPU coverage of the distributed entry points on one device, at one rank
(N-rank decompositions on one GPU are in test_gpu_vranks.py, virtual ranks;
RCCL with more than one peer runs only in the driver's multi-GPU bench).

* lz_block_lanczos_halo / lz_halo_init with no communicator and with a
  one-rank RCCL communicator: the per-step halo exchange, the b x b
  all-reduces and the compact-column fused pass, against the oracle
  (methods/block_lanczos.hpp:104-166 op order).
* lz_block_lanczos_dist (all-gather form) with a one-rank communicator.
* Gather sources of >= 2^24 rows / >= 2 GiB (what the all-gather path sees
  at 2+ ranks of 10M rows, and config C4 on one GPU): the windowed fused pass
  and SpMM kernels, and the 64-bit fallbacks when columns leave the window;
  checked against the oracle.
The decomposition at 2 and 3 ranks is checked on CPU (tests/test_dist_gloo.py).
"""
import numpy as np
import pytest

from test_gpu_lanczos import assert_close_run

pytestmark = pytest.mark.gpu


def _bufs(torch, n, nx, m, b=16):
    kw = dict(dtype=torch.float64, device="cuda")
    return (torch.zeros(m * b, **kw), torch.zeros(m, b, b, **kw), torch.zeros(m + 1, b, b, **kw),
            torch.zeros(n, b, **kw), torch.zeros(nx, b, **kw), torch.zeros(nx, b, **kw))


def _run_halo(lz, h, torch, A, B, m, lc):
    n = A.n
    cc, cnt, rows = lz.halo_plan(A.col, np.array([0, n], np.int64), 0)
    assert rows.size == 0 and np.array_equal(cc, A.col)
    h.halo_init(0, n, cnt, rows)
    assert h.halo_sizes() == (0, 0)
    Ad = lz.CsrDevice.from_host(lz.CsrHost(n, A.row_ptr, cc, A.val))
    q, al, be, _, X0, X1 = _bufs(torch, n, n, m)
    h.block_lanczos_halo(Ad, torch.from_numpy(B).cuda(), m, lc, 0, q, al, be, X0, X1)
    torch.cuda.synchronize()
    return q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()


@pytest.mark.parametrize("with_comm", [False, True])
def test_halo_single_rank(lz, orc, torch_cuda, with_comm):
    A = lz.gen_banded(40013, 10.0, 1024, seed=31)
    B = lz.uniform_B(A.n, 16, seed=32)
    m, lc = 8, 777
    h = lz.Handle(0)
    try:
        if with_comm:
            h.comm_init(1, 0, lz.comm_unique_id())
        got = _run_halo(lz, h, torch_cuda, A, B, m, lc)
        assert h.device_error() == 0
    finally:
        h.close()
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def test_halo_requires_init(lz, torch_cuda):
    h = lz.Handle(0)
    try:
        q, al, be, Q0, X0, X1 = _bufs(torch_cuda, 16, 16, 1)
        A = lz.CsrDevice.from_host(lz.gen_banded(16, 2.0, 4, seed=1))
        with pytest.raises(lz.LanczosError, match="lz_halo_init"):
            h.block_lanczos_halo(A, Q0, 1, 0, 0, q, al, be, X0, X1)
        with pytest.raises(lz.LanczosError):  # own rows listed as halo
            h.halo_init(0, 16, np.array([3], np.int64), np.arange(3, dtype=np.int32))
    finally:
        h.close()


def test_allgather_dist_single_rank(lz, orc, torch_cuda):
    A = lz.gen_banded(30011, 10.0, 700, seed=41)
    B = lz.uniform_B(A.n, 16, seed=42)
    m, lc = 6, 123
    n = A.n
    h = lz.Handle(0)
    try:
        h.comm_init(1, 0, lz.comm_unique_id())
        Ad = lz.CsrDevice.from_host(A)
        q, al, be, Q0, W, X = _bufs(torch_cuda, n, n, m)
        h.block_lanczos_dist(Ad, n, n, torch_cuda.from_numpy(B).cuda(), m, lc, 0, q, al, be, Q0, W, X)
        torch_cuda.cuda.synchronize()
        got = (q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy())
    finally:
        h.close()
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def _run_dist_wide(lz, h, torch, A, B, m, lc, n_pad):
    """One-rank all-gather run with a padded gather source of n_pad rows."""
    kw = dict(dtype=torch.float64, device="cuda")
    n = A.n
    Bp = torch.zeros(n_pad, 16, **kw)
    Bp[:n] = torch.from_numpy(B).cuda()
    W = torch.zeros(n_pad, 16, **kw)
    X = torch.zeros(n_pad, 16, **kw)
    Q0 = torch.zeros(n_pad, 16, **kw)
    q, al, be = torch.zeros(m * 16, **kw), torch.zeros(m, 16, 16, **kw), torch.zeros(m + 1, 16, 16, **kw)
    Ad = lz.CsrDevice.from_host(A, n_cols=n_pad)
    h.block_lanczos_dist(Ad, n_pad, n_pad, Bp, m, lc, 0, q, al, be, Q0, W, X)
    torch.cuda.synchronize()
    return q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()


@pytest.mark.parametrize("far", [False, True])
def test_wide_address_fused_pass(lz, orc, torch_cuda, far):
    """n_pad = 2^24 + 64 rows of gather source (2.1 GB, past a 32-bit buffer
    offset).  far=False: every strip's columns lie in its 2^24-row window, so
    the windowed k_fused_pp16 runs; far=True: a few columns point 2^24 rows
    away (padding rows, zero), the window check fails and the 64-bit tile
    kernel runs.  Both against the oracle."""
    torch = torch_cuda
    A = lz.gen_banded(20011, 10.0, 500, seed=51)
    B = lz.uniform_B(A.n, 16, seed=52)
    m, lc = 5, 4321
    n_pad = (1 << 24) + 64
    Ag = A
    if far:  # append one far column (a zero padding row of X) to a few rows
        import scipy.sparse as sp
        M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, n_pad)).tolil()
        for r in (3, 9000, A.n - 1):
            M[r, n_pad - 1] = 0.5
        M = M.tocsr()
        M.sort_indices()
        Ag = lz.CsrHost(A.n, M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data)
    h = lz.Handle(0)
    try:
        h.comm_init(1, 0, lz.comm_unique_id())
        got = _run_dist_wide(lz, h, torch, Ag, B, m, lc, n_pad)
        assert h.device_error() == 0
    finally:
        h.close()
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("nx,layout", [(50021, "random"), ((1 << 24) + 5, "random"), ((1 << 24) + 5, "banded"),
                                       ((1 << 24) + 5, "mixed")])
def test_rectangular_and_wide_address_spmm(lz, orc, handle, torch_cuda, nx, layout):
    """X with more rows than A (n_cols > n_rows).  At 2^24 + 5 rows (2.1 GB,
    b = 16 fp64) the windowed nnz-split kernel runs: "banded" -- every tile's
    columns fit one window (buffer-addressed gather based at the tile's
    smallest column); "random" -- columns spread over all of X, every tile is
    queued to the 64-bit long-tile kernel; "mixed" -- both kinds of tile."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    n = 3001
    cnt = rng.integers(0, 20, n)
    rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    rows = np.repeat(np.arange(n), cnt)
    if layout == "random":
        col = rng.integers(0, nx, rp[-1])
        col[:4] = [0, nx - 1, nx - 2, min(1 << 24, nx - 3)]
    else:
        base = rows * 3000 + rng.integers(0, 2000, rp[-1])  # banded, up to ~9M
        if layout == "mixed":
            far = rows >= n // 2
            base = np.where(far & (rng.random(rp[-1]) < 0.3), nx - 1 - rng.integers(0, 100, rp[-1]), base)
        col = base
    col = col.astype(np.int32)
    val = rng.standard_normal(rp[-1])
    A = lz.CsrHost(n, rp, col, val)
    X = torch.zeros(nx, 16, dtype=torch.float64, device="cuda")
    used = np.unique(col)
    Xu = rng.standard_normal((used.size, 16))
    X[torch.from_numpy(used.astype(np.int64)).cuda()] = torch.from_numpy(Xu).cuda()
    Y = torch.empty(n, 16, dtype=torch.float64, device="cuda")
    handle.spmm(lz.CsrDevice.from_host(A, n_cols=nx), X, Y)
    torch.cuda.synchronize()
    # reference on the compacted columns
    cmap = np.searchsorted(used, col).astype(np.int32)
    ref = orc.csr_spmm(lz.CsrHost(n, rp, cmap, val), Xu)
    assert np.allclose(Y.cpu().numpy(), ref, rtol=1e-13, atol=1e-12)
