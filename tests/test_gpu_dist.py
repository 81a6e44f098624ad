"""GPU coverage of the distributed entry points on one device (the driver's
multi-GPU bench is the only place more ranks run).

* lz_block_lanczos_halo / lz_halo_init with no communicator and with a
  one-rank RCCL communicator: the per-step halo exchange, the b x b
  all-reduces and the compact-column fused pass, against the oracle
  (methods/block_lanczos.hpp:104-166 op order).
* lz_block_lanczos_dist (all-gather form) with a one-rank communicator.
* The wide-address fallbacks: a gather source of >= 2^24 rows / >= 2 GiB
  (what the all-gather path sees at 2+ ranks of 10M rows) runs the 64-bit
  addressed fused pass and SpMM kernels; checked against the oracle.
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


def test_wide_address_fused_pass(lz, orc, torch_cuda):
    """n_pad = 2^24 + 64 rows of gather source (2.1 GB): the all-gather form's
    fused pass takes the 64-bit addressed tile kernel."""
    torch = torch_cuda
    A = lz.gen_banded(20011, 10.0, 500, seed=51)
    B = lz.uniform_B(A.n, 16, seed=52)
    m, lc = 5, 4321
    n, n_pad = A.n, (1 << 24) + 64
    kw = dict(dtype=torch.float64, device="cuda")
    h = lz.Handle(0)
    try:
        h.comm_init(1, 0, lz.comm_unique_id())
        Bp = torch.zeros(n_pad, 16, **kw)
        Bp[:n] = torch.from_numpy(B).cuda()
        W = torch.zeros(n_pad, 16, **kw)
        X = torch.zeros(n_pad, 16, **kw)
        q, al, be = torch.zeros(m * 16, **kw), torch.zeros(m, 16, 16, **kw), torch.zeros(m + 1, 16, 16, **kw)
        Q0 = torch.zeros(n_pad, 16, **kw)
        Ad = lz.CsrDevice.from_host(A, n_cols=n_pad)
        h.block_lanczos_dist(Ad, n_pad, n_pad, Bp, m, lc, 0, q, al, be, Q0, W, X)
        torch.cuda.synchronize()
        got = (q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy())
        del Bp, W, X
    finally:
        h.close()
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("nx", [50021, (1 << 24) + 5])
def test_rectangular_and_wide_address_spmm(lz, orc, handle, torch_cuda, nx):
    """X with more rows than A (n_cols > n_rows); at 2^24 + 5 rows (2.1 GB,
    b = 16 fp64) the 64-bit addressed kernel runs.  Columns spread over all of X."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    n = 3001
    cnt = rng.integers(0, 20, n)
    rp = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    col = rng.integers(0, nx, rp[-1]).astype(np.int32)
    col[:4] = [0, nx - 1, nx - 2, min(1 << 24, nx - 3)]
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
