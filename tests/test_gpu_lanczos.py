"""GPU parity of the full Lanczos iterations (liblz_hip.so via the C ABI)
against the CPU oracle and the committed golden vectors.

Bar (BASELINE.json north_star): Ritz values within 1e-10 (absolute, fp64) of
the reference restatement on the same input.  alpha/beta/q are compared with a
relative tolerance of 1e-9 (rounding of reordered reductions amplified by the
recurrence, m <= 20, no re-orthogonalisation).
"""
import numpy as np
import pytest

from conftest import golden_csr

pytestmark = pytest.mark.gpu

RITZ_TOL = 1e-10


def gpu_block(lz, h, torch, A, B, m, lc, fused=True):
    Ad = lz.CsrDevice.from_host(A)
    q, al, be = lz.run_block_lanczos(h, Ad, torch.from_numpy(B).cuda(), m, lc, fused=fused)
    torch.cuda.synchronize()
    return q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()


def assert_close_run(lz, m, b, got, ref, ritz_tol=RITZ_TOL, rtol=1e-9):
    q, al, be = got
    qo, ao, bo = ref
    scale = max(1.0, np.abs(ao).max(), np.abs(bo[:m]).max())
    assert np.max(np.abs(al - ao)) <= rtol * scale
    assert np.max(np.abs(be[:m] - bo[:m])) <= rtol * scale
    assert np.allclose(q, qo, rtol=rtol, atol=rtol * np.abs(qo).max())
    r_gpu = lz.ritz_values(m, b, al, be)
    r_ref = lz.ritz_values(m, b, ao, bo)
    assert np.max(np.abs(r_gpu - r_ref)) <= ritz_tol, np.max(np.abs(r_gpu - r_ref))


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("m", [1, 2, 10])
def test_block_b16_banded(lz, orc, handle, torch_cuda, fused, m):
    A = lz.gen_banded(50021, 10.0, 2048, seed=21)
    B = lz.uniform_B(A.n, 16, seed=4)
    lc = 84
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused)
    ref = orc.block_lanczos(A, B, m, lc)
    assert_close_run(lz, m, 16, got, ref)
    # beta[m] holds the last inverse square root, as the reference's beta[m]
    assert np.allclose(got[2][m], ref[2][m], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n", [50021, 1000 * 16 + 11, 224 * 40 + 16 * 3 + 5])
def test_block_b16_stale_lds(lz, orc, handle, torch_cuda, n):
    """Every CU's LDS filled with NaN bit patterns before each fused pass: a
    last tile whose trailing strips lie past n (no row order staged for them)
    must not carry unwritten LDS into the slabs (it once made alpha NaN by chance)."""
    A = lz.gen_banded(n, 10.0, 512, seed=n)
    B = lz.uniform_B(A.n, 16, seed=6)
    m, lc = 4, n // 2
    Ad = lz.CsrDevice.from_host(A)
    handle.debug_poison_lds()
    torch_cuda.cuda.synchronize()
    q, al, be = lz.run_block_lanczos(handle, Ad, torch_cuda.from_numpy(B).cuda(), m, lc)
    torch_cuda.cuda.synchronize()
    got = (q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy())
    assert np.isfinite(got[1]).all() and np.isfinite(got[2]).all()
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("c16", ["0", "1"])
@pytest.mark.parametrize("n,hw", [(60_013, 2048), (100_003, 40_000), (50_021, 16)])
def test_block_b16_col16(lz, orc, handle, torch_cuda, monkeypatch, c16, n, hw):
    """Pass 1 with 16-bit strip-relative columns (LZ_PASS1_C16, default on) and
    without; half width 40,000 puts columns out of int16 reach of their strip,
    so that operator keeps 32-bit columns either way.  n = 50,021 has an odd
    nnz whose last column is not its strip's first row: the last 4-B word of the
    16-bit columns holds one real column (a buffer range ending mid-dword once
    read it as 0)."""
    monkeypatch.setenv("LZ_PASS1_C16", c16)
    A = lz.gen_banded(n, 10.0, hw, seed=n % 101)
    B = lz.uniform_B(A.n, 16, seed=9)
    m, lc = 6, n - 100
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("wf", ["0", "1"])
@pytest.mark.parametrize("n,npr,hw", [(1000, 10.0, 16), (5_003, 10.0, 64), (60_013, 10.0, 4096),
                                      (200_003, 8.0, 2048), (777_777, 10.0, 8192), (300_007, 10.0, 40_000)])
def test_block_b16_wavefront(lz, orc, handle, torch_cuda, monkeypatch, wf, n, npr, hw):
    """The wavefront step (lz_wf.hip, LZ_PASS_WF default on) and the two-pass
    step against the oracle: fewer pass-1 tiles than XCD regions (n = 1000: 6
    tiles), a partial last tile, bands of 1-2 tiles up to ~85 (the pass-2
    wavefront leads by the widest), and half width 40,000 (32-bit columns, a
    tile reaching ~455 tiles)."""
    monkeypatch.setenv("LZ_PASS_WF", wf)
    A = lz.gen_banded(n, npr, hw, seed=n % 97)
    B = lz.uniform_B(A.n, 16, seed=5)
    m, lc = 9, n // 3
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert handle.device_error() == 0
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("c16", ["0", "1"])
@pytest.mark.parametrize("shape", ["111", "10", "11", "12"])
def test_block_b16_wavefront_shapes(lz, orc, handle, torch_cuda, monkeypatch, shape, c16):
    """Every block shape of the wavefront step (111: 1 loader + 11 consumers + 4
    updaters; NC: 2 loaders + NC consumers + 14 - NC updaters; LZ_WF_SHAPE)
    with 16- and 32-bit columns."""
    monkeypatch.setenv("LZ_WF_SHAPE", shape)
    monkeypatch.setenv("LZ_PASS1_C16", c16)
    A = lz.gen_banded(90_001, 10.0, 4096, seed=17)
    B = lz.uniform_B(A.n, 16, seed=2)
    m, lc = 8, 70_000
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert handle.device_error() == 0
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def _update_launches(lz, handle, torch, Ad, Bd, m, lc):
    """(result, update-pass launches) of one solve: the wavefront step has none."""
    handle.prof_enable(True)
    q, al, be = lz.run_block_lanczos(handle, Ad, Bd, m, lc)
    torch.cuda.synchronize()
    _, c2 = handle.prof_read(handle.PROF_UPDATE_PASS)
    handle.prof_enable(False)
    return (q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()), c2


@pytest.mark.parametrize("c16", ["0", "1"])
@pytest.mark.parametrize("n,npr,hw", [(40_009, 25.0, 2048), (300_007, 25.0, 20_000), (150_001, 26.5, 65_536),
                                      (20_011, 30.0, 1024)])
def test_block_b16_wavefront_wide(lz, orc, handle, torch_cuda, monkeypatch, c16, n, npr, hw):
    """The wide wavefront shape (rows of 10.2-27 entries on average, config C4's
    density: 10 consumers, two 4400-entry stages) against the oracle, with 16-
    and 32-bit columns; half width 65,536 reaches ~820 tiles (C4's band); 30
    entries per row is past the wide stage: the two-pass step runs."""
    monkeypatch.setenv("LZ_PASS1_C16", c16)
    A = lz.gen_banded(n, npr, hw, seed=n % 89)
    B = lz.uniform_B(A.n, 16, seed=4)
    m, lc = 7, n // 2
    got, upd = _update_launches(lz, handle, torch_cuda, lz.CsrDevice.from_host(A),
                                torch_cuda.from_numpy(B).cuda(), m, lc)
    assert handle.device_error() == 0
    assert (upd == 0) == (A.nnz <= 27.0 * n), (upd, A.nnz / n)
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def test_block_b16_wavefront_bitwise(lz, handle, torch_cuda, monkeypatch):
    """The wavefront step is deterministic (static tile assignment, fixed-order
    slabs): the same solve twice gives the same bits."""
    monkeypatch.setenv("LZ_PASS_WF", "1")
    A = lz.gen_banded(400_009, 10.0, 4096, seed=3)
    B = lz.uniform_B(A.n, 16, seed=3)
    r1 = gpu_block(lz, handle, torch_cuda, A, B, 12, 84)
    r2 = gpu_block(lz, handle, torch_cuda, A, B, 12, 84)
    for x, y in zip(r1, r2):
        assert np.array_equal(x, y)


def test_block_b16_tail_rows(lz, orc, handle, torch_cuda):
    """n not a multiple of the 16-row tiles, lc in the last partial tile."""
    A = lz.gen_banded(1000 * 16 + 11, 7.0, 64, seed=2)
    B = lz.uniform_B(A.n, 16, seed=8)
    lc = A.n - 3
    got = gpu_block(lz, handle, torch_cuda, A, B, 6, lc)
    assert_close_run(lz, 6, 16, got, orc.block_lanczos(A, B, 6, lc))


@pytest.mark.parametrize("b", [4, 16])
@pytest.mark.parametrize("m", [5, 20])
def test_block_matrix_a_golden(lz, orc, handle, torch_cuda, golden, b, m):
    """C1: the reference's own Yee operator (N=10) and glibc-rand B, golden vectors."""
    A = golden_csr(lz, golden, 10)
    n = A.n
    B = lz.rand_B(n, b)
    assert np.array_equal(B.T.ravel()[:64], golden[f"N10_b{b}_B_head"])
    lc = int(golden["lc"])
    key = f"N10_b{b}_m{m}"
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    ref = (golden[key + "_q"], golden[key + "_alpha"], golden[key + "_beta"])
    assert_close_run(lz, m, b, got, ref)
    r = lz.ritz_values(m, b, got[1], got[2])
    assert np.max(np.abs(r - golden[key + "_ritz"])) <= RITZ_TOL
    sol = lz.block_solution(m, b, 1.0, got[1], got[2], got[0])
    assert np.allclose(sol, golden[key + "_solution"], rtol=1e-9)


def test_block_bug_compat_operator(lz, orc, handle, torch_cuda, golden):
    """The as-run (change_order bug) operator: 1 nnz/row, non-symmetric."""
    A = golden_csr(lz, golden, 10, bug=True)
    B = lz.rand_B(A.n, 4)
    lc = int(golden["lc"])
    got = gpu_block(lz, handle, torch_cuda, A, B, 5, lc)
    assert_close_run(lz, 5, 4, got, orc.block_lanczos(A, B, 5, lc))


def _f32_checks(lz, m, b, got, ref, rtol):
    """fp32 run vs the fp32 oracle: alpha/beta/q within rtol relative to the
    largest entry, Ritz values within rtol of the spectrum's scale."""
    q, al, be = got
    qo, ao, bo = ref
    scale = max(np.abs(ao).max(), np.abs(bo[:m]).max())
    assert np.max(np.abs(al - ao)) <= rtol * scale, np.max(np.abs(al - ao)) / scale
    assert np.max(np.abs(be[:m] - bo[:m])) <= rtol * scale, np.max(np.abs(be[:m] - bo[:m])) / scale
    assert np.max(np.abs(q - qo)) <= rtol * np.abs(qo).max(), np.max(np.abs(q - qo)) / np.abs(qo).max()
    r_gpu = lz.ritz_values(m, b, al.astype(np.float64), be.astype(np.float64))
    r_ref = lz.ritz_values(m, b, ao.astype(np.float64), bo.astype(np.float64))
    assert np.max(np.abs(r_gpu - r_ref)) <= rtol * np.abs(r_ref).max(), np.max(np.abs(r_gpu - r_ref))


# fp32 bar: 1e-4 relative (about 800 fp32 ulps at the largest entry, through
# m steps of a recurrence without re-orthogonalisation and reordered fp32 sums)
F32_RTOL = 1e-4


@pytest.mark.parametrize("form", ["b2", "e", "unfused"])
@pytest.mark.parametrize("n,cap,m", [(20000, 2000, 4), (1_000_003, 100_000, 4), (20011, 2000, 8)])
def test_block_f32_b32_powerlaw(lz, orc, handle, torch_cuda, monkeypatch, n, cap, m, form):
    """C5 shape: fp32, b = 32, power-law rows (load imbalance); at n = 1M with
    rows up to 1e5 the long-tile queue of the SpMM runs.  alpha, beta, the row
    probe q and the Ritz values against the fp32 oracle for the Q-free step in
    its beta^2 form (default: U = A W_j - W_{j-1} M from the SpMM epilogue), in
    its pass-E form (LZ_C5_B2=0), and the reference op order."""
    fused = form != "unfused"
    if form == "e":
        monkeypatch.setenv("LZ_C5_B2", "0")
    else:
        monkeypatch.delenv("LZ_C5_B2", raising=False)
    A = lz.gen_powerlaw(n, 10.0, 2.1, cap, seed=5, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=6, dtype=np.float32)
    lc = 17
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=fused)
    _f32_checks(lz, m, 32, got, orc.block_lanczos(A, B, m, lc), F32_RTOL)
    assert handle.device_error() == 0


@pytest.mark.parametrize("form", ["b2", "e"])
@pytest.mark.parametrize("n,m", [(20_011, 4), (100_003, 3), (33, 2)])
def test_block_f32_b32_ub_dma_bitwise(lz, handle, torch_cuda, monkeypatch, n, m, form):
    """The b = 32 fp32 dense passes with their operands staged through LDS by
    DMA (the default: pass UB k_fused_ub32d in the beta^2 form; passes E and U,
    k_fused_e32d / k_fused_u32d, in the pass-E form, LZ_C5_B2=0) against the
    register-operand forms (LZ_UB_DMA=0): the same products in the same order,
    so alpha, beta, q and the post-call Q0 / Q1 / W are the same bits, including
    the ragged last strip (n not a multiple of 32) and the last step's Q store."""
    torch = torch_cuda
    if form == "e":
        monkeypatch.setenv("LZ_C5_B2", "0")
    A = lz.gen_powerlaw(n, 10.0, 2.1, max(2, n // 10), seed=n % 89, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=9, dtype=np.float32)
    Ad, Bd = lz.CsrDevice.from_host(A), torch.from_numpy(B).cuda()
    kw = dict(dtype=torch.float32, device="cuda")
    outs = []
    for dma in ("1", "0"):
        monkeypatch.setenv("LZ_UB_DMA", dma)
        q, al, be = torch.zeros(m * 32, **kw), torch.zeros(m, 32, 32, **kw), torch.zeros(m + 1, 32, 32, **kw)
        Q0, Q1, W = (torch.full((A.n, 32), float("nan"), **kw) for _ in range(3))
        handle.block_lanczos_blas(Ad, Bd, m, min(84, A.n - 1), q, al, be, Q0, Q1, W)
        torch.cuda.synchronize()
        assert handle.device_error() == 0
        outs.append([t.cpu().numpy() for t in (q, al, be, Q0, Q1, W)])
    for x, y in zip(*outs):
        assert np.array_equal(x, y, equal_nan=True)


@pytest.mark.parametrize("b", [1, 3, 4, 5, 8, 32])
def test_block_fused_any_b_f64(lz, orc, handle, torch_cuda, b):
    """The Q-free iteration at every block width but 16 (separate SpMM + VALU
    passes E and U, lz_fused32.hip; b = 4 is the reference driver's N_COL):
    fused and unfused against the oracle, Ritz within 1e-10."""
    A = lz.gen_banded(20011, 10.0, 600, seed=b)
    B = lz.uniform_B(A.n, b, seed=b + 1)
    m, lc = 6, 20010
    ref = orc.block_lanczos(A, B, m, lc)
    for fused in (True, False):
        got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=fused)
        assert_close_run(lz, m, b, got, ref)
    assert handle.device_error() == 0


@pytest.mark.parametrize("b", [4, 16])
def test_block_fused_any_b_f32(lz, orc, handle, torch_cuda, b):
    """fp32 at b != 32 (VALU passes, fp64 accumulation rounded to fp32 once)."""
    A = lz.gen_banded(20011, 10.0, 600, seed=b, dtype=np.float32)
    B = lz.uniform_B(A.n, b, seed=b + 1, dtype=np.float32)
    m, lc = 5, 77
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=True)
    _f32_checks(lz, m, b, got, orc.block_lanczos(A, B, m, lc), F32_RTOL)
    assert handle.device_error() == 0


@pytest.mark.parametrize("n,lc,m", [(33, 32, 1), (127, 100, 3), (4099, 4098, 5), (300_007, 300_000, 5)])
def test_block_f32_b32_fused_shapes(lz, orc, handle, torch_cuda, n, lc, m):
    """The b = 32 fp32 Q-free passes at ragged sizes: fewer rows than one 32-row
    tile or one 128-row unit, the row probe in the last partial tile, a banded
    operator (C3 generator) in fp32.  m b <= n keeps the Krylov block full rank."""
    A = lz.gen_banded(n, 10.0, 300, seed=n, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=7, dtype=np.float32)
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=True)
    _f32_checks(lz, m, 32, got, orc.block_lanczos(A, B, m, lc), F32_RTOL)
    assert handle.device_error() == 0


def test_block_c3_full_size(lz, orc, handle, torch_cuda):
    """BASELINE config C3 at full size (n = 1e7, nnz = 1e8, half-width 4096,
    b = 16 fp64; the bench operator): Ritz values within 1e-10 of the oracle."""
    A = lz.gen_banded(10_000_000, 10.0, 4096, seed=20261015)
    B = lz.uniform_B(A.n, 16, seed=20261015)
    m, lc = 4, 84
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert handle.device_error() == 0
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


def test_block_c5_full_size(lz, orc, handle, torch_cuda):
    """BASELINE config C5 at full size (the bench operator: n = 1e7 power-law
    rows, alpha 2.1, rows up to 1e5, ~9.9e7 nnz; b = 32 fp32, the beta^2 form
    with the long-tile queue): alpha, beta, q and the Ritz values against the
    fp32 oracle (methods/block_lanczos.hpp:104-166) to 1e-4 relative."""
    A = lz.gen_powerlaw(10_000_000, 10.0, 2.1, 100000, seed=20261015, dtype=np.float32)
    B = lz.uniform_B(A.n, 32, seed=20261015, dtype=np.float32)
    m, lc = 4, 9_999_991
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert handle.device_error() == 0
    _f32_checks(lz, m, 32, got, orc.block_lanczos(A, B, m, lc), F32_RTOL)


def test_block_b16_c4_density(lz, orc, handle, torch_cuda):
    """C4's row density (25 nnz/row, half-width 2^16) at small n: pass 1's
    10-consumer / 4400-entry shape and the SpMM's 1536-entry stage."""
    A = lz.gen_banded(200_003, 25.0, 1 << 16, seed=44)
    B = lz.uniform_B(A.n, 16, seed=45)
    m, lc = 6, 100_000
    for fused in (True, False):
        got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=fused)
        assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))
    assert handle.device_error() == 0


def test_block_b16_window_2e24_rows(lz, orc, handle, torch_cuda):
    """n = 2^24 + 4099 rows on one GPU (X past 2 GiB: the C4-on-one-GPU
    regime): the windowed pass-1 and SpMM kernels, fused and unfused, against
    the oracle.  12 nnz/row, half-width 2^16."""
    A = lz.gen_banded((1 << 24) + 4099, 12.0, 1 << 16, seed=46)
    B = lz.uniform_B(A.n, 16, seed=47)
    m, lc = 3, (1 << 24) + 17
    ref = orc.block_lanczos(A, B, m, lc)
    for fused in (True, False):
        got = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=fused)
        assert_close_run(lz, m, 16, got, ref)
    assert handle.device_error() == 0


def test_vector_lanczos(lz, orc, handle, torch_cuda, golden):
    torch = torch_cuda
    for A, m, lc in ((lz.gen_banded(200003, 10.0, 4096, seed=1), 12, 84),
                     (golden_csr(lz, golden, 10), 10, int(golden["lc"]))):
        bv = lz.uniform_B(A.n, 1, seed=3)[:, 0].copy()
        Ad = lz.CsrDevice.from_host(A)
        kw = dict(dtype=torch.float64, device="cuda")
        q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
        ws = [torch.empty(A.n, **kw) for _ in range(3)]
        handle.vector_lanczos(Ad, torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
        qo, ao, bo = orc.vector_lanczos(A, bv, m, lc)
        assert np.allclose(al.cpu().numpy(), ao, rtol=1e-9, atol=1e-12)
        assert np.allclose(be.cpu().numpy(), bo, rtol=1e-9)
        assert np.allclose(q.cpu().numpy(), qo, rtol=1e-9, atol=1e-14)
        bt = np.concatenate([be.cpu().numpy(), [0.0]])
        r = lz.ritz_values(m, 1, al.cpu().numpy(), bt)
        ro = lz.ritz_values(m, 1, ao, np.concatenate([bo, [0.0]]))
        assert np.max(np.abs(r - ro)) <= RITZ_TOL


def test_vector_lanczos_c2_full_size(lz, orc, handle, torch_cuda):
    """BASELINE config C2 as benchmarked: n = 1,000,000, ~1e7 nnz, half width
    4096, fp64, lc = 84, 30 steps, against the oracle (alpha / beta / q and the
    Ritz values of the 30 x 30 T)."""
    torch = torch_cuda
    A = lz.gen_banded(1_000_000, 10.0, 4096, 20261015)
    bv = lz.uniform_B(A.n, 1, 20261015)[:, 0].copy()
    m, lc = 30, 84
    Ad = lz.CsrDevice.from_host(A)
    kw = dict(dtype=torch.float64, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    ws = [torch.empty(A.n, **kw) for _ in range(3)]
    handle.vector_lanczos(Ad, torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
    qo, ao, bo = orc.vector_lanczos(A, bv, m, lc)
    assert np.allclose(al.cpu().numpy(), ao, rtol=1e-9, atol=1e-12)
    assert np.allclose(be.cpu().numpy(), bo, rtol=1e-9)
    assert np.allclose(q.cpu().numpy(), qo, rtol=1e-9, atol=1e-14)
    r = lz.ritz_values(m, 1, al.cpu().numpy(), np.concatenate([be.cpu().numpy(), [0.0]]))
    ro = lz.ritz_values(m, 1, ao, np.concatenate([bo, [0.0]]))
    assert np.max(np.abs(r - ro)) <= RITZ_TOL


@pytest.mark.parametrize("kernel", ["win", "row", "cs", "cs2"])
def test_vector_lanczos_heavy_tiles(lz, orc, handle, torch_cuda, monkeypatch, kernel):
    """Power-law rows, every SpMV kernel (LZ_VL_KERNEL): tiles whose CSR run
    exceeds the CSR-stream kernels' LDS capacity take their wave-per-row path;
    nnz not a multiple of 4 (tail quad)."""
    torch = torch_cuda
    if kernel == "win":  # default: band-window kernel; this operator's band exceeds the ring
        monkeypatch.delenv("LZ_VL_KERNEL", raising=False)
    else:
        monkeypatch.setenv("LZ_VL_KERNEL", kernel)
    A = lz.gen_powerlaw(60001, 10.0, 1.8, 30000, seed=9, dtype=np.float64)
    m, lc = 10, 4321
    bv = lz.uniform_B(A.n, 1, seed=4)[:, 0].copy()
    kw = dict(dtype=torch.float64, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    ws = [torch.empty(A.n, **kw) for _ in range(3)]
    handle.vector_lanczos(lz.CsrDevice.from_host(A), torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
    qo, ao, bo = orc.vector_lanczos(A, bv, m, lc)
    assert np.allclose(al.cpu().numpy(), ao, rtol=1e-9, atol=1e-12)
    assert np.allclose(be.cpu().numpy(), bo, rtol=1e-9)
    assert np.allclose(q.cpu().numpy(), qo, rtol=1e-9, atol=1e-14)


@pytest.mark.parametrize("n,H,kernel", [(600013, 4096, None), (600013, 4097, None), (600013, 7168, None),
                                        (600013, 7169, None), (60013, 7168, None), (60013, 7168, "win512")])
def test_vector_lanczos_band_window_edge(lz, orc, handle, torch_cuda, monkeypatch, n, H, kernel):
    """Half bands at each band-window shape's limit (2H + 2R <= ring: 4096 for
    <512, 9216>, 7168 for <1024, 16384>) and one past it; several tiles per
    block and blocks with a single partial tile; a forced shape whose ring is
    too small (the kernel's global-gather instantiation)."""
    import scipy.sparse as sp
    torch = torch_cuda
    if kernel:
        monkeypatch.setenv("LZ_VL_KERNEL", kernel)
    else:
        monkeypatch.delenv("LZ_VL_KERNEL", raising=False)
    A0 = lz.gen_banded(n, 8.0, 3000, seed=H)
    M = sp.csr_matrix((A0.val, A0.col, A0.row_ptr), shape=(n, n))
    r = np.array([17, n - 1 - H, n // 2])
    E = sp.coo_matrix((np.full(6, 0.01), (np.r_[r, r + H], np.r_[r + H, r])), shape=(n, n))
    M = (M + E).tocsr()
    M.sort_indices()
    A = lz.CsrHost(n, M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data.astype(np.float64))
    assert np.max(np.abs(M.indices - np.repeat(np.arange(n), np.diff(M.indptr)))) == H
    m, lc = 10, n // 3
    bv = lz.uniform_B(n, 1, seed=5)[:, 0].copy()
    kw = dict(dtype=torch.float64, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    ws = [torch.empty(n, **kw) for _ in range(3)]
    handle.vector_lanczos(lz.CsrDevice.from_host(A), torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
    qo, ao, bo = orc.vector_lanczos(A, bv, m, lc)
    assert np.allclose(al.cpu().numpy(), ao, rtol=1e-9, atol=1e-12)
    assert np.allclose(be.cpu().numpy(), bo, rtol=1e-9)
    assert np.allclose(q.cpu().numpy(), qo, rtol=1e-9, atol=1e-14)


@pytest.mark.parametrize("op,kernel", [("banded", None), ("banded", "row"), ("powerlaw", None),
                                       ("banded", "win1024")])
def test_vector_lanczos_f32(lz, orc, handle, torch_cuda, monkeypatch, op, kernel):
    """fp32 single-vector Lanczos (test_lanczos.cu:355, test_VectorLanczos<float>)
    against the oracle's fp32 restatement.  Tolerances are fp32-sized: the
    oracle itself moves alpha by 1.4e-6 (relative to max|alpha|) when b is
    perturbed by one ulp in every 7th entry, so 2e-5 is ~15x that and ~1e3x
    below what an indexing error produces."""
    torch = torch_cuda
    if kernel:
        monkeypatch.setenv("LZ_VL_KERNEL", kernel)
    else:
        monkeypatch.delenv("LZ_VL_KERNEL", raising=False)
    if op == "banded":  # half band 4096: the band-window kernel's ring path by default
        A = lz.gen_banded(200003, 10.0, 4096, seed=1, dtype=np.float32)
    else:  # wide band: the window kernel's global-gather instantiation / lanes per row
        A = lz.gen_powerlaw(60001, 10.0, 1.8, 30000, seed=9, dtype=np.float32)
    m, lc = 10, 84
    bv = lz.uniform_B(A.n, 1, seed=3, dtype=np.float32)[:, 0].copy()
    kw = dict(dtype=torch.float32, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    ws = [torch.empty(A.n, **kw) for _ in range(3)]
    handle.vector_lanczos(lz.CsrDevice.from_host(A), torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
    qo, ao, bo = orc.vector_lanczos(A, bv, m, lc)
    al, be, q = al.cpu().numpy(), be.cpu().numpy(), q.cpu().numpy()
    assert np.all(np.isfinite(al)) and np.all(np.isfinite(be))
    assert np.max(np.abs(al - ao)) <= 2e-5 * np.abs(ao).max()
    assert np.max(np.abs(be - bo)) <= 2e-5 * np.abs(bo).max()
    assert np.max(np.abs(q - qo)) <= 2e-5 * np.abs(qo).max()
    r = lz.ritz_values(m, 1, al.astype(np.float64), np.r_[be, 0].astype(np.float64))
    ro = lz.ritz_values(m, 1, ao.astype(np.float64), np.r_[bo, 0].astype(np.float64))
    assert np.max(np.abs(r - ro)) <= 1e-5 * np.abs(ro).max()


def test_vector_lanczos_golden(lz, handle, torch_cuda, golden):
    torch = torch_cuda
    A = golden_csr(lz, golden, 10)
    bv = lz.rand_B(A.n, 4)[:, 0].copy()
    m, lc = 10, int(golden["lc"])
    kw = dict(dtype=torch.float64, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    ws = [torch.empty(A.n, **kw) for _ in range(3)]
    handle.vector_lanczos(lz.CsrDevice.from_host(A), torch.from_numpy(bv).cuda(), m, lc, q, al, be, *ws)
    assert np.allclose(al.cpu().numpy(), golden["N10_vec_m10_alpha"], rtol=1e-9, atol=1e-13)
    assert np.allclose(be.cpu().numpy(), golden["N10_vec_m10_beta"], rtol=1e-9)


def test_fdtd_block(lz, orc, handle, torch_cuda, golden):
    torch = torch_cuda
    A = golden_csr(lz, golden, 3)
    B = lz.rand_B(A.n, 4)
    lc = int(golden["lc"])
    kw = dict(dtype=torch.float64, device="cuda")
    out = torch.empty(4, **kw)
    handle.ftdt_block(lz.CsrDevice.from_host(A), torch.from_numpy(B).cuda(), 2000, 1.0, lc,
                      torch.empty(A.n, 4, **kw), torch.empty(A.n, 4, **kw), out)
    assert np.allclose(out.cpu().numpy(), orc.fdtd_block(A, B, 2000, 1.0, lc), rtol=1e-12)


@pytest.mark.parametrize("n,b,steps,graph", [(3001, 3, 1001, None), (3001, 16, 513, None), (3001, 16, 513, "0"),
                                             ((1 << 18) + 1, 4, 3, None)])
def test_fdtd_block_shapes(lz, orc, handle, torch_cuda, monkeypatch, n, b, steps, graph):
    """Odd step counts (final state in the ping-pong buffer), b not a power of
    two, a graph replay count with eager remainder, the eager loop
    (LZ_FDTD_GRAPH=0, read per call), and the unfused large-n path."""
    torch = torch_cuda
    if graph is None:
        monkeypatch.delenv("LZ_FDTD_GRAPH", raising=False)
    else:
        monkeypatch.setenv("LZ_FDTD_GRAPH", graph)
    A = lz.gen_banded(n, 6.0, 200, seed=n)
    A = lz.CsrHost(A.n, A.row_ptr, A.col, A.val * 0.05)
    B = lz.uniform_B(n, b, seed=7)
    lc = n // 3
    kw = dict(dtype=torch.float64, device="cuda")
    U = torch.empty(n, b, **kw)
    out = torch.empty(b, **kw)
    handle.ftdt_block(lz.CsrDevice.from_host(A), torch.from_numpy(B).cuda(), steps, 1.0, lc,
                      U, torch.empty(n, b, **kw), out)
    ref = orc.fdtd_block(A, B, steps, 1.0, lc)
    assert np.allclose(out.cpu().numpy(), ref, rtol=1e-12, atol=1e-14)


def test_block_large_properties(lz, orc, handle, torch_cuda):
    """n = 2M, b = 16: fused == unfused (two GPU paths), bitwise run-to-run
    determinism, and the oracle (OpenMP) on the same input."""
    A = lz.gen_banded(2_000_000, 10.0, 4096, seed=20261015)
    B = lz.uniform_B(A.n, 16, seed=20261015)
    m, lc = 5, 1234567
    g1 = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    g2 = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert all(np.array_equal(x, y) for x, y in zip(g1, g2)), "fused path not deterministic"
    gu = gpu_block(lz, handle, torch_cuda, A, B, m, lc, fused=False)
    assert_close_run(lz, m, 16, g1, gu)
    assert_close_run(lz, m, 16, g1, orc.block_lanczos(A, B, m, lc))


def test_block_b16_long_runs(lz, orc, handle, torch_cuda):
    """Fused pass with 128-row tiles whose CSR run exceeds the LDS staging
    buffer (power-law rows up to 5000 nnz): chunked staging path, fp64."""
    A = lz.gen_powerlaw(30011, 12.0, 1.8, 5000, seed=13, dtype=np.float64)
    rp = np.asarray(A.row_ptr)
    tile_runs = rp[np.minimum(np.arange(0, A.n + 128, 128), A.n)]
    assert np.diff(tile_runs).max() > 2048, "test operator must overflow the staging buffer"
    B = lz.uniform_B(A.n, 16, seed=14)
    m, lc = 6, 4321
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))
    # the persistent pass-1 kernels' bounded spins never timed out
    assert handle.device_error() == 0


@pytest.mark.parametrize("wf", ["0", "1"])
def test_prof_class_mask(lz, handle, torch_cuda, monkeypatch, wf):
    """lz_prof_enable_mask records only the selected kernel classes (the bench's
    timed region records pass 1 alone); lz_prof_enable(1) records all of them;
    results do not depend on what is recorded.  The wavefront step (wf = 1) has
    m launches in the pass-1 class and no update pass."""
    monkeypatch.setenv("LZ_PASS_WF", wf)
    torch = torch_cuda
    A = lz.gen_banded(20011, 10.0, 1024, seed=5)
    B = lz.uniform_B(A.n, 16, seed=6)
    Ad = lz.CsrDevice.from_host(A)
    Bd = torch.from_numpy(B).cuda()
    m = 3
    outs = []
    for classes in ([handle.PROF_SPMM_PASS], None):
        handle.prof_enable(True, classes=classes)
        q, al, be = lz.run_block_lanczos(handle, Ad, Bd, m, 84)
        torch.cuda.synchronize()
        ms1, c1 = handle.prof_read(handle.PROF_SPMM_PASS)
        ms2, c2 = handle.prof_read(handle.PROF_UPDATE_PASS)
        handle.prof_enable(False)
        assert c1 == m and ms1 > 0.0
        assert (c2 == 0) if (classes or wf == "1") else (c2 == m)
        outs.append((q.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()))
    assert all(np.array_equal(x, y) for x, y in zip(outs[0], outs[1]))
    assert handle.device_error() == 0


@pytest.mark.parametrize("m", [1, 2, 5])
@pytest.mark.parametrize("path", ["wavefront", "shape10", "shape10_lds", "shape12", "twopass", "unfused", "sep_b4",
                                  "b2_f32_b32"])
def test_block_final_state(lz, orc, handle, torch_cuda, monkeypatch, path, m):
    """On return Q0 = Q1 = Q_{m-1} and W = the last residual, as the reference
    leaves them (methods/block_lanczos.hpp:145,159,162; Q1 is not written at
    m = 1): every step form against the oracle's final blocks.  The default
    wavefront shape (111) writes the state in a pass-2-only step launch (QO);
    the other shapes (LZ_WF_SHAPE 10 / 12) take the final_state pass, by MFMA
    strips (k_final_state16m) or, LZ_FS_MFMA=0, its LDS form (k_final_state16),
    each reading the residual buffers the parity of m chose."""
    torch = torch_cuda
    b, dt = (4, np.float64) if path == "sep_b4" else (32, np.float32) if path == "b2_f32_b32" else (16, np.float64)
    if path == "twopass":
        monkeypatch.setenv("LZ_PASS_WF", "0")
    if path.startswith("shape"):
        monkeypatch.setenv("LZ_WF_SHAPE", path[5:7])
    if path == "shape10_lds":  # the LDS form of the post-call pass (default: MFMA strips)
        monkeypatch.setenv("LZ_FS_MFMA", "0")
    A = lz.gen_banded(30_011, 10.0, 700, seed=70 + m, dtype=dt)
    B = lz.uniform_B(A.n, b, seed=71, dtype=dt)
    lc = 29_000
    Ad = lz.CsrDevice.from_host(A)
    kw = dict(dtype=torch.float64 if dt == np.float64 else torch.float32, device="cuda")
    q, al, be = torch.zeros(m * b, **kw), torch.zeros(m, b, b, **kw), torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.full((A.n, b), float("nan"), **kw) for _ in range(3))
    handle.block_lanczos_blas(Ad, torch.from_numpy(B).cuda(), m, lc, q, al, be, Q0, Q1, W,
                              fused=path != "unfused")
    torch.cuda.synchronize()
    assert handle.device_error() == 0
    qo, ao, bo, Qf, Wf = orc.block_lanczos_final(A, B, m, lc)
    tol = 1e-8 if dt == np.float64 else 2e-3
    Qg, Wg = Q0.cpu().numpy(), W.cpu().numpy()
    assert np.max(np.abs(Qg - Qf)) <= tol * np.abs(Qf).max()
    assert np.max(np.abs(Wg - Wf)) <= tol * np.abs(Wf).max()
    if m >= 2:
        assert np.array_equal(Q1.cpu().numpy(), Qg)
    else:
        assert bool(torch.isnan(Q1).all())  # untouched, as the reference's
    assert np.allclose(al.cpu().numpy(), ao, rtol=tol, atol=tol * np.abs(ao).max())


def test_block_final_state_off(lz, orc, handle, torch_cuda):
    """lz_set_final_state(h, 0): the same alpha / beta / q bits, the blocks are scratch."""
    torch = torch_cuda
    A = lz.gen_banded(20_011, 10.0, 500, seed=75)
    B = lz.uniform_B(A.n, 16, seed=76)
    m, lc = 4, 77
    runs = []
    for on in (True, False):
        handle.set_final_state(on)
        try:
            runs.append(gpu_block(lz, handle, torch, A, B, m, lc))
        finally:
            handle.set_final_state(True)
    for x, y in zip(*runs):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("m", [1, 2, 3, 6])
def test_vector_final_state(lz, handle, torch_cuda, m):
    """vector_lanczos leaves q0 = q1 = q_{m-1} and w = the last residual
    (methods/vector_lanczos.hpp:60,62; q1 untouched at m = 1)."""
    import scipy.sparse as sp
    torch = torch_cuda
    A = lz.gen_banded(20_011, 10.0, 400, seed=80 + m)
    bv = lz.uniform_B(A.n, 1, seed=81)[:, 0].copy()
    M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))
    b0 = np.linalg.norm(bv)
    q0 = bv / b0
    w = M @ q0
    w = w - (w @ q0) * q0
    for _ in range(1, m):
        q1 = w / np.linalg.norm(w)
        w = M @ q1 - np.linalg.norm(w) * q0
        w = w - (w @ q1) * q1
        q0 = q1
    Ad = lz.CsrDevice.from_host(A)
    kw = dict(dtype=torch.float64, device="cuda")
    q, al, be = torch.zeros(m, **kw), torch.zeros(m, **kw), torch.zeros(m, **kw)
    g0 = torch.zeros(A.n, **kw)
    g1, gw = (torch.full((A.n,), float("nan"), **kw) for _ in range(2))
    handle.vector_lanczos(Ad, torch.from_numpy(bv).cuda(), m, 5, q, al, be, g0, g1, gw)
    torch.cuda.synchronize()
    assert np.allclose(g0.cpu().numpy(), q0, rtol=1e-9, atol=1e-12 * np.abs(q0).max())
    assert np.allclose(gw.cpu().numpy(), w, rtol=1e-8, atol=1e-10 * np.abs(w).max())
    if m >= 2:
        assert np.array_equal(g1.cpu().numpy(), g0.cpu().numpy())
    else:
        assert bool(torch.isnan(g1).all())


def test_device_error_word_cleared_by_next_solve(lz, orc, handle, torch_cuda):
    """A device error word left behind by an earlier call (here stored by the
    test hook, as a wait that gave up would) must not fail the next solve: every
    checked solve clears the word when it starts.  The hook itself
    is visible through lz_device_error, which reads and clears."""
    A = lz.gen_banded(20_011, 10.0, 512, seed=31)
    B = lz.uniform_B(A.n, 16, seed=3)
    m, lc = 4, 777
    handle.debug_set_device_error(5)
    assert handle.device_error() == 5
    assert handle.device_error() == 0
    handle.debug_set_device_error(6)
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)  # raises on LZ_E_DEVICE
    assert handle.device_error() == 0
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))


@pytest.mark.parametrize("cap", ["32", "7"])
def test_block_b16_wavefront_grid_cap(lz, orc, handle, torch_cuda, monkeypatch, cap):
    """LZ_GRID_CAP (read per call): the wavefront step on at most `cap` blocks,
    as one virtual rank's share of the CUs runs (bench --config c4rank with the
    cap measures that share alone); same results as the oracle."""
    monkeypatch.setenv("LZ_GRID_CAP", cap)
    A = lz.gen_banded(60_013, 10.0, 2048, seed=77)
    B = lz.uniform_B(A.n, 16, seed=2)
    m, lc = 5, 30_000
    got = gpu_block(lz, handle, torch_cuda, A, B, m, lc)
    assert_close_run(lz, m, 16, got, orc.block_lanczos(A, B, m, lc))
