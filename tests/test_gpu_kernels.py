"""GPU parity of the individual hot-path kernels (liblz_hip.so through the C ABI)
against the CPU oracle / exact numpy references.

Tolerances: fp64 results of a sum of k products are compared with
|gpu - ref| <= 64 * eps * sum|terms| (reordered summation, FMA), fp32 likewise
with the fp32 eps.  Integer/index work (row probe) is bit-exact.
"""
import numpy as np
import pytest

from conftest import golden_csr

pytestmark = pytest.mark.gpu

EPS = {np.float64: np.finfo(np.float64).eps, np.float32: np.finfo(np.float32).eps}


def spmm_bound(A, X):
    absA = A.__class__(A.n, A.row_ptr, A.col, np.abs(A.val))
    return absA, np.abs(X)


def dense_of(A):
    import scipy.sparse as sp
    return sp.csr_matrix((A.val.astype(np.float64), A.col, A.row_ptr), shape=(A.n, A.n))


def check_spmm(lz, orc, h, torch, A, b, dtype, layout="row"):
    rng = np.random.default_rng(b * 7 + A.n)
    X = rng.uniform(-1, 1, (A.n, b)).astype(dtype)
    Ad = lz.CsrDevice.from_host(lz.CsrHost(A.n, A.row_ptr, A.col, A.val.astype(dtype)))
    M = dense_of(A)
    ref = M @ X.astype(np.float64)
    bound = abs(M) @ np.abs(X.astype(np.float64))
    if layout == "row":
        Xd = torch.from_numpy(X).cuda()
        Yd = torch.full((A.n, b), np.nan, dtype=Xd.dtype, device="cuda")
        h.spmm(Ad, Xd, Yd)
        Y = Yd.cpu().numpy()
    else:  # column-major (the reference's Dense_matrix layout): tensors (b, n)
        Xd = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
        Yd = torch.full((b, A.n), np.nan, dtype=Xd.dtype, device="cuda")
        h.spmm(Ad, Xd, Yd, layout=lz.LZ_COL_MAJOR)
        Y = Yd.cpu().numpy().T
    tol = 64 * EPS[dtype] * bound + 1e-300
    assert np.all(np.abs(Y - ref) <= tol), f"b={b} {dtype} max err {np.max(np.abs(Y - ref))}"
    if dtype == np.float64 and layout == "row":
        Yo = orc.csr_spmm(A, X)
        assert np.all(np.abs(Y - Yo) <= tol)


@pytest.mark.parametrize("b", [1, 2, 3, 4, 5, 8, 16, 32])
def test_spmm_rowmajor_f64(lz, orc, handle, torch_cuda, b):
    A = lz.gen_banded(20011, 10.0, 500, seed=3)
    check_spmm(lz, orc, handle, torch_cuda, A, b, np.float64)


@pytest.mark.parametrize("b", [4, 8, 16, 32])
def test_spmm_rowmajor_f32(lz, orc, handle, torch_cuda, b):
    A = lz.gen_banded(9001, 12.0, 300, seed=5)
    check_spmm(lz, orc, handle, torch_cuda, A, b, np.float32)


@pytest.mark.parametrize("n", [3001, 3072])
@pytest.mark.parametrize("b", [1, 2, 4, 5, 16, 32, 64])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_spmm_colmajor(lz, orc, handle, torch_cuda, b, dtype, n):
    """Column-major X/Y (b >= 2: X transposed in, the row-major kernels store
    their Y tiles column by column; n = 3072: the 16-B column pieces)."""
    A = lz.gen_banded(n, 8.0, 100, seed=9)
    check_spmm(lz, orc, handle, torch_cuda, A, b, dtype, layout="col")


@pytest.mark.parametrize("n", [20011, 20016])
@pytest.mark.parametrize("b,dtype", [(16, np.float64), (32, np.float32)])
def test_spmm_colmajor_long_tiles(lz, orc, handle, torch_cuda, b, dtype, n):
    """128-B rows in the column-major layout: the nnz-split kernel stores its Y
    tile column by column, in both its tile pass and its long-tile pass
    (power-law rows longer than the 768-entry stage), n not a multiple of the
    48-row tile."""
    A = lz.gen_powerlaw(n, 10.0, 1.3, 8000, seed=8, dtype=np.float64)
    tiles = np.diff(A.row_ptr[np.minimum(np.arange(0, A.n + 48, 48), A.n)])
    assert (tiles > 768).sum() > 10 and np.diff(A.row_ptr).max() > 768  # long tiles, and a row longer than the stage
    check_spmm(lz, orc, handle, torch_cuda, A, b, dtype, layout="col")


@pytest.mark.parametrize("direct", [False, True])
def test_spmm_colmajor_padded_ld(lz, handle, torch_cuda, monkeypatch, direct):
    """The reference's Dense_matrix: leading dimension = padded rows (> n)."""
    torch = torch_cuda
    if direct:
        monkeypatch.setenv("LZ_SPMM_CM", "direct")  # read per call: k_spmm_cm runs
    A = lz.gen_banded(1000, 6.0, 50, seed=4)
    n, b, ld = A.n, 16, 1024 + 7
    rng = np.random.default_rng(2)
    X = rng.uniform(-1, 1, (n, b))
    Xp = torch.full((b, ld), np.nan, dtype=torch.float64, device="cuda")
    Xp[:, :n] = torch.from_numpy(X.T.copy()).cuda()
    Yp = torch.full((b, ld), 7.0, dtype=torch.float64, device="cuda")
    handle.spmm(lz.CsrDevice.from_host(A), Xp[:, :n], Yp[:, :n], layout=lz.LZ_COL_MAJOR)
    M = dense_of(A)
    Y = Yp.cpu().numpy()
    assert np.all(np.abs(Y[:, :n].T - M @ X) <= 64 * EPS[np.float64] * (abs(M) @ np.abs(X)))
    assert np.all(Y[:, n:] == 7.0)  # padding untouched


def test_spmm_matrix_a_and_bug_compat(lz, orc, handle, torch_cuda, golden):
    for bug in (False, True):
        A = golden_csr(lz, golden, 10, bug)
        check_spmm(lz, orc, handle, torch_cuda, A, 4, np.float64)
        check_spmm(lz, orc, handle, torch_cuda, A, 16, np.float64)


def test_spmm_edge_cases(lz, orc, handle, torch_cuda):
    # empty rows, a dense row, n = 1, nnz = 0
    rng = np.random.default_rng(1)
    n = 777
    rows = []
    for r in range(n):
        k = 0 if r % 5 == 0 else (n if r == 3 else rng.integers(1, 20))
        rows.append(np.sort(rng.choice(n, size=min(k, n), replace=False)))
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(-1, 1, col.size)
    A = lz.CsrHost(n, rp, col, val)
    for b in (1, 4, 16, 32):
        check_spmm(lz, orc, handle, torch_cuda, A, b, np.float64)
    one = lz.CsrHost(1, np.array([0, 1], np.int64), np.array([0], np.int32), np.array([2.5]))
    check_spmm(lz, orc, handle, torch_cuda, one, 16, np.float64)
    empty = lz.CsrHost(5, np.zeros(6, np.int64), np.zeros(0, np.int32), np.zeros(0))
    check_spmm(lz, orc, handle, torch_cuda, empty, 16, np.float64)


def test_spmv(lz, orc, handle, torch_cuda):
    torch = torch_cuda
    for npr in (3.0, 10.0, 40.0, 100.0):
        A = lz.gen_banded(10007, npr, 2000, seed=int(npr))
        x = np.random.default_rng(2).uniform(-1, 1, A.n)
        Ad = lz.CsrDevice.from_host(A)
        y = torch.empty(A.n, dtype=torch.float64, device="cuda")
        handle.spmv(Ad, torch.from_numpy(x).cuda(), y)
        ref = orc.csr_spmm(A, x)[:, 0]
        bound = abs(dense_of(A)) @ np.abs(x)
        assert np.all(np.abs(y.cpu().numpy() - ref) <= 64 * EPS[np.float64] * bound)


@pytest.mark.parametrize("b,n", [(16, 100003), (16, 13), (4, 5003), (8, 777), (32, 4099), (1, 1000)])
def test_gram_and_cross_gram(lz, handle, torch_cuda, b, n):
    torch = torch_cuda
    rng = np.random.default_rng(b + n)
    W = rng.uniform(-1, 1, (n, b))
    Q = rng.uniform(-1, 1, (n, b))
    Wd, Qd = torch.from_numpy(W).cuda(), torch.from_numpy(Q).cuda()
    R = torch.empty(b, b, dtype=torch.float64, device="cuda")
    handle.mm_tt(Wd, R)
    bound = np.abs(W).T @ np.abs(W)
    assert np.all(np.abs(R.cpu().numpy() - W.T @ W) <= 64 * EPS[np.float64] * bound)
    handle.mm_tt2(Wd, Qd, R)
    ref = 0.5 * (W.T @ Q + Q.T @ W)
    bound = np.abs(W).T @ np.abs(Q) + np.abs(Q).T @ np.abs(W)
    assert np.all(np.abs(R.cpu().numpy() - ref) <= 64 * EPS[np.float64] * bound)


def test_gram_deterministic(lz, handle, torch_cuda):
    torch = torch_cuda
    W = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, (1 << 20, 16))).cuda()
    R1 = torch.empty(16, 16, dtype=torch.float64, device="cuda")
    R2 = torch.empty_like(R1)
    handle.mm_tt(W, R1)
    handle.mm_tt(W, R2)
    assert torch.equal(R1, R2)


@pytest.mark.parametrize("b,n", [(16, 100003), (16, 7), (4, 999), (32, 3001), (8, 64)])
@pytest.mark.parametrize("sw", [0.0, 1.0])
def test_tsmm(lz, handle, torch_cuda, b, n, sw):
    torch = torch_cuda
    rng = np.random.default_rng(b * n)
    Q = rng.uniform(-1, 1, (n, b))
    S = rng.uniform(-1, 1, (b, b))
    W0 = rng.uniform(-1, 1, (n, b))
    Wd = torch.from_numpy(W0.copy()).cuda()
    handle.mm_ts(sw, -1.0, torch.from_numpy(Q).cuda(), torch.from_numpy(S).cuda(), Wd)
    ref = sw * W0 - Q @ S
    bound = np.abs(sw * W0) + np.abs(Q) @ np.abs(S)
    assert np.all(np.abs(Wd.cpu().numpy() - ref) <= 64 * EPS[np.float64] * bound)


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("n", [5000, 131, 128])
@pytest.mark.parametrize("sw", [0.0, 1.0])
def test_tsmm_f32(lz, handle, torch_cuda, b, n, sw):
    """fp32: b = 32 on the 32x32x2 MFMA kernel (transposed product, 16-B row
    pieces); b = 16 on the f64 16x16x4 kernel (operands widened on load)."""
    torch = torch_cuda
    rng = np.random.default_rng(3 + n + b)
    Q = rng.uniform(-1, 1, (n, b)).astype(np.float32)
    S = rng.uniform(-1, 1, (b, b)).astype(np.float32)
    W0 = rng.uniform(-1, 1, (n, b)).astype(np.float32)
    W = torch.from_numpy(W0.copy()).cuda()
    handle.mm_ts(sw, -0.5, torch.from_numpy(Q).cuda(), torch.from_numpy(S).cuda(), W)
    ref = sw * W0.astype(np.float64) - 0.5 * (Q.astype(np.float64) @ S.astype(np.float64))
    bound = np.abs(sw * W0).astype(np.float64) + 0.5 * (np.abs(Q).astype(np.float64) @ np.abs(S).astype(np.float64))
    assert np.all(np.abs(W.cpu().numpy() - ref) <= 64 * EPS[np.float32] * bound)


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("n", [100003, 77])
def test_gram_f32(lz, handle, torch_cuda, b, n):
    """fp32 Gram and symmetric cross-Gram: b = 32 on the 32x32x2 MFMA kernel,
    b = 16 on the f64 16x16x4 kernel."""
    torch = torch_cuda
    rng = np.random.default_rng(n + b)
    W = rng.uniform(-1, 1, (n, b)).astype(np.float32)
    Q = rng.uniform(-1, 1, (n, b)).astype(np.float32)
    W64, Q64 = W.astype(np.float64), Q.astype(np.float64)
    R = torch.empty(b, b, dtype=torch.float32, device="cuda")
    handle.mm_tt(torch.from_numpy(W).cuda(), R)
    bound = np.abs(W64).T @ np.abs(W64)
    assert np.all(np.abs(R.cpu().numpy() - W64.T @ W64) <= 64 * EPS[np.float32] * bound)
    handle.mm_tt2(torch.from_numpy(W).cuda(), torch.from_numpy(Q).cuda(), R)
    ref = 0.5 * (W64.T @ Q64 + Q64.T @ W64)
    bound = np.abs(W64).T @ np.abs(Q64) + np.abs(Q64).T @ np.abs(W64)
    assert np.all(np.abs(R.cpu().numpy() - ref) <= 64 * EPS[np.float32] * bound)


@pytest.mark.parametrize("b", [1, 2, 3, 4, 7, 16, 32])
def test_sqrtm_pair(lz, orc, handle, torch_cuda, b):
    torch = torch_cuda
    rng = np.random.default_rng(b)
    X = rng.uniform(-1, 1, (4 * b + 3, b))
    G = X.T @ X + 1e-3 * np.eye(b)
    beta = torch.empty(b, b, dtype=torch.float64, device="cuda")
    binv = torch.empty_like(beta)
    ev = torch.empty(b, dtype=torch.float64, device="cuda")
    handle.sqrtm(torch.from_numpy(G).cuda(), beta, binv, ev)
    s, si = orc.sqrtm_pair(G)
    scale = np.linalg.norm(G, 2)
    assert np.max(np.abs(beta.cpu().numpy() - s)) <= 1e-12 * np.sqrt(scale) * b
    assert np.max(np.abs(binv.cpu().numpy() @ beta.cpu().numpy() - np.eye(b))) <= 1e-10 * np.linalg.cond(G) ** 0.5
    assert np.allclose(ev.cpu().numpy(), np.linalg.eigvalsh(G), rtol=1e-12, atol=1e-13 * scale)


def test_sqrtm_known_answer(lz, handle, torch_cuda, golden):
    """The 4x4 matrix of kernels/my_sqrtm_solver.cpp:385 (indefinite: |lambda| is used)."""
    torch = torch_cuda
    K = golden["ka4_matrix"]
    beta = torch.empty(4, 4, dtype=torch.float64, device="cuda")
    binv = torch.empty_like(beta)
    ev = torch.empty(4, dtype=torch.float64, device="cuda")
    handle.sqrtm(torch.from_numpy(K).cuda(), beta, binv, ev)
    assert np.allclose(ev.cpu().numpy(), golden["ka4_eigvals"], rtol=0, atol=1e-13)
    assert np.allclose(beta.cpu().numpy(), golden["ka4_sqrtm"], rtol=0, atol=1e-13)
    assert np.allclose(binv.cpu().numpy(), golden["ka4_inv_sqrtm"], rtol=0, atol=1e-12)


def test_copy_row_exact(lz, handle, torch_cuda):
    torch = torch_cuda
    Q = torch.arange(1000 * 16, dtype=torch.float64, device="cuda").reshape(1000, 16)
    q = torch.zeros(64, dtype=torch.float64, device="cuda")
    handle.copy_row_to_vector(84, 16, Q, q)
    assert torch.equal(q[16:32], Q[84]) and torch.count_nonzero(q[:16]) == 0


def test_errors_are_loud(lz, handle, torch_cuda):
    torch = torch_cuda
    W = torch.zeros(10, 3, dtype=torch.float64, device="cuda")
    with pytest.raises(lz.LanczosError):
        handle.sqrtm(torch.zeros(40, 40, dtype=torch.float64, device="cuda"), W, W)
    A = lz.CsrDevice.from_host(lz.gen_banded(100, 5.0, 10))
    with pytest.raises(lz.LanczosError):  # b = 65 > the 64-column limit
        handle.spmm(A, torch.zeros(100, 65, dtype=torch.float64, device="cuda"),
                    torch.zeros(100, 65, dtype=torch.float64, device="cuda"))


@pytest.mark.parametrize("b,dtype,ld_pad", [(4, "float64", 768), (16, "float64", 5), (32, "float32", 0), (3, "float64", 17)])
def test_to_row_major(lz, handle, torch_cuda, b, dtype, ld_pad):
    """lz_to_row_major: the reference's column-major Dense_matrix (leading
    dimension = rows padded, objects/dense_matrix.hpp:9) into a row-major block."""
    torch = torch_cuda
    rows = 7001
    ld = rows + ld_pad
    tdt = getattr(torch, dtype)
    Xcm = torch.randn(b, ld, dtype=tdt, device="cuda")
    Y = torch.empty(rows, b, dtype=tdt, device="cuda")
    handle.to_row_major(Xcm, Y)
    torch.cuda.synchronize()
    assert torch.equal(Y, Xcm[:, :rows].t())


@pytest.mark.parametrize("n,npr,hw,dtype,b", [(50021, 10.0, 2048, "float64", 16), (3001, 30.0, 100, "float64", 16),
                                              (100003, 3.0, 500, "float64", 16), (40009, 12.0, 900, "float32", 32),
                                              (449, 10.0, 40, "float64", 16)])
def test_spmm_fixed_nnz_tiles(lz, orc, handle, torch_cuda, monkeypatch, n, npr, hw, dtype, b):
    """LZ_SPMM_FNZ=1: tiles of 448 entries owning the rows that start in them
    (row ends in the column's bit 31) against the oracle; 3 nnz/row puts > 88
    rows in a tile, so that operator takes the default kernel."""
    torch = torch_cuda
    monkeypatch.setenv("LZ_SPMM_FNZ", "1")
    npdt = np.float64 if dtype == "float64" else np.float32
    A = lz.gen_banded(n, npr, hw, seed=n % 997, dtype=npdt)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((n, b)).astype(npdt)
    Y = torch.empty(n, b, dtype=getattr(torch, dtype), device="cuda")
    Ad = lz.CsrDevice.from_host(A)
    handle.spmm(Ad, torch.from_numpy(X).cuda(), Y)
    torch.cuda.synchronize()
    ref = orc.csr_spmm(A, X)
    tol = 1e-13 if dtype == "float64" else 1e-5
    assert np.allclose(Y.cpu().numpy(), ref, rtol=tol, atol=tol * np.abs(ref).max())


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("cond", [1.0, 1e2, 1e4, 1e6, 1e8, 1e10, -1.0])
def test_sqrtm_b32_newton_schulz(lz, orc, handle, torch_cuda, monkeypatch, cond, dtype):
    """b = 32 (config C5's block): the Newton-Schulz route on the f64 MFMA by four
    waves (lz_sqrtm.hpp sqrtm_ns32) where |Z|_F^2 bounds kappa(G) by 4e6, the
    one-wave Jacobi route past it and for an indefinite G -- both against the
    oracle's eigendecomposition sqrtm (utils/lib_utils.hpp:696-745) and against
    each other (LZ_SQRTM_NS=0: Jacobi always)."""
    torch = torch_cuda
    b = 32
    rng = np.random.default_rng(int(abs(cond)) % 1000 + 7)
    Q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    ev = 3.0 * np.power(abs(cond), -np.arange(b) / (b - 1))
    if cond < 0:
        ev[[2, 17]] *= -1.0
    G = (Q * ev) @ Q.T
    G = (0.5 * (G + G.T)).astype(dtype)
    s, si = orc.sqrtm_pair(G.astype(np.float64))
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    out = {}
    for ns in ("1", "0"):
        monkeypatch.setenv("LZ_SQRTM_NS", ns)
        beta = torch.empty(b, b, dtype=tdt, device="cuda")
        binv = torch.empty_like(beta)
        handle.sqrtm(torch.from_numpy(G).cuda(), beta, binv)
        out[ns] = (beta.cpu().numpy().astype(np.float64), binv.cpu().numpy().astype(np.float64))
    kap = abs(cond)
    floor = 1e-12 if dtype == np.float64 else 2e-6
    for ns, (bg, big) in out.items():
        assert np.max(np.abs(bg - s)) <= max(floor, 1e-16 * kap ** 0.5) * np.abs(s).max(), ns
        assert np.max(np.abs(big - si)) <= max(floor, 1e-16 * kap) * np.abs(si).max(), ns
    if kap >= 1e7:  # past the kappa bound both take the Jacobi route: the same bits
        assert np.array_equal(out["1"][0], out["0"][0]) and np.array_equal(out["1"][1], out["0"][1])


@pytest.mark.parametrize("cond", [1.0, 1e2, 1e4, 1e6, 1e8, 1e10, -1.0])
def test_sqrtm_b16_newton_schulz(lz, orc, handle, torch_cuda, monkeypatch, cond):
    """b = 16 without eigenvalues asked for: the Newton-Schulz route (lz_sqrtm.hpp
    sqrtm_ns16) where G is well conditioned, the Jacobi route past ~1e6 (and for
    an indefinite G, cond < 0: |lambda| as the reference's) -- both against the
    oracle's eigendecomposition sqrtm and against each other (LZ_SQRTM_NS=0)."""
    torch = torch_cuda
    b = 16
    rng = np.random.default_rng(int(abs(cond)) % 1000 + 5)
    Q, _ = np.linalg.qr(rng.standard_normal((b, b)))
    ev = 2.5 * np.power(abs(cond), -np.arange(b) / (b - 1))
    if cond < 0:
        ev[[3, 9]] *= -1.0  # indefinite: the eigendecomposition route takes |lambda|
    G = (Q * ev) @ Q.T
    G = 0.5 * (G + G.T)
    s, si = orc.sqrtm_pair(G)
    out = {}
    for ns in ("1", "0"):
        monkeypatch.setenv("LZ_SQRTM_NS", ns)
        beta = torch.empty(b, b, dtype=torch.float64, device="cuda")
        binv = torch.empty_like(beta)
        handle.sqrtm(torch.from_numpy(G).cuda(), beta, binv)
        out[ns] = (beta.cpu().numpy(), binv.cpu().numpy())
    kap = abs(cond)
    for ns, (bg, big) in out.items():
        # (two eigendecomposition routes differ by ~eps sqrt(kappa) in beta at kappa = 1e10)
        assert np.max(np.abs(bg - s)) <= max(1e-12, 1e-16 * kap ** 0.5) * np.abs(s).max(), ns
        assert np.max(np.abs(big - si)) <= max(1e-12, 1e-16 * kap) * np.abs(si).max(), ns
    assert np.max(np.abs(out["1"][1] - out["0"][1])) <= max(1e-12, 1e-16 * kap) * np.abs(si).max()
    if kap >= 1e7:
        # past the |Z|_F^2 <= 4e6 bound (kappa(G) <= 4e6) both take the Jacobi
        # route: the same bits (before round 5, kappa = 1e8 stopped in
        # Newton-Schulz with beta^-1 ~6e-10 off)
        assert np.array_equal(out["1"][0], out["0"][0]) and np.array_equal(out["1"][1], out["0"][1])
