"""Host logic (liblz_host.so): problem generation, formats, post-processing,
partitioning -- pinned to the reference's own host code (oracle/_ref, when the
reference tree is present) and to the committed golden vectors."""
import ctypes
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr


def csr_equal(A, B):
    return (A.n == B.n and np.array_equal(A.row_ptr, B.row_ptr) and np.array_equal(A.col, B.col)
            and A.val.tobytes() == B.val.tobytes())


@pytest.mark.parametrize("N", [3, 10])
@pytest.mark.parametrize("bug", [False, True])
def test_matrix_a_matches_golden_bitwise(lz, golden, N, bug):
    assert csr_equal(lz.matrix_a(N, bug), golden_csr(lz, golden, N, bug))


@pytest.mark.parametrize("N", [1, 2, 4, 7, 12])
def test_matrix_a_matches_reference_host_code(lz, orc, N):
    """Restated generator vs the reference's Matrix_A compiled in place."""
    if not orc.ref_available(4):
        pytest.skip("oracle/_ref not built (reference tree absent)")
    for bug in (False, True):
        n, d, ix = lz.matrix_a_ell(N, bug)
        nr, dr, ixr = orc.ref_matrix_a(N, bug)
        if bug:  # the reference returns the as-run row-major stride-4 layout
            dr = dr.reshape(nr, 4).T.ravel()
            ixr = ixr.reshape(nr, 4).T.ravel()
        assert n == nr == 3 * N * (N + 1) * (2 * N + 1)
        assert d.tobytes() == dr.tobytes() and np.array_equal(ix, ixr)


def test_matrix_a_structure(lz):
    A = lz.matrix_a(10)
    M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))
    assert A.n == 6930 and A.nnz == 26400
    assert abs(M - M.T).max() < 1e-16
    Ab = lz.matrix_a(10, bug_compat=True)
    assert np.all(np.diff(Ab.row_ptr) <= 1)


def test_ell_to_csr_keep_zeros(lz):
    n = 6930
    _, d, ix = lz.matrix_a_ell(10)
    A0 = lz.ell_to_csr(n, 4, d, ix, keep_zeros=False)
    A1 = lz.ell_to_csr(n, 4, d, ix, keep_zeros=True)
    assert A1.nnz == 4 * n and A0.nnz == 26400
    x = np.random.default_rng(0).uniform(size=n)
    y0 = sp.csr_matrix((A0.val, A0.col, A0.row_ptr), shape=(n, n)) @ x
    y1 = sp.csr_matrix((A1.val, A1.col, A1.row_ptr), shape=(n, n)) @ x
    assert np.allclose(y0, y1, rtol=0, atol=1e-15)


def test_rand_B_is_glibc_stream(lz, golden):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    draws = np.array([libc.rand() for _ in range(1 + 4 * 100)], np.float64)
    B = lz.rand_B(100, 4)  # after the lc draw, column-major fill
    assert np.array_equal(B.T.ravel(), draws[1:] / 2147483647 + 1.0)
    assert lz.rand_lc(1) == 1 + int(draws[0]) % 100 == int(golden["lc"]) == 84
    n = int(golden["N10_n"])
    for b in (4, 16):
        Bc = lz.rand_B(n, b, row_major=False)
        flat = np.asarray(Bc).T.ravel()
        assert np.array_equal(flat[:64], golden[f"N10_b{b}_B_head"])
        assert flat.sum() == pytest.approx(float(golden[f"N10_b{b}_B_sum"]), rel=1e-14)


def test_sym_eig_vs_numpy(lz):
    rng = np.random.default_rng(1)
    for k in (1, 2, 5, 33, 160):
        A = rng.uniform(-1, 1, (k, k))
        A = A + A.T
        ev, V = lz.sym_eig(A, vectors=True)
        assert np.allclose(ev, np.linalg.eigvalsh(A), atol=1e-12 * max(1, abs(ev).max()))
        assert np.allclose(A @ V, V * ev, atol=1e-11 * max(1, abs(ev).max()))
        assert np.allclose(V.T @ V, np.eye(k), atol=1e-12)


@pytest.mark.parametrize("key", ["N10_b4_m5", "N10_b4_m20", "N10_b16_m5", "N10_b16_m20", "N3_b4_m8"])
def test_ritz_and_solution_from_golden(lz, golden, key):
    """Host eigensolver (tred2/tql2) vs the oracle's Jacobi on the golden alpha/beta."""
    m = int(key.split("_m")[1])
    b = int(key.split("_b")[1].split("_")[0])
    al, be, q = golden[key + "_alpha"], golden[key + "_beta"], golden[key + "_q"]
    assert np.max(np.abs(lz.ritz_values(m, b, al, be) - golden[key + "_ritz"])) <= 1e-13
    assert np.allclose(lz.block_solution(m, b, 1.0, al, be, q), golden[key + "_solution"], rtol=1e-11)


def test_assemble_T_layout(lz):
    b, m = 2, 3
    al = np.arange(m * b * b, dtype=float).reshape(m, b, b)
    be = 100 + np.arange((m + 1) * b * b, dtype=float).reshape(m + 1, b, b)
    T = lz.Assemble_T(m, b, al, be)
    assert np.array_equal(T[0:2, 0:2], al[0]) and np.array_equal(T[2:4, 2:4], al[1])
    assert np.array_equal(T[0:2, 2:4], be[1]) and np.array_equal(T[2:4, 0:2], be[1].T)
    assert np.array_equal(T[2:4, 4:6], be[2]) and not T[0:2, 4:6].any()


def test_banded_generator(lz):
    A = lz.gen_banded(50000, 10.0, 1000, seed=3)
    M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))
    assert abs(M - M.T).max() == 0.0
    assert 9.5 < A.nnz / A.n < 10.5
    for r in (0, 17, 49999):
        c = A.col[A.row_ptr[r]:A.row_ptr[r + 1]]
        assert np.all(np.diff(c) > 0) and np.all(np.abs(c - r) <= 1000)
    again = lz.gen_banded(50000, 10.0, 1000, seed=3)
    assert csr_equal(A, again)
    L = lz.gen_banded_local(50000, 12345, 40000, 10.0, 1000, seed=3)
    s, e = A.row_ptr[12345], A.row_ptr[40000]
    assert np.array_equal(L.row_ptr, A.row_ptr[12345:40001] - s)
    assert np.array_equal(L.col, A.col[s:e]) and L.val.tobytes() == A.val[s:e].tobytes()
    A32 = lz.gen_banded(1000, 10.0, 100, seed=3, dtype=np.float32)
    A64 = lz.gen_banded(1000, 10.0, 100, seed=3)
    assert np.array_equal(A32.val, A64.val.astype(np.float32))


def test_powerlaw_generator(lz):
    A = lz.gen_powerlaw(100000, 10.0, 2.1, 100000, seed=1)
    M = sp.csr_matrix((A.val.astype(np.float64), A.col, A.row_ptr), shape=(A.n, A.n))
    assert abs(M - M.T).max() == 0.0
    deg = np.diff(A.row_ptr)
    assert 7 < deg.mean() < 13 and deg.max() > 20 * deg.mean()


def test_partition_and_remap(lz):
    A = lz.gen_banded(10007, 10.0, 200, seed=2)
    for parts in (1, 2, 3, 8):
        bnd = lz.partition_rows(A, parts)
        assert bnd[0] == 0 and bnd[-1] == A.n and np.all(np.diff(bnd) >= 0)
        per = np.diff(A.row_ptr[bnd])
        assert per.max() - per.min() <= 2 * np.diff(A.row_ptr).max()
        n_pad = int(np.diff(bnd).max())
        cm = lz.remap_cols_padded(A.col, bnd, n_pad)
        owner = np.searchsorted(bnd, A.col, side="right") - 1
        assert np.array_equal(cm, owner * n_pad + (A.col - bnd[owner]))


def test_csr_file_roundtrip(lz, tmp_path):
    A = lz.gen_banded(3000, 6.0, 50, seed=4)
    p = str(tmp_path / "a.lzcsr")
    lz.csr_write(p, A)
    assert csr_equal(lz.csr_read(p), A)
    with pytest.raises(lz.LanczosError):
        lz.csr_read(os.path.join(str(tmp_path), "missing"))
