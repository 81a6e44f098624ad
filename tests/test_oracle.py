"""Pinning the CPU oracle (oracle/lz_oracle.c): against the reference's own host
code (oracle/_ref), an independent numpy restatement, the golden vectors and
the reference's recorded FDTD convergence (lanczos_plots.m:168-169)."""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_csr

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden import numpy_block_lanczos  # noqa: E402


@pytest.mark.parametrize("key,N,b,m", [("N10_b4_m5", 10, 4, 5), ("N10_b4_m20", 10, 4, 20),
                                       ("N10_b16_m5", 10, 16, 5), ("N10_b16_m20", 10, 16, 20),
                                       ("N3_b4_m8", 3, 4, 8)])
def test_oracle_reproduces_golden(lz, orc, golden, key, N, b, m):
    A = golden_csr(lz, golden, N)
    B = lz.rand_B(A.n, b)
    q, al, be = orc.block_lanczos(A, B, m, int(golden["lc"]))
    sc = max(1.0, np.abs(golden[key + "_alpha"]).max())
    assert np.max(np.abs(al - golden[key + "_alpha"])) <= 1e-12 * sc
    assert np.allclose(be, golden[key + "_beta"], rtol=1e-12, atol=1e-13)
    assert np.allclose(q, golden[key + "_q"], rtol=1e-11, atol=1e-14)
    assert np.max(np.abs(orc.ritz_values(m, b, al, be) - golden[key + "_ritz"])) <= 1e-13


@pytest.mark.parametrize("b", [1, 3, 4, 16])
def test_oracle_vs_numpy_restatement(lz, orc, b):
    A = lz.gen_banded(3001, 9.0, 150, seed=b)
    B = lz.uniform_B(A.n, b, seed=2)
    m, lc = 7, 10
    q, al, be = orc.block_lanczos(A, B, m, lc)
    qn, aln, ben = numpy_block_lanczos(A, B, m, lc)
    assert np.allclose(al, aln, rtol=1e-9, atol=1e-12)
    assert np.allclose(be[:m], ben, rtol=1e-9, atol=1e-12)
    assert np.allclose(q, qn, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("m", [1, 2, 5])
def test_oracle_final_state_vs_numpy(lz, orc, m):
    """The blocks the reference leaves in Q0 (= Q1) and W on return
    (block_lanczos.hpp:159,162): oracle against the numpy restatement."""
    A = lz.gen_banded(2001, 8.0, 120, seed=30 + m)
    B = lz.uniform_B(A.n, 4, seed=3)
    q, al, be, Qf, Wf = orc.block_lanczos_final(A, B, m, 5)
    qn, aln, ben, Qn, Wn = numpy_block_lanczos(A, B, m, 5, final=True)
    assert np.allclose(al, aln, rtol=1e-9, atol=1e-12)
    assert np.allclose(Qf, Qn, rtol=1e-9, atol=1e-12 * np.abs(Qn).max())
    assert np.allclose(Wf, Wn, rtol=1e-8, atol=1e-10 * np.abs(Wn).max())


def test_oracle_spmm_vs_reference_ell_spmm(lz, orc, golden):
    """CSR SpMM restatement == the reference's host Ell_matrix::spmm (ell_matrix.hpp:287-300)."""
    if not orc.ref_available(4):
        pytest.skip("oracle/_ref not built")
    n, d, ix = orc.ref_matrix_a(10)
    X = np.random.default_rng(0).uniform(-1, 1, (n, 4))
    Yref = orc.ref_ell_spmm(n, d, ix, X.T.ravel()).reshape(4, n).T
    Y = orc.csr_spmm(golden_csr(lz, golden, 10), X)
    assert np.allclose(Y, Yref, rtol=0, atol=1e-15 * np.abs(Yref).max())


def test_vector_lanczos_vs_numpy(lz, orc, golden):
    A = golden_csr(lz, golden, 10)
    bv = lz.rand_B(A.n, 4)[:, 0].copy()
    m, lc = 10, int(golden["lc"])
    q, al, be = orc.vector_lanczos(A, bv, m, lc)
    M = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))
    b0 = np.linalg.norm(bv)
    q0 = bv / b0
    w = M @ q0
    a = w @ q0
    w = w - a * q0
    aa, bb, qq = [a], [b0], [q0[lc]]
    for _ in range(1, m):
        bj = np.linalg.norm(w)
        q1 = w / bj
        w = M @ q1 - bj * q0
        a = w @ q1
        w = w - a * q1
        q0 = q1
        aa.append(a); bb.append(bj); qq.append(q0[lc])
    assert np.allclose(al, aa, rtol=1e-10, atol=1e-15)
    assert np.allclose(be, bb, rtol=1e-10)
    assert np.allclose(q, qq, rtol=1e-10, atol=1e-16)
    assert np.allclose(al, golden["N10_vec_m10_alpha"], rtol=1e-11, atol=1e-15)


def test_oracle_sqrtm_known_answer(orc, golden):
    s, si = orc.sqrtm_pair(golden["ka4_matrix"])
    assert np.allclose(s, golden["ka4_sqrtm"], atol=1e-13)
    assert np.allclose(si, golden["ka4_inv_sqrtm"], atol=1e-12)


def test_lanczos_vs_fdtd_convergence(golden):
    """m = 8 at n = 252 reaches the FDTD-limited plateau (1.83e-9 in lanczos_plots.m:168-169)."""
    f = golden["N3_b4_fdtd_1e6"]
    errs = {m: np.linalg.norm(golden[f"N3_b4_m{m}_solution"] - f) / np.linalg.norm(f) for m in (5, 8)}
    assert errs[8] < 2e-9 and errs[5] > errs[8]


def test_oracle_fp32_tracks_fp64(lz, orc):
    A = lz.gen_banded(4000, 10.0, 100, seed=8)
    B = lz.uniform_B(A.n, 8, seed=1)
    _, al64, _ = orc.block_lanczos(A, B, 4, 0)
    A32 = lz.CsrHost(A.n, A.row_ptr, A.col, A.val.astype(np.float32))
    _, al32, _ = orc.block_lanczos(A32, B.astype(np.float32), 4, 0)
    assert np.max(np.abs(al32 - al64)) < 1e-3 * np.abs(al64).max()


def test_oracle_vector_f32_tracks_f64(lz, orc, golden):
    """The fp32 single-vector restatement (test_VectorLanczos<float>) follows the
    fp64 one on the driver's operator to fp32 accuracy, and reproduces the
    golden fp64 run's Ritz values to 1e-5 relative."""
    A = golden_csr(lz, golden, 10)
    bv = lz.rand_B(A.n, 4)[:, 0].copy()
    m, lc = 10, int(golden["lc"])
    q, al, be = orc.vector_lanczos(A, bv, m, lc)
    A32 = lz.CsrHost(A.n, A.row_ptr, A.col, A.val.astype(np.float32))
    qf, alf, bef = orc.vector_lanczos(A32, bv.astype(np.float32), m, lc)
    assert alf.dtype == np.float32 and bef.dtype == np.float32
    assert np.max(np.abs(alf - al)) <= 1e-5 * np.abs(al).max()
    assert np.max(np.abs(bef - be)) <= 1e-5 * np.abs(be).max()
    assert np.max(np.abs(qf - q)) <= 1e-5 * np.abs(q).max()
    r = orc.ritz_values(m, 1, alf.astype(np.float64), np.r_[bef, 0].astype(np.float64))
    ref = orc.ritz_values(m, 1, golden["N10_vec_m10_alpha"], np.r_[golden["N10_vec_m10_beta"], 0.0])
    assert np.max(np.abs(r - ref)) <= 1e-5 * np.abs(ref).max()
