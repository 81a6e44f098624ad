"""Generate the committed golden fixtures (run in the build container, where
/root/reference exists).  Inputs come from the reference's OWN host code
compiled in place (oracle/_ref: Matrix_A + mult_diagonal [+ change_order],
random_matrix_B after the lc draw); the Lanczos outputs come from the oracle's
CPU restatement of block_lanczos_blas / vector_lanczos, cross-checked here
against an independent numpy restatement before anything is written.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402


class Csr:
    def __init__(self, n, rp, col, val):
        self.n, self.row_ptr, self.col, self.val = n, rp, col, val


def ell_to_csr(n, d, ix, row_major_stride4=False):
    w = d.size // n
    if row_major_stride4:   # layout after change_order(4): slot s of row r at r*4+s
        d = d.reshape(n, w).T.ravel()
        ix = ix.reshape(n, w).T.ravel()
    rows = np.tile(np.arange(n), w)
    keep = d != 0.0
    A = sp.csr_matrix((d[keep], (rows[keep], ix[keep].astype(np.int64))), shape=(n, n))
    A.sort_indices()
    return Csr(n, A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float64))


def numpy_block_lanczos(A, B, m, lc, final=False):
    """Independent restatement (dense numpy) of methods/block_lanczos.hpp:104-166.
    final: also return the Q0 (= Q1) and W blocks the reference leaves behind."""
    Ad = sp.csr_matrix((A.val, A.col, A.row_ptr), shape=(A.n, A.n))

    def sq(G):
        lam, V = np.linalg.eigh(G)
        return (V * np.sqrt(abs(lam))) @ V.T, (V / np.sqrt(abs(lam))) @ V.T
    b0, bi = sq(B.T @ B)
    Q0 = B @ bi
    W = Ad @ Q0
    a = 0.5 * (W.T @ Q0 + Q0.T @ W)
    W = W - Q0 @ a
    al, be, q = [a], [b0], [Q0[lc]]
    for _ in range(1, m):
        bj, bi = sq(W.T @ W)
        Q1 = W @ bi
        W = Ad @ Q1
        W = W - Q0 @ bj
        a = 0.5 * (W.T @ Q1 + Q1.T @ W)
        W = W - Q1 @ a
        Q0 = Q1
        al.append(a); be.append(bj); q.append(Q0[lc])
    if final:
        return np.concatenate(q), np.array(al), np.array(be), Q0, W
    return np.concatenate(q), np.array(al), np.array(be)


def main():
    assert oracle.ref_available(4) and oracle.ref_available(16), "build oracle/_ref first (make -C oracle)"
    lc = oracle.ref_lc(4)
    out = {"lc": np.int64(lc)}
    for N in (3, 10):
        n, d, ix = oracle.ref_matrix_a(N, False)
        A = ell_to_csr(n, d, ix)
        nb, db, ixb = oracle.ref_matrix_a(N, True)
        Ab = ell_to_csr(nb, db, ixb, row_major_stride4=True)
        out[f"N{N}_n"] = np.int64(n)
        for tag, M in (("", A), ("_bug", Ab)):
            out[f"N{N}{tag}_row_ptr"] = M.row_ptr
            out[f"N{N}{tag}_col"] = M.col
            out[f"N{N}{tag}_val"] = M.val
        for b in (4, 16):
            Bc = oracle.ref_random_B(n, b)
            B = Bc.reshape(b, n).T.copy()
            out[f"N{N}_b{b}_B_head"] = Bc[:64].copy()
            out[f"N{N}_b{b}_B_sum"] = np.float64(Bc.sum())
            for m in ((5, 8) if N == 3 else (5, 20)):
                q, al, be = oracle.block_lanczos(A, B, m, lc)
                qn, aln, ben = numpy_block_lanczos(A, B, m, lc)
                assert np.allclose(q, qn, rtol=1e-9, atol=1e-12), "oracle vs numpy: q"
                assert np.allclose(al, aln, rtol=1e-9, atol=1e-12), "oracle vs numpy: alpha"
                assert np.allclose(be[:m], ben, rtol=1e-9, atol=1e-12), "oracle vs numpy: beta"
                ritz = oracle.ritz_values(m, b, al, be)
                T = np.zeros((m * b, m * b))
                for j in range(m):
                    T[j*b:(j+1)*b, j*b:(j+1)*b] = aln[j]
                    if j:
                        T[(j-1)*b:j*b, j*b:(j+1)*b] = ben[j]
                        T[j*b:(j+1)*b, (j-1)*b:j*b] = ben[j].T
                assert np.max(np.abs(ritz - np.linalg.eigvalsh(T))) < 1e-12, "oracle vs numpy: Ritz"
                key = f"N{N}_b{b}_m{m}"
                out[key + "_q"] = q
                out[key + "_alpha"] = al
                out[key + "_beta"] = be
                out[key + "_ritz"] = ritz
                out[key + "_solution"] = oracle.block_solution(m, b, 1.0, al, be, q)
        # single-vector Lanczos on the first column of the b=4 B
        Bc = oracle.ref_random_B(n, 4)
        bv = Bc[:n].copy()
        q, al, be = oracle.vector_lanczos(A, bv, 10, lc)
        out[f"N{N}_vec_m10_q"], out[f"N{N}_vec_m10_alpha"], out[f"N{N}_vec_m10_beta"] = q, al, be
    # the 4x4 known-answer matrix of kernels/my_sqrtm_solver.cpp:385
    K = np.array([4, 1, -2, 2, 1, 2, 0, 1, -2, 0, 3, -2, 2, 1, -2, -1], np.float64).reshape(4, 4)
    out["ka4_matrix"] = K
    out["ka4_eigvals"] = np.linalg.eigvalsh(K)
    lam, V = np.linalg.eigh(K)
    out["ka4_sqrtm"] = (V * np.sqrt(abs(lam))) @ V.T
    out["ka4_inv_sqrtm"] = (V / np.sqrt(abs(lam))) @ V.T
    # FDTD cross-check at n = 252 (lanczos_plots.m:168-169 plateau 1.83e-9 at m >= 8)
    n3 = int(out["N3_n"])
    A3 = Csr(n3, out["N3_row_ptr"], out["N3_col"], out["N3_val"])
    B3 = oracle.ref_random_B(n3, 4).reshape(4, n3).T.copy()
    out["N3_b4_fdtd_1e6"] = oracle.fdtd_block(A3, B3, 1000000, 1.0, lc)
    np.savez_compressed(os.path.join(HERE, "golden_matrix_a.npz"), **out)
    print("wrote", os.path.join(HERE, "golden_matrix_a.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
