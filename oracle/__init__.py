"""TEST INFRASTRUCTURE ONLY -- ctypes bindings of the CPU oracle (liblz_oracle.so)
and of the reference's own host code compiled in place (oracle/_ref).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package, and only as the checker / the CPU baseline; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(ORACLE_DIR, "liblz_oracle.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")
REFERENCE_SRC = "/root/reference/source"

_lib = None
_c_i64, _c_int, _c_dbl, _c_vp = ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_void_p


def build() -> None:
    """Compile the oracle (and oracle/_ref when /root/reference is present)."""
    out = subprocess.run(["make", "-C", ORACLE_DIR], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(ORACLE_LIB)
        sig = {
            "lzo_num_threads": (_c_int, []),
            "lzo_set_num_threads": (None, [_c_int]),
            "lzo_csr_spmm": (None, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_int]),
            "lzo_csr_spmm_f32": (None, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_i64, _c_vp, _c_i64]),
            "lzo_sym_eig": (_c_int, [_c_int, _c_vp, _c_vp, _c_vp]),
            "lzo_sqrtm_pair": (_c_int, [_c_int, _c_vp, _c_vp, _c_vp]),
            "lzo_block_lanczos": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_block_lanczos_f32": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_block_lanczos_final": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp, _c_vp,
                                                 _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_block_lanczos_final_f32": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp,
                                                     _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_vector_lanczos": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_vector_lanczos_f32": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_vp, _c_vp, _c_vp,
                                                _c_vp]),
            "lzo_assemble_T": (None, [_c_int, _c_int, _c_vp, _c_vp, _c_vp]),
            "lzo_ritz_values": (_c_int, [_c_int, _c_int, _c_vp, _c_vp, _c_vp]),
            "lzo_block_solution": (_c_int, [_c_int, _c_int, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_fdtd_block": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_i64, _c_dbl, _c_i64, _c_vp]),
            "lzo_block_lanczos_timed": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp, _c_vp,
                                                 _c_vp, _c_vp, _c_vp]),
            "lzo_block_lanczos_f32_timed": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64, _c_vp,
                                                     _c_vp, _c_vp, _c_vp, _c_vp]),
            "lzo_vector_lanczos_timed": (_c_int, [_c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_vp, _c_vp, _c_vp,
                                                  _c_vp, _c_vp]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_c_vp)


def _csr(A):
    return (np.ascontiguousarray(A.row_ptr, np.int64), np.ascontiguousarray(A.col, np.int32),
            np.ascontiguousarray(A.val))


def set_threads(n: int) -> None:
    lib().lzo_set_num_threads(n)


def num_threads() -> int:
    return lib().lzo_num_threads()


def csr_spmm(A, X: np.ndarray) -> np.ndarray:
    rp, col, val = _csr(A)
    X = np.ascontiguousarray(X)
    if X.ndim == 1:
        X = X[:, None]
    b = X.shape[1]
    Y = np.empty((A.n, b), X.dtype)
    if X.dtype == np.float32:
        lib().lzo_csr_spmm_f32(A.n, _p(rp), _p(col), _p(val.astype(np.float32)), b, _p(X), b, _p(Y), b)
    else:
        lib().lzo_csr_spmm(A.n, _p(rp), _p(col), _p(val.astype(np.float64)), b, _p(X), b, _p(Y), b, 0)
    return Y


def sqrtm_pair(G: np.ndarray):
    G = np.ascontiguousarray(G, np.float64)
    b = G.shape[0]
    s, si = np.empty_like(G), np.empty_like(G)
    lib().lzo_sqrtm_pair(b, _p(G), _p(s), _p(si))
    return s, si


def block_lanczos(A, B: np.ndarray, m: int, lc: int):
    """block_lanczos_blas restated; returns (q[m*b], alpha[m,b,b], beta[m+1,b,b])."""
    rp, col, val = _csr(A)
    B = np.ascontiguousarray(B)
    n, b = B.shape
    dt = B.dtype
    q = np.zeros(m * b, dt)
    alpha = np.zeros((m, b, b), dt)
    beta = np.zeros((m + 1, b, b), dt)
    if dt == np.float32:
        rc = lib().lzo_block_lanczos_f32(n, _p(rp), _p(col), _p(val.astype(np.float32)), b, m, lc, _p(B),
                                         _p(q), _p(alpha), _p(beta))
    else:
        rc = lib().lzo_block_lanczos(n, _p(rp), _p(col), _p(val.astype(np.float64)), b, m, lc, _p(B),
                                     _p(q), _p(alpha), _p(beta))
    if rc:
        raise RuntimeError(f"lzo_block_lanczos rc={rc}")
    return q, alpha, beta


def block_lanczos_final(A, B: np.ndarray, m: int, lc: int):
    """block_lanczos plus the final Q0 (= Q1 = Q_{m-1}) and W (last residual)
    the reference leaves in its arguments: (q, alpha, beta, Qf, Wf)."""
    rp, col, val = _csr(A)
    B = np.ascontiguousarray(B)
    n, b = B.shape
    dt = B.dtype
    q = np.zeros(m * b, dt)
    alpha = np.zeros((m, b, b), dt)
    beta = np.zeros((m + 1, b, b), dt)
    Qf = np.zeros((n, b), dt)
    Wf = np.zeros((n, b), dt)
    if dt == np.float32:
        rc = lib().lzo_block_lanczos_final_f32(n, _p(rp), _p(col), _p(val.astype(np.float32)), b, m, lc, _p(B),
                                               _p(q), _p(alpha), _p(beta), _p(Qf), _p(Wf))
    else:
        rc = lib().lzo_block_lanczos_final(n, _p(rp), _p(col), _p(val.astype(np.float64)), b, m, lc, _p(B),
                                           _p(q), _p(alpha), _p(beta), _p(Qf), _p(Wf))
    if rc:
        raise RuntimeError(f"lzo_block_lanczos_final rc={rc}")
    return q, alpha, beta, Qf, Wf


def vector_lanczos(A, bvec: np.ndarray, m: int, lc: int):
    """vector_lanczos restated; fp32 when bvec is float32 (returns float32 arrays)."""
    rp, col, val = _csr(A)
    f32 = np.asarray(bvec).dtype == np.float32
    dt = np.float32 if f32 else np.float64
    bvec = np.ascontiguousarray(bvec, dt).ravel()
    q, alpha, beta = np.zeros(m, dt), np.zeros(m, dt), np.zeros(m, dt)
    fn = lib().lzo_vector_lanczos_f32 if f32 else lib().lzo_vector_lanczos
    fn(A.n, _p(rp), _p(col), _p(val.astype(dt)), m, lc, _p(bvec), _p(q), _p(alpha), _p(beta))
    return q, alpha, beta


def assemble_T(m, b, alpha, beta):
    T = np.empty((m * b, m * b))
    lib().lzo_assemble_T(m, b, _p(np.ascontiguousarray(alpha, np.float64)),
                         _p(np.ascontiguousarray(beta, np.float64)), _p(T))
    return T


def ritz_values(m, b, alpha, beta):
    r = np.empty(m * b)
    lib().lzo_ritz_values(m, b, _p(np.ascontiguousarray(alpha, np.float64)),
                          _p(np.ascontiguousarray(beta, np.float64)), _p(r))
    return r


def block_solution(m, b, T_end, alpha, beta, q):
    s = np.empty(b)
    lib().lzo_block_solution(m, b, T_end, _p(np.ascontiguousarray(alpha, np.float64)),
                             _p(np.ascontiguousarray(beta, np.float64)),
                             _p(np.ascontiguousarray(q, np.float64)), _p(s))
    return s


def fdtd_block(A, B, steps, T_end, lc):
    rp, col, val = _csr(A)
    B = np.ascontiguousarray(B, np.float64)
    out = np.empty(B.shape[1])
    lib().lzo_fdtd_block(A.n, _p(rp), _p(col), _p(val.astype(np.float64)), B.shape[1], _p(B), steps,
                         T_end, lc, _p(out))
    return out


def block_lanczos_timed(A, B: np.ndarray, m: int, lc: int):
    """block_lanczos restated, with the wall seconds of each iteration j = 1..m-1
    (the start-up step untimed): (q, alpha, beta, t_each[m-1]).  fp32 when B is
    float32."""
    rp, col, val = _csr(A)
    f32 = np.asarray(B).dtype == np.float32
    dt = np.float32 if f32 else np.float64
    B = np.ascontiguousarray(B, dt)
    n, b = B.shape
    q = np.zeros(m * b, dt)
    alpha = np.zeros((m, b, b), dt)
    beta = np.zeros((m + 1, b, b), dt)
    t = np.zeros(max(m - 1, 1))
    fn = lib().lzo_block_lanczos_f32_timed if f32 else lib().lzo_block_lanczos_timed
    rc = fn(n, _p(rp), _p(col), _p(val.astype(dt, copy=False)), b, m, lc, _p(B), _p(q), _p(alpha), _p(beta), _p(t))
    if rc:
        raise RuntimeError(f"lzo_block_lanczos_timed rc={rc}")
    return q, alpha, beta, t[: m - 1]


def vector_lanczos_timed(A, bvec: np.ndarray, m: int, lc: int):
    """vector_lanczos restated (fp64) with the wall seconds of each iteration j = 1..m-1."""
    rp, col, val = _csr(A)
    bvec = np.ascontiguousarray(bvec, np.float64).ravel()
    q, alpha, beta = np.zeros(m), np.zeros(m), np.zeros(m)
    t = np.zeros(max(m - 1, 1))
    rc = lib().lzo_vector_lanczos_timed(A.n, _p(rp), _p(col), _p(val.astype(np.float64, copy=False)), m, lc,
                                        _p(bvec), _p(q), _p(alpha), _p(beta), _p(t))
    if rc:
        raise RuntimeError(f"lzo_vector_lanczos_timed rc={rc}")
    return q, alpha, beta, t[: m - 1]


def csr_spmm_timed(A, X: np.ndarray, reps: int = 3):
    """(Y, best seconds) of `reps` oracle SpMMs Y = A X (OpenMP over rows; X row-major)."""
    import time
    rp, col, val = _csr(A)
    X = np.ascontiguousarray(X)
    b = X.shape[1]
    f32 = X.dtype == np.float32
    v = val.astype(np.float32 if f32 else np.float64, copy=False)
    Y = np.empty((A.n, b), X.dtype)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        if f32:
            lib().lzo_csr_spmm_f32(A.n, _p(rp), _p(col), _p(v), b, _p(X), b, _p(Y), b)
        else:
            lib().lzo_csr_spmm(A.n, _p(rp), _p(col), _p(v), b, _p(X), b, _p(Y), b, 0)
        best = min(best, time.perf_counter() - t0)
    return Y, best


# ------------------------------------------------- reference host code (_ref)
_ref = {}


def ref_available(ncol: int = 4) -> bool:
    return os.path.exists(os.path.join(REF_DIR, f"libref_N{ncol}.so"))


def ref_lib(ncol: int = 4):
    if ncol not in _ref:
        L = ctypes.CDLL(os.path.join(REF_DIR, f"libref_N{ncol}.so"))
        _ref[ncol] = L
    return _ref[ncol]


def ref_matrix_a(N: int, change_order: bool = False, ncol: int = 4):
    """The reference's own Matrix_A + mult_diagonal (+ host change_order(4)).
    Returns (n, data, idx) in the reference's layout."""
    L = ref_lib(ncol)
    n, s, w = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
    getattr(L, f"ref_matrix_a_shape_N{ncol}")(N, ctypes.byref(n), ctypes.byref(s), ctypes.byref(w))
    d = np.empty(s.value)
    ix = np.empty(s.value, np.uint32)
    getattr(L, f"ref_matrix_a_N{ncol}")(N, int(change_order), _p(d), _p(ix))
    return n.value, d, ix


def ref_random_B(n: int, ncol: int = 4) -> np.ndarray:
    """random_matrix_B after the lc draw, column-major flat (n*ncol)."""
    out = np.empty(n * ncol)
    getattr(ref_lib(ncol), f"ref_random_B_N{ncol}")(n, _p(out))
    return out


def ref_lc(ncol: int = 4) -> int:
    f = getattr(ref_lib(ncol), f"ref_lc_N{ncol}")
    f.restype = ctypes.c_uint
    return int(f())


def ref_ell_spmm(n, data, idx, X_colmajor, ncol: int = 4):
    Y = np.empty(n * ncol)
    f = getattr(ref_lib(ncol), f"ref_ell_spmm_N{ncol}")
    f.argtypes = [ctypes.c_ulonglong, ctypes.c_ulonglong, _c_vp, _c_vp, _c_vp, _c_vp]
    f(n, data.size, _p(np.ascontiguousarray(data)), _p(np.ascontiguousarray(idx, np.uint32)),
      _p(np.ascontiguousarray(X_colmajor)), _p(Y))
    return Y
