"""MI355X (gfx950) single- and block-Lanczos -- Python host mirror of the C ABI.

The product is two in-tree shared libraries built by ``make`` in this directory:

* ``lib/liblz_hip.so``  -- the gfx950 kernels and the Lanczos iteration behind the
  extern "C" boundary declared in ``include/lz_hip.h``;
* ``lib/liblz_host.so`` -- host logic (generators, formats, post-processing) from
  ``include/lz_host.h``.

This module binds both with ctypes and mirrors the reference's operator API
(ibrohimmn1994/GPU-implementation-of-signle-and-block-Lanczos, paths relative to
``source/``): ``spmm`` / ``spmv`` (kernels/spmv_spmm.hpp:209-333),
``mm_tt`` / ``mm_tt2`` / ``mm_ts`` (utils/lib_utils.hpp:28-202), ``sqrtm``
(lib_utils.hpp:721-745), ``block_lanczos_blas`` (methods/block_lanczos.hpp:88-167),
``vector_lanczos`` (methods/vector_lanczos.hpp:8-67), ``ftdt_block``
(methods/fdtd.hpp:33-56), ``Assemble_T`` + Ritz values + ``solution``
(test_lanczos.cu:272-286).  Device memory, streams and torch.distributed come
from PyTorch (plumbing only); every computation runs in liblz_hip.so.  There is
no CPU fallback: a GPU entry point raises if the HIP library cannot be loaded or
no gfx950 device is present.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
# LZ_HIP_LIB: another build of the same library (A/B of kernel versions in scripts/)
HIP_LIB = os.environ.get("LZ_HIP_LIB") or os.path.join(LIB_DIR, "liblz_hip.so")
HOST_LIB = os.path.join(LIB_DIR, "liblz_host.so")

LZ_F64, LZ_F32 = 0, 1
LZ_ROW_MAJOR, LZ_COL_MAJOR = 0, 1

_c_i64, _c_i32, _c_int, _c_dbl, _c_vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_int, ctypes.c_double, ctypes.c_void_p
_c_u32, _c_u64 = ctypes.c_uint32, ctypes.c_uint64


class LanczosError(RuntimeError):
    """Raised for a non-zero status from liblz_hip.so / liblz_host.so."""


# --------------------------------------------------------------- library load
_hip = None
_host = None

# (name, restype, argtypes) of every symbol in include/lz_hip.h
HIP_SYMBOLS = [
    ("lz_init", _c_int, [_c_int, ctypes.POINTER(_c_vp)]),
    ("lz_finalize", _c_int, [_c_vp]),
    ("lz_set_stream", _c_int, [_c_vp, _c_vp]),
    ("lz_set_final_state", _c_int, [_c_vp, _c_int]),
    ("lz_last_error", ctypes.c_char_p, []),
    ("lz_version", ctypes.c_char_p, []),
    ("lz_device_ok", _c_int, [_c_int]),
    ("lz_device_error", _c_int, [_c_vp, ctypes.POINTER(_c_int)]),
    ("lz_debug_poison_lds", _c_int, [_c_vp, ctypes.c_uint32]),
    ("lz_debug_set_device_error", _c_int, [_c_vp, _c_int]),
    ("lz_debug_fail_next_setup", _c_int, [_c_vp, _c_int]),
    ("lz_prof_enable", _c_int, [_c_vp, _c_int]),
    ("lz_prof_enable_mask", _c_int, [_c_vp, ctypes.c_uint]),
    ("lz_prof_read", _c_int, [_c_vp, _c_int, ctypes.POINTER(_c_dbl), ctypes.POINTER(_c_int)]),
    ("lz_csr_spmm", _c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int,
                             _c_vp, _c_i64, _c_int, _c_vp, _c_i64]),
    ("lz_to_row_major", _c_int, [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_i64, _c_vp]),
    ("lz_to_col_major", _c_int, [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_i64]),
    ("lz_csr_spmv", _c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp]),
    ("lz_gram", _c_int, [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_i64, _c_vp]),
    ("lz_sym_cross_gram", _c_int, [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_i64, _c_vp]),
    ("lz_tsmm", _c_int, [_c_vp, _c_i64, _c_int, _c_int, _c_dbl, _c_dbl, _c_vp, _c_vp, _c_vp, _c_i64]),
    ("lz_sqrtm_pair", _c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lz_copy_row", _c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_i64, _c_int, _c_i64, _c_vp, _c_i64]),
    ("lz_block_lanczos", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                                  _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lz_block_lanczos_unfused", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int,
                                          _c_int, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lz_vector_lanczos", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_i64,
                                   _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lz_fdtd_block", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp,
                               _c_i64, _c_dbl, _c_i64, _c_vp, _c_vp, _c_vp]),
    ("lz_comm_unique_id", _c_int, [_c_vp]),
    ("lz_comm_init", _c_int, [_c_vp, _c_int, _c_int, _c_vp]),
    ("lz_halo_init", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp]),
    ("lz_halo_sizes", _c_int, [_c_vp, _c_vp, _c_vp]),
    ("lz_halo_exchange", _c_int, [_c_vp, _c_int, _c_int, _c_vp]),
    ("lz_block_lanczos_halo", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int,
                                       _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lz_comm_destroy", _c_int, [_c_vp]),
    ("lz_local_group_create", _c_int, [_c_int, _c_int, ctypes.POINTER(_c_vp)]),
    ("lz_local_group_destroy", _c_int, [_c_vp]),
    ("lz_local_group_abort", _c_int, [_c_vp]),
    ("lz_comm_init_local", _c_int, [_c_vp, _c_vp, _c_int]),
    ("lz_comm_abort", _c_int, [_c_vp]),
    ("lz_debug_last_split", _c_int, [_c_vp, _c_vp]),
    ("lz_debug_last_wf", _c_int, [_c_vp, ctypes.POINTER(_c_int)]),
    ("lz_debug_wf_plan", _c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp,
                                  ctypes.POINTER(_c_int)]),
    ("lz_block_lanczos_dist", _c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp,
                                       _c_int, _c_int, _c_int, _c_i64, _c_int, _c_vp, _c_vp, _c_vp,
                                       _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
]

HOST_SYMBOLS = [
    ("lzh_gen_banded_count", _c_i64, [_c_i64, _c_dbl, _c_i64, _c_u64, _c_vp]),
    ("lzh_gen_banded_fill", _c_int, [_c_i64, _c_dbl, _c_i64, _c_u64, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lzh_gen_banded_local_count", _c_i64, [_c_i64, _c_dbl, _c_i64, _c_u64, _c_i64, _c_i64, _c_vp]),
    ("lzh_gen_banded_local_fill", _c_int, [_c_i64, _c_dbl, _c_i64, _c_u64, _c_i64, _c_i64, _c_vp, _c_vp,
                                           _c_vp, _c_vp]),
    ("lzh_gen_powerlaw_count", _c_i64, [_c_i64, _c_dbl, _c_dbl, _c_i64, _c_u64, _c_vp]),
    ("lzh_gen_powerlaw_fill", _c_int, [_c_i64, _c_dbl, _c_dbl, _c_i64, _c_u64, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lzh_matrix_a_shape", _c_int, [_c_int, _c_vp, _c_vp]),
    ("lzh_matrix_a_ell", _c_int, [_c_int, _c_int, _c_vp, _c_vp]),
    ("lzh_ell_to_csr_count", _c_i64, [_c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp]),
    ("lzh_ell_to_csr_fill", _c_int, [_c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    ("lzh_rand_B", _c_int, [_c_i64, _c_int, _c_u32, _c_i64, _c_int, _c_vp]),
    ("lzh_rand_lc", _c_i64, [_c_u32]),
    ("lzh_uniform_B", _c_int, [_c_i64, _c_int, _c_u64, _c_vp, _c_vp]),
    ("lzh_uniform_B_rows", _c_int, [_c_i64, _c_i64, _c_int, _c_u64, _c_vp, _c_vp]),
    ("lzh_sym_eig", _c_int, [_c_int, _c_vp, _c_vp, _c_vp]),
    ("lzh_assemble_T", _c_int, [_c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    ("lzh_ritz_values", _c_int, [_c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    ("lzh_block_solution", _c_int, [_c_int, _c_int, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lzh_partition_rows", _c_int, [_c_i64, _c_vp, _c_int, _c_vp]),
    ("lzh_remap_cols_padded", _c_int, [_c_i64, _c_vp, _c_int, _c_vp, _c_i64, _c_vp]),
    ("lzh_halo_plan", _c_i64, [_c_i64, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    ("lzh_csr_write", _c_int, [ctypes.c_char_p, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int]),
    ("lzh_csr_read_header", _c_int, [ctypes.c_char_p, _c_vp, _c_vp, _c_vp, _c_vp]),
    ("lzh_csr_read", _c_int, [ctypes.c_char_p, _c_vp, _c_vp, _c_vp]),
    ("lzh_num_threads", _c_int, []),
]


def _bind(lib, symbols, strict=True):
    for name, res, args in symbols:
        if not strict and not hasattr(lib, name):
            continue  # (an older build loaded through LZ_HIP_LIB for an A/B: only what it has)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def build(verbose: bool = False) -> None:
    """Compile liblz_hip.so (hipcc --offload-arch=gfx950), liblz_host.so and test_lanczos in-tree."""
    import subprocess
    jobs = str(min(16, os.cpu_count() or 4))
    out = subprocess.run(["make", "-C", PKG_DIR, "-j", jobs], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise LanczosError("build failed:\n" + (out.stdout or "") + (out.stderr or ""))


def host_lib():
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise LanczosError(f"{HOST_LIB} missing: run make in {PKG_DIR}")
        _host = _bind(ctypes.CDLL(HOST_LIB), HOST_SYMBOLS)
    return _host


def hip_lib():
    """liblz_hip.so with every symbol of include/lz_hip.h bound (loads without a GPU)."""
    global _hip
    if _hip is None:
        if not os.path.exists(HIP_LIB):
            raise LanczosError(f"{HIP_LIB} missing: run make in {PKG_DIR}")
        # PyTorch bundles its own HIP runtime / RCCL under the same SONAMEs
        # (libamdhip64.so.7, librccl.so.1).  Import it first so the dynamic
        # loader resolves liblz_hip.so's dependencies to the copies already in
        # the process: one HIP runtime per process, shared with torch's
        # allocator and streams.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _hip = _bind(ctypes.CDLL(HIP_LIB), HIP_SYMBOLS, strict=not os.environ.get("LZ_HIP_LIB"))
    return _hip


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = hip_lib().lz_last_error().decode(errors="replace") if _hip is not None else ""
        raise LanczosError(f"{what} failed with status {rc}: {msg}")


def _p(a: np.ndarray):
    return a.ctypes.data_as(_c_vp)


# ============================================================ host helpers
@dataclass
class CsrHost:
    """CSR on the host: int64 row_ptr, int32 col, float64/float32 val."""
    n: int
    row_ptr: np.ndarray
    col: np.ndarray
    val: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1])


def gen_banded(n: int, nnz_per_row: float = 10.0, halfwidth: int = 4096, seed: int = 20261015,
               dtype=np.float64) -> CsrHost:
    """Symmetric banded-random CSR."""
    L = host_lib()
    rp = np.empty(n + 1, np.int64)
    nnz = L.lzh_gen_banded_count(n, nnz_per_row, halfwidth, seed, _p(rp))
    if nnz < 0:
        raise LanczosError("lzh_gen_banded_count failed")
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, dtype)
    v64 = _p(val) if dtype == np.float64 else None
    v32 = _p(val) if dtype == np.float32 else None
    if L.lzh_gen_banded_fill(n, nnz_per_row, halfwidth, seed, _p(rp), _p(col), v64, v32):
        raise LanczosError("lzh_gen_banded_fill failed")
    return CsrHost(n, rp, col, val)


def gen_banded_local(n: int, r0: int, r1: int, nnz_per_row: float = 10.0, halfwidth: int = 4096,
                     seed: int = 20261015, dtype=np.float64) -> CsrHost:
    """Rows [r0, r1) of gen_banded(n, ...) with global column indices (one rank's slab)."""
    L = host_lib()
    nl = r1 - r0
    rp = np.empty(nl + 1, np.int64)
    nnz = L.lzh_gen_banded_local_count(n, nnz_per_row, halfwidth, seed, r0, r1, _p(rp))
    if nnz < 0:
        raise LanczosError("lzh_gen_banded_local_count failed")
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, dtype)
    v64 = _p(val) if dtype == np.float64 else None
    v32 = _p(val) if dtype == np.float32 else None
    if L.lzh_gen_banded_local_fill(n, nnz_per_row, halfwidth, seed, r0, r1, _p(rp), _p(col), v64, v32):
        raise LanczosError("lzh_gen_banded_local_fill failed")
    return CsrHost(nl, rp, col, val)


def gen_powerlaw(n: int, nnz_per_row: float = 10.0, a: float = 2.1, cap: int = 100000,
                 seed: int = 20261015, dtype=np.float32) -> CsrHost:
    """Symmetric power-law-degree CSR (config C5)."""
    L = host_lib()
    rp = np.empty(n + 1, np.int64)
    nnz = L.lzh_gen_powerlaw_count(n, nnz_per_row, a, cap, seed, _p(rp))
    if nnz < 0:
        raise LanczosError("lzh_gen_powerlaw_count failed")
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, dtype)
    v64 = _p(val) if dtype == np.float64 else None
    v32 = _p(val) if dtype == np.float32 else None
    if L.lzh_gen_powerlaw_fill(n, nnz_per_row, a, cap, seed, _p(rp), _p(col), v64, v32):
        raise LanczosError("lzh_gen_powerlaw_fill failed")
    return CsrHost(n, rp, col, val)


def matrix_a_ell(N: int, bug_compat: bool = False):
    """The reference's Yee operator A = D*W as ELL (column-major slots, width 4)."""
    L = host_lib()
    n, s = _c_i64(), _c_i64()
    L.lzh_matrix_a_shape(N, ctypes.byref(n), ctypes.byref(s))
    d = np.empty(s.value, np.float64)
    ix = np.empty(s.value, np.uint32)
    if L.lzh_matrix_a_ell(N, int(bug_compat), _p(d), _p(ix)):
        raise LanczosError("lzh_matrix_a_ell failed")
    return n.value, d, ix


def ell_to_csr(n: int, width: int, data: np.ndarray, idx: np.ndarray, keep_zeros: bool = False) -> CsrHost:
    L = host_lib()
    data = np.ascontiguousarray(data, np.float64)
    idx = np.ascontiguousarray(idx, np.uint32)
    rp = np.empty(n + 1, np.int64)
    nnz = L.lzh_ell_to_csr_count(n, width, _p(data), _p(idx), int(keep_zeros), _p(rp))
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, np.float64)
    L.lzh_ell_to_csr_fill(n, width, _p(data), _p(idx), int(keep_zeros), _p(rp), _p(col), _p(val))
    return CsrHost(n, rp, col, val)


def matrix_a(N: int, bug_compat: bool = False) -> CsrHost:
    """Matrix_A<double>(N,N,N) + mult_diagonal (+ the as-run change_order) as CSR."""
    n, d, ix = matrix_a_ell(N, bug_compat)
    return ell_to_csr(n, 4, d, ix)


def rand_B(n: int, b: int, seed: int = 1, skip: int = 1, row_major: bool = True) -> np.ndarray:
    """random_matrix_B from the glibc rand() stream (after the lc draw)."""
    out = np.empty(n * b, np.float64)
    if host_lib().lzh_rand_B(n, b, seed, skip, int(row_major), _p(out)):
        raise LanczosError("lzh_rand_B failed")
    return out.reshape(n, b) if row_major else out.reshape(b, n).T


def rand_lc(seed: int = 1) -> int:
    return int(host_lib().lzh_rand_lc(seed))


def uniform_B(n: int, b: int, seed: int = 20261015, dtype=np.float64, r0: int = 0) -> np.ndarray:
    """Start block, uniform [1, 2) per row from a counter-based stream: rows
    [r0, r0 + n) of the global block (a rank's slab)."""
    out = np.empty((n, b), dtype)
    L = host_lib()
    if dtype == np.float64:
        L.lzh_uniform_B_rows(r0, n, b, seed, _p(out), None)
    else:
        L.lzh_uniform_B_rows(r0, n, b, seed, None, _p(out))
    return out


def sym_eig(A: np.ndarray, vectors: bool = False):
    A = np.ascontiguousarray(A, np.float64)
    k = A.shape[0]
    ev = np.empty(k)
    V = np.empty((k, k)) if vectors else None
    host_lib().lzh_sym_eig(k, _p(A), _p(ev), _p(V) if vectors else None)
    return (ev, V) if vectors else ev


def Assemble_T(m: int, b: int, alpha: np.ndarray, beta: np.ndarray) -> np.ndarray:
    T = np.empty((m * b, m * b))
    host_lib().lzh_assemble_T(m, b, _p(np.ascontiguousarray(alpha, np.float64)),
                              _p(np.ascontiguousarray(beta, np.float64)), _p(T))
    return T


def ritz_values(m: int, b: int, alpha: np.ndarray, beta: np.ndarray) -> np.ndarray:
    r = np.empty(m * b)
    host_lib().lzh_ritz_values(m, b, _p(np.ascontiguousarray(alpha, np.float64)),
                               _p(np.ascontiguousarray(beta, np.float64)), _p(r))
    return r


def block_solution(m: int, b: int, T_end: float, alpha, beta, q) -> np.ndarray:
    s = np.empty(b)
    host_lib().lzh_block_solution(m, b, T_end, _p(np.ascontiguousarray(alpha, np.float64)),
                                  _p(np.ascontiguousarray(beta, np.float64)),
                                  _p(np.ascontiguousarray(q, np.float64)), _p(s))
    return s


def partition_rows(A: CsrHost, parts: int) -> np.ndarray:
    bounds = np.empty(parts + 1, np.int64)
    host_lib().lzh_partition_rows(A.n, _p(A.row_ptr), parts, _p(bounds))
    return bounds


def remap_cols_padded(col: np.ndarray, bounds: np.ndarray, n_pad: int) -> np.ndarray:
    col = np.ascontiguousarray(col, np.int32)
    out = np.empty_like(col)
    rc = host_lib().lzh_remap_cols_padded(col.size, _p(col), bounds.size - 1,
                                          _p(np.ascontiguousarray(bounds, np.int64)), n_pad, _p(out))
    if rc:
        raise LanczosError("lzh_remap_cols_padded failed")
    return out


def halo_plan(col: np.ndarray, bounds: np.ndarray, rank: int):
    """lzh_halo_plan: (compact columns, recv_counts[parts], halo_rows[n_halo]) for part
    `rank` of the row partition `bounds` (columns global on input)."""
    col = np.ascontiguousarray(col, np.int32)
    bounds = np.ascontiguousarray(bounds, np.int64)
    parts = bounds.size - 1
    out = np.empty_like(col)
    counts = np.zeros(parts, np.int64)
    rows = np.empty(max(col.size, 1), np.int32)
    nh = host_lib().lzh_halo_plan(col.size, _p(col), parts, _p(bounds), rank, _p(out), _p(counts), _p(rows))
    if nh < 0:
        raise LanczosError(f"lzh_halo_plan failed ({nh})")
    return out, counts, rows[:nh].copy()


def csr_write(path: str, A: CsrHost) -> None:
    dt = 0 if A.val.dtype == np.float64 else 1
    if host_lib().lzh_csr_write(path.encode(), A.n, A.n, A.nnz, _p(A.row_ptr), _p(A.col), _p(A.val), dt):
        raise LanczosError("lzh_csr_write failed")


def csr_read(path: str) -> CsrHost:
    L = host_lib()
    n, nc, nnz, dt = _c_i64(), _c_i64(), _c_i64(), _c_int()
    if L.lzh_csr_read_header(path.encode(), ctypes.byref(n), ctypes.byref(nc), ctypes.byref(nnz), ctypes.byref(dt)):
        raise LanczosError("bad CSR file")
    rp = np.empty(n.value + 1, np.int64)
    col = np.empty(nnz.value, np.int32)
    val = np.empty(nnz.value, np.float64 if dt.value == 0 else np.float32)
    if L.lzh_csr_read(path.encode(), _p(rp), _p(col), _p(val)):
        raise LanczosError("CSR read failed")
    return CsrHost(n.value, rp, col, val)


# ============================================================= GPU (torch)
def _torch():
    import torch  # plumbing: device memory + streams
    return torch


def _ld(t) -> int:
    """Leading dimension of a 2-D tensor (stride of a size-1 dim is arbitrary)."""
    if t.shape[1] > 1 and t.stride(1) != 1:
        raise LanczosError("inner dimension must be contiguous")
    return t.stride(0) if t.shape[0] > 1 else t.shape[1]


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _dt(t) -> int:
    torch = _torch()
    if t.dtype == torch.float64:
        return LZ_F64
    if t.dtype == torch.float32:
        return LZ_F32
    raise LanczosError(f"unsupported dtype {t.dtype}")


@dataclass
class CsrDevice:
    """CSR operator resident in HBM (torch tensors on cuda)."""
    n: int
    n_cols: int
    row_ptr: "object"
    col: "object"
    val: "object"

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @property
    def dtype(self) -> int:
        return _dt(self.val)

    @staticmethod
    def from_host(A: CsrHost, device="cuda", n_cols: Optional[int] = None) -> "CsrDevice":
        torch = _torch()
        return CsrDevice(A.n, A.n if n_cols is None else n_cols,
                         torch.from_numpy(A.row_ptr).to(device),
                         torch.from_numpy(A.col).to(device),
                         torch.from_numpy(A.val).to(device))


class Handle:
    """lz_handle on one device, bound to torch's current stream at each call."""

    def __init__(self, device: int = 0):
        L = hip_lib()
        if not L.lz_device_ok(device):
            raise LanczosError(f"no gfx950 device {device} visible to liblz_hip.so")
        h = _c_vp()
        _check(L.lz_init(device, ctypes.byref(h)), "lz_init")
        self._h = h
        self.device = device
        self.L = L

    def close(self):
        if self._h:
            self.L.lz_finalize(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync_stream(self):
        torch = _torch()
        s = torch.cuda.current_stream(self.device).cuda_stream
        _check(self.L.lz_set_stream(self._h, _c_vp(s)), "lz_set_stream")

    @property
    def ptr(self):
        self._sync_stream()
        return self._h

    # --- operator API (reference names) -------------------------------
    def spmm(self, A: CsrDevice, X, Y, layout: int = LZ_ROW_MAJOR):
        """Y = A*X (kernels/spmv_spmm.hpp:262-333). X/Y (rows, b) row-major tensors, or
        column-major (b, rows) tensors viewed transposed when layout=LZ_COL_MAJOR."""
        b = X.shape[1] if layout == LZ_ROW_MAJOR else X.shape[0]
        ldx, ldy = _ld(X), _ld(Y)
        _check(self.L.lz_csr_spmm(self.ptr, A.n, A.n_cols, A.nnz, _ptr(A.row_ptr), _ptr(A.col),
                                  _ptr(A.val), A.dtype, b, _ptr(X), ldx, layout, _ptr(Y), ldy), "lz_csr_spmm")
        return Y

    def to_row_major(self, Xcm, Y):
        """Y (rows, b) row-major <- the column-major block viewed as Xcm (b, ld) (ld >= rows)."""
        b, ld = Xcm.shape
        rows = Y.shape[0]
        _check(self.L.lz_to_row_major(self.ptr, rows, b, _dt(Xcm), _ptr(Xcm), ld, _ptr(Y)), "lz_to_row_major")
        return Y

    def spmv(self, A: CsrDevice, x, y):
        _check(self.L.lz_csr_spmv(self.ptr, A.n, A.n_cols, A.nnz, _ptr(A.row_ptr), _ptr(A.col),
                                  _ptr(A.val), A.dtype, _ptr(x), _ptr(y)), "lz_csr_spmv")
        return y

    def mm_tt(self, W, R):
        """R = W^T W (mm_tt_cublas, utils/lib_utils.hpp:102-123)."""
        n, b = W.shape
        _check(self.L.lz_gram(self.ptr, n, b, _dt(W), _ptr(W), W.stride(0), _ptr(R)), "lz_gram")
        return R

    def mm_tt2(self, W, Q, R):
        """R = 0.5 (W^T Q + Q^T W) (mm_tt2_cublas, lib_utils.hpp:164-202)."""
        n, b = W.shape
        _check(self.L.lz_sym_cross_gram(self.ptr, n, b, _dt(W), _ptr(W), _ptr(Q), W.stride(0), _ptr(R)),
               "lz_sym_cross_gram")
        return R

    def mm_ts(self, beta: float, alpha: float, Q, S, W):
        """W = beta W + alpha Q S (mm_cublas(beta, alpha, Q, S, W), lib_utils.hpp:28-51)."""
        n, b = Q.shape
        _check(self.L.lz_tsmm(self.ptr, n, b, _dt(Q), beta, alpha, _ptr(Q), _ptr(S), _ptr(W), W.stride(0)),
               "lz_tsmm")
        return W

    def sqrtm(self, G, beta, beta_inv, eigval=None):
        """beta = sqrtm(G), beta_inv = inverse (sqrtm_cusolver, lib_utils.hpp:721-745)."""
        b = G.shape[0]
        _check(self.L.lz_sqrtm_pair(self.ptr, b, _dt(G), _ptr(G), _ptr(beta), _ptr(beta_inv), _ptr(eigval)),
               "lz_sqrtm_pair")

    def copy_row_to_vector(self, lc: int, start: int, Q, q):
        n, b = Q.shape
        _check(self.L.lz_copy_row(self.ptr, b, _dt(Q), _ptr(Q), Q.stride(0), LZ_ROW_MAJOR, lc, _ptr(q), start),
               "lz_copy_row")

    def block_lanczos_blas(self, A: CsrDevice, B, m: int, lc: int, q, alpha, beta, Q0, Q1, W,
                           fused: bool = True):
        """block_lanczos_blas (methods/block_lanczos.hpp:88-167).  q[m*b], alpha[m,b,b],
        beta[m+1,b,b] device tensors are written in place."""
        n, b = B.shape
        fn = self.L.lz_block_lanczos if fused else self.L.lz_block_lanczos_unfused
        _check(fn(self.ptr, n, A.nnz, _ptr(A.row_ptr), _ptr(A.col), _ptr(A.val), A.dtype, b, m, lc,
                  _ptr(B), _ptr(q), _ptr(alpha), _ptr(beta), _ptr(Q0), _ptr(Q1), _ptr(W)),
               "lz_block_lanczos")

    def set_final_state(self, on: bool) -> None:
        """True (default): block_lanczos_blas leaves Q0 = Q1 = Q_{m-1} and W = the
        last residual, as the reference does; False: they are scratch on return."""
        _check(self.L.lz_set_final_state(self.ptr, 1 if on else 0), "lz_set_final_state")

    def vector_lanczos(self, A: CsrDevice, bvec, m: int, lc: int, q, alpha, beta, q0, q1, w):
        """vector_lanczos (methods/vector_lanczos.hpp:8-67); alpha/beta are device tensors.
        fp64 or fp32: every vector must have A's element type."""
        n = bvec.shape[0]
        for t in (bvec, q, alpha, beta, q0, q1, w):
            if t.element_size() != (8 if A.dtype == LZ_F64 else 4):
                raise ValueError("vector_lanczos: every vector must have A's element type")
        _check(self.L.lz_vector_lanczos(self.ptr, n, A.nnz, _ptr(A.row_ptr), _ptr(A.col), _ptr(A.val), A.dtype,
                                        m, lc, _ptr(bvec), _ptr(q), _ptr(alpha), _ptr(beta), _ptr(q0),
                                        _ptr(q1), _ptr(w)), "lz_vector_lanczos")

    def ftdt_block(self, A: CsrDevice, U0, steps: int, T_end: float, lc: int, U, D, out):
        n, b = U0.shape
        _check(self.L.lz_fdtd_block(self.ptr, n, A.nnz, _ptr(A.row_ptr), _ptr(A.col), _ptr(A.val), A.dtype, b,
                                    _ptr(U0), steps, T_end, lc, _ptr(U), _ptr(D), _ptr(out)), "lz_fdtd_block")
        return out

    # --- hipEvent timing of kernel classes ------------------------------
    PROF_SPMM_PASS, PROF_UPDATE_PASS, PROF_SMALL, PROF_GRAM, PROF_TSMM, PROF_SPMM = range(6)

    def device_error(self) -> int:
        """Synchronise and return (then clear) the device error word (0 = ok)."""
        c = _c_int()
        _check(self.L.lz_device_error(self._h, ctypes.byref(c)), "lz_device_error")
        return c.value

    def debug_set_device_error(self, code: int):
        """Store `code` into the device error word (test support)."""
        _check(self.L.lz_debug_set_device_error(self.ptr, code), "lz_debug_set_device_error")

    def debug_fail_next_setup(self, code: int = 5):
        """The next distributed solve on this handle fails its set-up with `code`
        on this rank (test support: its peers must return, not wait)."""
        _check(self.L.lz_debug_fail_next_setup(self._h, code), "lz_debug_fail_next_setup")

    def debug_poison_lds(self, pattern: int = 0xFFFFFFFF):
        """Fill every CU's LDS with `pattern` (test support: stale-LDS reads show as NaN)."""
        _check(self.L.lz_debug_poison_lds(self._h, pattern), "lz_debug_poison_lds")

    def prof_enable(self, on: bool = True, classes=None):
        """Record kernel-class timings (all classes, or only `classes`)."""
        if classes is None:
            _check(self.L.lz_prof_enable(self._h, int(on)), "lz_prof_enable")
        else:
            mask = 0
            for c in classes:
                mask |= 1 << int(c)
            _check(self.L.lz_prof_enable_mask(self._h, mask if on else 0), "lz_prof_enable_mask")

    def prof_read(self, cls: int):
        """(total ms, launches) of a kernel class since prof_enable."""
        ms, cnt = _c_dbl(), _c_int()
        _check(self.L.lz_prof_read(self._h, cls, ctypes.byref(ms), ctypes.byref(cnt)), "lz_prof_read")
        return ms.value, cnt.value

    # --- multi-GPU ------------------------------------------------------
    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = ctypes.create_string_buffer(uid, 128)
        _check(self.L.lz_comm_init(self._h, nranks, rank, buf), "lz_comm_init")

    def comm_init_local(self, group: "LocalGroup", rank: int):
        """Attach this handle as virtual rank `rank` of an in-process group (one device)."""
        _check(self.L.lz_comm_init_local(self.ptr, group.ptr, rank), "lz_comm_init_local")
        group._keep.append(self)

    def last_wf(self):
        """(wavefront step, pass-2-first overlap) flags of the last distributed solve."""
        v = (_c_int * 2)()
        _check(self.L.lz_debug_last_wf(self._h, v), "lz_debug_last_wf")
        return bool(v[0]), bool(v[1])

    def wf_plan(self, A, nx=None, xoff=0):
        """The wavefront step's plan of device operator A (test hook): (info dict,
        deps (T, 2) int32 tensor, col16 (nnz,) int16 tensor)."""
        import torch
        T_max = A.n // 16 + 2
        deps = torch.zeros(T_max * 2, dtype=torch.int32, device=A.row_ptr.device)
        c16 = torch.zeros(max(A.nnz, 1), dtype=torch.int16, device=A.row_ptr.device)
        info = (_c_int * 8)()
        _check(self.L.lz_debug_wf_plan(self.ptr, A.n, A.nnz, A.row_ptr.data_ptr(), A.col.data_ptr(),
                                       A.n if nx is None else nx, xoff, deps.data_ptr(), c16.data_ptr(), info),
               "lz_debug_wf_plan")
        T = int(info[2])
        d = {"ok": bool(info[0]), "col16": bool(info[1]), "T": T, "tr": int(info[3]),
             "spans": [int(info[4 + i]) for i in range(4)]}
        return d, deps[: 2 * T].view(T, 2), c16[: A.nnz]

    def last_split(self):
        """(i0, i1) of the last distributed solve's interior rows (pass 1 beside the
        exchange), or None when it ran unsplit."""
        v = (_c_i64 * 2)()
        _check(self.L.lz_debug_last_split(self._h, v), "lz_debug_last_split")
        return None if v[0] < 0 else (int(v[0]), int(v[1]))

    def comm_abort(self):
        _check(self.L.lz_comm_abort(self._h), "lz_comm_abort")

    def comm_destroy(self):
        _check(self.L.lz_comm_destroy(self._h), "lz_comm_destroy")

    def block_lanczos_dist(self, A_local: CsrDevice, n_pad: int, n_global: int, B_local, m: int,
                           lc_local: int, lc_rank: int, q, alpha, beta, Q0, W, X_full):
        n_local, b = A_local.n, B_local.shape[1]
        _check(self.L.lz_block_lanczos_dist(self.ptr, n_local, n_pad, n_global, A_local.nnz,
                                            _ptr(A_local.row_ptr), _ptr(A_local.col), _ptr(A_local.val),
                                            A_local.dtype, b, m, lc_local, lc_rank, _ptr(B_local), _ptr(q),
                                            _ptr(alpha), _ptr(beta), _ptr(Q0), None, _ptr(W), _ptr(X_full)),
               "lz_block_lanczos_dist")


    def halo_init(self, row0: int, n_local: int, recv_counts: np.ndarray, halo_rows: np.ndarray):
        rc = np.ascontiguousarray(recv_counts, np.int64)
        hr = np.ascontiguousarray(halo_rows, np.int32)
        _check(self.L.lz_halo_init(self.ptr, row0, n_local, _p(rc), _p(hr) if hr.size else None),
               "lz_halo_init")

    def halo_sizes(self):
        nh, ns = _c_i64(), _c_i64()
        _check(self.L.lz_halo_sizes(self.ptr, ctypes.byref(nh), ctypes.byref(ns)), "lz_halo_sizes")
        return nh.value, ns.value

    def halo_exchange(self, X):
        _check(self.L.lz_halo_exchange(self.ptr, _dt(X), X.shape[1], _ptr(X)), "lz_halo_exchange")

    def block_lanczos_halo(self, A_local: CsrDevice, B_local, m: int, lc_local: int, lc_rank: int,
                           q, alpha, beta, X0, X1):
        """Distributed block Lanczos over the halo plan (A_local.col in the compact numbering)."""
        n_local, b = A_local.n, B_local.shape[1]
        _check(self.L.lz_block_lanczos_halo(self.ptr, n_local, A_local.nnz, _ptr(A_local.row_ptr),
                                            _ptr(A_local.col), _ptr(A_local.val), A_local.dtype, b, m,
                                            lc_local, lc_rank, _ptr(B_local), _ptr(q), _ptr(alpha),
                                            _ptr(beta), _ptr(X0), _ptr(X1)),
               "lz_block_lanczos_halo")


class LocalGroup:
    """N virtual ranks on one device in this process (lz_local_group_create):
    every rank's Handle attaches with comm_init_local and then runs the same
    distributed entry points an RCCL rank runs, from its own thread."""

    def __init__(self, nranks: int, device: int = 0):
        L = hip_lib()
        g = _c_vp()
        _check(L.lz_local_group_create(device, nranks, ctypes.byref(g)), "lz_local_group_create")
        self.ptr, self.nranks, self.device, self.L = g, nranks, device, L
        self._keep = []

    def abort(self):
        if self.ptr:
            self.L.lz_local_group_abort(self.ptr)

    def close(self):
        if self.ptr:
            self.L.lz_local_group_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_virtual_ranks(nranks: int, fn, device: int = 0, timeout: float = 600.0):
    """Run fn(rank, handle) for ranks 0..nranks-1, each in its own thread with its
    own torch stream and its own lz Handle attached to one LocalGroup.  Inputs
    made before the call are synchronised first; returns the list of results.
    A rank that raises aborts the group, so no other rank waits for it."""
    import threading
    torch = _torch()
    torch.cuda.synchronize(device)
    group = LocalGroup(nranks, device)
    handles = [Handle(device) for _ in range(nranks)]
    # the ranks' streams are made here and outlive every handle (closed below
    # after a device synchronise), so no handle ever refers to a stream whose
    # Python object a finished thread dropped
    streams = [torch.cuda.Stream(device) for _ in range(nranks)]
    out, errs = [None] * nranks, [None] * nranks

    def body(r):
        try:
            with torch.cuda.device(device), torch.cuda.stream(streams[r]):
                handles[r].comm_init_local(group, r)
                out[r] = fn(r, handles[r])
                torch.cuda.current_stream(device).synchronize()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs[r] = e
            group.abort()

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(nranks)]
    try:
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout)
        if any(t.is_alive() for t in threads):
            group.abort()
            for t in threads:
                t.join(30)
        if any(t.is_alive() for t in threads):  # never free what a live thread may still use
            raise LanczosError("virtual ranks did not finish")
    finally:
        if not any(t.is_alive() for t in threads):
            torch.cuda.synchronize(device)
            for h in handles:
                h.close()
            group.close()
            group._keep.clear()
            del streams[:]
    for r, e in enumerate(errs):
        if e is not None:
            raise LanczosError(f"virtual rank {r}: {e}") from e
    return out


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(hip_lib().lz_comm_unique_id(buf), "lz_comm_unique_id")
    return buf.raw


def run_block_lanczos(h: Handle, A: CsrDevice, B, m: int, lc: int, fused: bool = True):
    """Allocate the reference's workspaces and run block_lanczos_blas; returns device
    tensors (q, alpha, beta)."""
    torch = _torch()
    n, b = B.shape
    kw = dict(dtype=B.dtype, device=B.device)
    q = torch.zeros(m * b, **kw)
    alpha = torch.zeros(m, b, b, **kw)
    beta = torch.zeros(m + 1, b, b, **kw)
    Q0, Q1, W = (torch.empty(n, b, **kw) for _ in range(3))
    h.block_lanczos_blas(A, B, m, lc, q, alpha, beta, Q0, Q1, W, fused=fused)
    return q, alpha, beta
