// lz_internal.hpp -- internal (C++) entry points between the .hip units.
#pragma once
#include "lz_common.hpp"

namespace lz {

// ---- sparse (lz_spmm.hip)
template <typename T>
int spmm_rm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy);  // nx: rows of X
template <typename T>
int spmm_cm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, T *Y, int64_t ldy);
template <typename T>
int spmv(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, const T *x,
         T *y, int64_t nnz_hint);

// ---- dense (lz_dense.hip)
// partial b x b products of X^T Y, one slab per workgroup, into h->partials;
// returns the number of slabs in *nparts.
template <typename T>
int gram_partials(lz_handle *h, int64_t n, int b, const T *X, const T *Y, int64_t ld, int *nparts);
// reduce nparts slabs (fixed order); mode 0: R = sum, mode 1: R = 0.5 (S + S^T)
template <typename T>
int gram_finish(lz_handle *h, int b, int nparts, int mode, T *R, const double *slabs = nullptr);
// symmetric square root pair of G (device double b x b) or, when nparts > 0,
// of the sum of the nparts slabs in h->partials.
template <typename T>
int sqrtm_pair(lz_handle *h, int b, const T *G, int nparts, T *beta, T *beta_inv, T *eig,
               const double *slabs = nullptr);
// W = sw*W + sq*Q*S
template <typename T>
int tsmm(lz_handle *h, int64_t n, int b, T sw, T sq, const T *Q, const T *S, T *W, int64_t ld);
template <typename T>
int copy_row(lz_handle *h, int b, const T *Q, int64_t ld, int col_major, int64_t lc, T *q);

// ---- fused block-Lanczos passes, b = 16 fp64 (lz_fused.hip)
// Pass 1: Y = A*Wg; Qbuf[r] <- Wg[r]*binv (after reading Qbuf[r] when beta
// != nullptr); Wn[r] = Y[r]*binv - Qprev[r]*beta; slabs of Qbuf^T Wn; row probe.
// nx: rows of Wg.  Wown: the rows r of Wg this rank owns (== Wg single-GPU; a slice of the
// all-gathered block multi-GPU).
int fused_spmm16(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col,
                 const double *val, const double *Wg, int64_t nx, const double *Wown, double *Qbuf, double *Wn,
                 const double *binv, const double *beta, int64_t lc, double *qrow, int *nparts);
// Pass 2: Wn <- Wn - Q*alpha; slabs of Wn^T Wn.
int fused_update16(lz_handle *h, int64_t n, double *Wn, const double *Q, const double *alpha,
                   int *nparts);

// fp64 scalar helpers for the vector Lanczos (lz_fused.hip)
int vector_lanczos_dev(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                       const double *val, int m, int64_t lc, const double *b, double *q,
                       double *alpha, double *beta, double *q0, double *q1, double *w);

}  // namespace lz
