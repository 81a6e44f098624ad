/* include/lz_host.h -- C ABI of liblz_host.so: the host-side logic around the
 * GPU hot path (no GPU calls; runs anywhere).  Problem generation, formats,
 * the small dense post-processing of the Lanczos outputs, and the row
 * partition of the multi-GPU path.  All arrays are HOST memory.
 */
#ifndef LZ_HOST_H
#define LZ_HOST_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------- generators */
/* Deterministic symmetric "banded-random" CSR: strict upper
 * triangle with k_r in {floor(h), ceil(h)}, h = (nnz_per_row-1)/2 entries per row
 * at distinct offsets 1..halfwidth right of the diagonal (clipped at n), values
 * uniform in (-1,1), mirrored, plus a diagonal entry uniform in (-1,1).
 * splitmix64 keyed on (seed, row) -- identical on every host and thread count.
 * Two phases: *_count fills row_ptr[n+1] (and returns nnz), *_fill fills
 * col/val (val64 or val32 may be NULL).  Columns sorted within a row. */
int64_t lzh_gen_banded_count(int64_t n, double nnz_per_row, int64_t halfwidth, uint64_t seed,
                             int64_t *row_ptr);
int lzh_gen_banded_fill(int64_t n, double nnz_per_row, int64_t halfwidth, uint64_t seed,
                        const int64_t *row_ptr, int32_t *col, double *val64, float *val32);
/* Rows [r0, r1) of the same matrix (row_ptr[r1-r0+1] local, GLOBAL column
 * indices), generated without the other rows: the slab of one rank. */
int64_t lzh_gen_banded_local_count(int64_t n, double nnz_per_row, int64_t halfwidth, uint64_t seed,
                                   int64_t r0, int64_t r1, int64_t *row_ptr);
int lzh_gen_banded_local_fill(int64_t n, double nnz_per_row, int64_t halfwidth, uint64_t seed,
                              int64_t r0, int64_t r1, const int64_t *row_ptr, int32_t *col,
                              double *val64, float *val32);

/* Power-law-degree symmetric CSR (BASELINE config 5): upper-triangle count per
 * row k_r = min(cap, floor(xmin * U^(-1/a))), columns uniform in (r, n),
 * mirrored; xmin chosen so the mean row length is ~nnz_per_row. */
int64_t lzh_gen_powerlaw_count(int64_t n, double nnz_per_row, double a, int64_t cap, uint64_t seed,
                               int64_t *row_ptr);
int lzh_gen_powerlaw_fill(int64_t n, double nnz_per_row, double a, int64_t cap, uint64_t seed,
                          const int64_t *row_ptr, int32_t *col, double *val64, float *val32);

/* The reference's Yee-grid operator A = D*W for grid size N (matrix_a/
 * build_A_ell.hpp:8-255 + Ell_matrix::mult_diagonal, objects/ell_matrix.hpp:
 * 340-361), restated: n = 3N(N+1)(2N+1) rows.  bug_compat = 1 applies the
 * reference's host change_order(4) as it actually runs (objects/
 * ell_matrix.hpp:389 keeps ELL slot 0 only).  Returns the ELL arrays in the
 * reference's column-major slot order (slot s of row r at r + s*n), width 4.
 * *_shape gives n and the slot count (= 4n). */
int lzh_matrix_a_shape(int N, int64_t *n_rows, int64_t *slots);
int lzh_matrix_a_ell(int N, int bug_compat, double *data, uint32_t *idx);

/* ELL (column-major slots, width w) -> CSR.  keep_zeros = 0 drops explicit
 * zeros (ELL padding).  Two phases like the generators. */
int64_t lzh_ell_to_csr_count(int64_t n, int64_t width, const double *data, const uint32_t *idx,
                             int keep_zeros, int64_t *row_ptr);
int lzh_ell_to_csr_fill(int64_t n, int64_t width, const double *data, const uint32_t *idx,
                        int keep_zeros, const int64_t *row_ptr, int32_t *col, double *val);

/* glibc rand() stream (TYPE_3 additive feedback, srand(seed)), restated so B
 * is reproducible without libc: out[i] = (double)rand()/RAND_MAX + 1 for the
 * draws after the first `skip` ones (random_matrix_B, matrix_a/build_ell_utils.hpp:
 * 271-280, with skip = 1 for the lc draw of test_lanczos.cu:326).  The i-th
 * value is B's column-major element i (row i % n, column i / n); row_major = 1
 * writes it to out[(i % n) * b + i / n]. */
int lzh_rand_B(int64_t n, int b, uint32_t seed, int64_t skip, int row_major, double *out);
/* first lc of the reference driver: 1 + rand() % 100 after srand(seed) */
int64_t lzh_rand_lc(uint32_t seed);
/* uniform [1,2) start block from splitmix64 (row-major n x b) */
int lzh_uniform_B(int64_t n, int b, uint64_t seed, double *out64, float *out32);
/* rows [r0, r0 + n) of the same block (one rank's slab of the global start block) */
int lzh_uniform_B_rows(int64_t r0, int64_t n, int b, uint64_t seed, double *o64, float *o32);

/* ------------------------------------------------------ post-processing */
/* symmetric eigen-decomposition: Householder tridiagonalisation + implicit QL.
 * A k x k row-major (lower triangle read); eval ascending; evec column i =
 * eigenvector i (NULL: values only). */
int lzh_sym_eig(int k, const double *A, double *eval, double *evec);
/* T = Assemble_T(m, alpha, beta) (objects/tridiagonal_matrix.hpp:90-126):
 * alpha_j diagonal blocks, beta_j above (block row j-1, block col j), beta_j^T
 * below.  (m*b)^2 row-major. */
int lzh_assemble_T(int m, int b, const double *alpha, const double *beta, double *T);
/* Ritz values = ascending eigenvalues of T */
int lzh_ritz_values(int m, int b, const double *alpha, const double *beta, double *ritz);
/* solution = (expm(T_end T)[:, :b] beta_0)^T q  (test_lanczos.cu:272-286) */
int lzh_block_solution(int m, int b, double T_end, const double *alpha, const double *beta,
                       const double *q, double *solution);

/* --------------------------------------------------------- partition */
/* contiguous row blocks with ~equal nnz: bounds[0]=0 .. bounds[p]=n */
int lzh_partition_rows(int64_t n, const int64_t *row_ptr, int parts, int64_t *bounds);
/* global column j -> padded numbering (owner p = the part holding row j):
 * p*n_pad + (j - bounds[p]) -- the row of X_full the all-gather puts it in. */
int lzh_remap_cols_padded(int64_t nnz, const int32_t *col, int parts, const int64_t *bounds,
                          int64_t n_pad, int32_t *col_out);
/* Halo plan of part `rank` for lz_block_lanczos_halo: halo_rows[0..n_halo) =
 * the distinct global columns outside [bounds[rank], bounds[rank+1]) that the
 * local CSR references, ascending (hence grouped by owner part in part order);
 * recv_counts[p] = how many of them part p owns; col_out = the columns in the
 * compact numbering (own row j -> j - bounds[rank], halo_rows[i] -> n_local+i).
 * halo_rows needs room for nnz entries.  Returns n_halo, < 0 on error. */
int64_t lzh_halo_plan(int64_t nnz, const int32_t *col, int parts, const int64_t *bounds, int rank,
                      int32_t *col_out, int64_t *recv_counts, int32_t *halo_rows);

/* ---------------------------------------------------------- CSR files */
/* binary CSR: "LZCSR001", int64 n_rows, n_cols, nnz, int32 dtype (0 f64, 1 f32),
 * int32 0, row_ptr[n+1] int64, col[nnz] int32, val[nnz]. */
int lzh_csr_write(const char *path, int64_t n_rows, int64_t n_cols, int64_t nnz,
                  const int64_t *row_ptr, const int32_t *col, const void *val, int dtype);
int lzh_csr_read_header(const char *path, int64_t *n_rows, int64_t *n_cols, int64_t *nnz,
                        int *dtype);
int lzh_csr_read(const char *path, int64_t *row_ptr, int32_t *col, void *val);

int lzh_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
