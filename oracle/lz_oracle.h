/* oracle/lz_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's hot path (block / single-vector
 * Lanczos on a sparse operator), used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker.  The product (liblz_hip.so) never
 * links, loads or calls anything in this directory.
 *
 * Conventions: CSR with int64 row_ptr, int32 col; Krylov blocks are row-major
 * n x b (element (r,c) at r*ld + c); every b x b matrix (alpha, beta) is
 * row-major b*b.  The reference stores them column-major, but every one of
 * them is symmetric, so the two layouts hold the same numbers.
 *
 * Pinning: see oracle/README in DESIGN.md -- the restatement is checked against
 * the reference's own host code compiled in place (oracle/_ref, matrix_a,
 * random_matrix_B, Ell_matrix::spmm) and against an independent numpy
 * restatement on the reference's matrix_a operator (tests/test_oracle.py).
 */
#ifndef LZ_ORACLE_H
#define LZ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* number of OpenMP threads the oracle uses (1 when built without OpenMP) */
int lzo_num_threads(void);
void lzo_set_num_threads(int n);

/* Y = A*X, b columns.  col_major=0: X[r*ldx+c]; col_major=1: X[r + c*ldx].
 * Restates ell::SpMM (kernels/spmv_spmm.hpp:137-199) / Ell_matrix::spmm
 * (objects/ell_matrix.hpp:287-300) on CSR. */
void lzo_csr_spmm(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                  int b, const double *X, int64_t ldx, double *Y, int64_t ldy, int col_major);
void lzo_csr_spmm_f32(int64_t n, const int64_t *row_ptr, const int32_t *col, const float *val,
                      int b, const float *X, int64_t ldx, float *Y, int64_t ldy);

/* symmetric eigen-decomposition by cyclic Jacobi: A (k x k row-major) ->
 * eval[k] ascending, evec (k x k row-major, column i = eigenvector i). */
int lzo_sym_eig(int k, const double *A, double *eval, double *evec);

/* beta <- V sqrt|L| V^T, beta_inv <- V |L|^-1/2 V^T of the symmetric G.
 * Restates sqrtm_cusolver + custom_mult2 (utils/lib_utils.hpp:649-745). */
int lzo_sqrtm_pair(int b, const double *G, double *beta, double *beta_inv);

/* block_lanczos_blas (methods/block_lanczos.hpp:88-167) in reference op order.
 * B: n x b row-major start block.  Outputs: q[m*b] (row lc of each Q_j),
 * alpha[m*b*b], beta[(m+1)*b*b] (beta[0..m-1] as the reference stores them;
 * beta[m] = last inverse square root).  Workspace allocated internally. */
int lzo_block_lanczos(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                      int b, int m, int64_t lc, const double *B,
                      double *q, double *alpha, double *beta);

/* Same, fp32 arithmetic (for the C5 fp32 configuration). */
int lzo_block_lanczos_f32(int64_t n, const int64_t *row_ptr, const int32_t *col,
                          const float *val, int b, int m, int64_t lc, const float *B,
                          float *q, float *alpha, float *beta);

/* lzo_block_lanczos plus the blocks the reference leaves in its arguments on
 * return (block_lanczos.hpp:159,162): Qf = Q0 = Q1 = Q_{m-1}, Wf = W (the last
 * residual, unnormalised); n x b row-major each.  fp64 and fp32. */
int lzo_block_lanczos_final(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                            int b, int m, int64_t lc, const double *B, double *q, double *alpha,
                            double *beta, double *Qf, double *Wf);
int lzo_block_lanczos_final_f32(int64_t n, const int64_t *row_ptr, const int32_t *col, const float *val,
                                int b, int m, int64_t lc, const float *B, float *q, float *alpha,
                                float *beta, float *Qf, float *Wf);

/* vector_lanczos (methods/vector_lanczos.hpp:8-67, the correct variant).
 * q[m], alpha[m], beta[m] (beta[0] = ||b||). */
int lzo_vector_lanczos(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                       int m, int64_t lc, const double *bvec,
                       double *q, double *alpha, double *beta);
/* the same at T = float (test_lanczos.cu:355); reductions accumulated in double. */
int lzo_vector_lanczos_f32(int64_t n, const int64_t *row_ptr, const int32_t *col, const float *val,
                           int m, int64_t lc, const float *bvec, float *q, float *alpha, float *beta);

/* T = Assemble_T(m, alpha, beta) (objects/tridiagonal_matrix.hpp:90-126, device
 * path): alpha_j on the diagonal, beta_j above (rows j-1, cols j) and beta_j^T
 * below.  T is (m*b) x (m*b) row-major. */
void lzo_assemble_T(int m, int b, const double *alpha, const double *beta, double *T);

/* Ritz values: ascending eigenvalues of T (the `eigen_val` of expm_cusolver,
 * utils/lib_utils.hpp:547-577). */
int lzo_ritz_values(int m, int b, const double *alpha, const double *beta, double *ritz);

/* solution = (expm(T_end*T)[:, :b] * beta[0])^T q   (test_lanczos.cu:272-286). */
int lzo_block_solution(int m, int b, double T_end, const double *alpha, const double *beta,
                       const double *q, double *solution);

/* Forward Euler U += dt*A*U, returns row lc (methods/fdtd.hpp:33-56). */
int lzo_fdtd_block(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                   int b, const double *B, int64_t steps, double T_end, int64_t lc,
                   double *out);

/* lzo_block_lanczos with per-iteration wall times: t_each[j - 1] = seconds of
 * iteration j (j = 1..m-1; the start-up step is not timed).  bench.py's CPU
 * baseline (best of the timed iterations) and its parity field (q/alpha/beta
 * of the same run against the GPU's) both come from one call. */
int lzo_block_lanczos_timed(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val,
                            int b, int m, int64_t lc, const double *B, double *q, double *alpha,
                            double *beta, double *t_each);

/* The single-vector and the fp32 block iterations with the wall seconds of
 * each iteration j = 1..m-1 (bench.py's CPU baselines at configs C2 and C5). */
int lzo_vector_lanczos_timed(int64_t n, const int64_t *row_ptr, const int32_t *col, const double *val, int m,
                             int64_t lc, const double *bvec, double *q, double *alpha, double *beta, double *t_each);
int lzo_block_lanczos_f32_timed(int64_t n, const int64_t *row_ptr, const int32_t *col, const float *val, int b,
                                int m, int64_t lc, const float *B, float *q, float *alpha, float *beta,
                                double *t_each);

#ifdef __cplusplus
}
#endif

#endif
