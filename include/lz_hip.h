/* include/lz_hip.h -- C ABI of liblz_hip.so, the MI355X (gfx950) Lanczos hot path.
 *
 * Drop-in boundary for the reference's header-only operator API
 * (ibrohimmn1994/GPU-implementation-of-signle-and-block-Lanczos, paths relative
 * to source/).  Each entry point names the reference interface it replaces.
 *
 * Conventions (all entry points):
 *   - return 0 on success, a negative LZ_E* code on failure; lz_last_error()
 *     gives a message (thread-local).  No exceptions cross the ABI.
 *   - every array argument is a DEVICE pointer owned by the caller unless the
 *     comment says "host"; sizes are element counts.
 *   - work is enqueued on the handle's stream (lz_set_stream; default: the
 *     legacy null stream) and is asynchronous unless stated otherwise.  Some
 *     solves fork internal streams of the handle (the b = 32 sqrtm beside the
 *     next SpMM, the long-tile SpMM pass beside the tile pass, a distributed
 *     rank's exchange) and join them back into the handle's stream by events
 *     before the call returns: callers order against the handle's stream only.
 *   - sparse operator: CSR, int64 row_ptr[n_rows+1], int32 col[nnz], values in
 *     `dtype`.  Dense blocks ("tall-skinny", n x b) are ROW-MAJOR with leading
 *     dimension ld >= b (element (r,c) at r*ld + c) unless a layout argument says
 *     LZ_COL_MAJOR (the reference's Dense_matrix layout, element at r + c*ld).
 *   - b x b matrices (alpha, beta, S) are row-major b*b; every one the Lanczos
 *     iteration produces is symmetric, so they equal the reference's
 *     column-major storage element for element.
 */
#ifndef LZ_HIP_H
#define LZ_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { LZ_F64 = 0, LZ_F32 = 1 } lz_dtype;
typedef enum { LZ_ROW_MAJOR = 0, LZ_COL_MAJOR = 1 } lz_layout;

enum {
    LZ_OK = 0,
    LZ_E_ARG = -1,      /* invalid argument (shape, null pointer, unsupported b/dtype) */
    LZ_E_HIP = -2,      /* HIP runtime error (includes "no device") */
    LZ_E_COMM = -3,     /* RCCL error */
    LZ_E_STATE = -4,    /* handle not initialised / wrong call order */
    LZ_E_DEVICE = -5    /* a persistent kernel abandoned a bounded wait (lz_device_error
                           gives its code); the call's results are invalid */
};

typedef struct lz_handle lz_handle;  /* opaque */

/* ---------------------------------------------------------------- runtime */
/* Replaces the implicit CUDA context + cublasCreate/initiate_cusolver of the
 * driver (test_lanczos.cu:224-236, utils/lib_utils.hpp:777-805).  Allocates the
 * handle's small device workspace (partial sums, b x b scratch). */
int lz_init(int device, lz_handle **h);
int lz_finalize(lz_handle *h);
int lz_set_stream(lz_handle *h, void *hip_stream);
/* 1 (default): lz_block_lanczos / lz_block_lanczos_unfused leave Q0, Q1, W as
 * the reference does (see lz_block_lanczos); 0: they are scratch on return. */
int lz_set_final_state(lz_handle *h, int on);
const char *lz_last_error(void);
const char *lz_version(void);
/* 1 when a gfx950 device is visible and the code object loads on it. */
int lz_device_ok(int device);

/* Per-kernel-class timing with hipEvents recorded on the handle's stream
 * around every launch of the class (no host synchronisation; read after the
 * work).  Classes: 0 fused SpMM pass, 1 fused update pass, 2 one-workgroup
 * finish/sqrtm kernels, 3 Gram slabs, 4 tall x small products, 5 plain SpMM.
 * lz_prof_enable resets the record (capacity 4096 launches). */
/* Synchronises the handle's stream and returns (then clears) the device error
 * word: nonzero if a persistent kernel abandoned a bounded spin-wait (its
 * results are then invalid).  0 in normal operation.  Every solve that checks
 * the word (lz_block_lanczos at b = 16 fp64, the distributed solves) clears it
 * on its stream when it starts, so a word left by an earlier call never fails a
 * later solve; a solve that fails with LZ_E_DEVICE leaves its word readable
 * here. */
int lz_device_error(lz_handle *h, int *code);
/* Test support: store `code` into the device error word (on the handle's
 * stream), as a kernel that gave up a wait would. */
int lz_debug_set_device_error(lz_handle *h, int code);
/* Test support: the handle's next distributed solve (lz_block_lanczos_dist /
 * _halo) fails its set-up with status `code` (nonzero) on this rank only; the
 * rank still joins the solve's first collective (the ranks' set-up vote), so
 * every peer returns LZ_E_STATE instead of waiting. */
int lz_debug_fail_next_setup(lz_handle *h, int code);

/* Test support: fills the LDS of every CU with a 32-bit pattern (0xFFFFFFFF
 * reads back as a double NaN), and the handle's slab and scratch workspaces
 * with its low byte, on the handle's stream, so a kernel that reads LDS or
 * workspace it did not write shows it deterministically instead of by chance. */
int lz_debug_poison_lds(lz_handle *h, uint32_t pattern);
/* (LZ_POISON=1 in the environment: lz_init fills the new handle's workspaces with 0xFF.) */

int lz_prof_enable(lz_handle *h, int on);
/* As lz_prof_enable, recording only the classes whose bit is set in
 * class_mask (1 << class; 0 = off).  Each recorded launch adds two event
 * records to the stream (~3.5 us per launch on MI355X), so a timed run records
 * only the class it reports. */
int lz_prof_enable_mask(lz_handle *h, unsigned class_mask);
int lz_prof_read(lz_handle *h, int kernel_class, double *ms_total, int *count);

/* ----------------------------------------------------------- sparse kernels */
/* Y = A*X with b columns.  Replaces spmm(Ell_matrix<T>&, Dense_matrix<T>&,
 * Dense_matrix<T>&) (kernels/spmv_spmm.hpp:262-333, kernel :137-199) and,
 * at b == 1, spmv(Ell_matrix<T>&, Vector<T>&, Vector<T>&) (:209-260, kernel
 * :105-135).  Row-major X/Y: b in {1,2,4,8,16,32,64}; column-major: any b<=64.
 * X has n_cols rows, Y has n_rows rows. */
int lz_csr_spmm(lz_handle *h, int64_t n_rows, int64_t n_cols, int64_t nnz,
                const int64_t *row_ptr, const int32_t *col, const void *val, lz_dtype dtype,
                int b, const void *X, int64_t ldx, lz_layout layout, void *Y, int64_t ldy);

/* Y (rows x b, row-major, ld = b) = X (rows x b, COLUMN-major, leading
 * dimension ldx >= rows: the reference's Dense_matrix storage,
 * objects/dense_matrix.hpp:9, whose ld is the row count padded to a multiple of
 * 768, test_lanczos.cu:174-187).  One pass through LDS (coalesced column reads
 * and row writes); lz_methods.hpp uses it to take the reference's column-major
 * start block into the row-major iteration once. */
int lz_to_row_major(lz_handle *h, int64_t rows, int b, lz_dtype dtype, const void *X, int64_t ldx, void *Y);

/* The inverse: Y (rows x b, COLUMN-major, leading dimension ldy >= rows) = X
 * (rows x b, row-major, ld = b).  lz_methods.hpp uses it to hand the final
 * Q0 / Q1 / W blocks back in the caller's column-major layout. */
int lz_to_col_major(lz_handle *h, int64_t rows, int b, lz_dtype dtype, const void *X, void *Y, int64_t ldy);

/* y = A*x  (spmv, kernels/spmv_spmm.hpp:209-260) */
int lz_csr_spmv(lz_handle *h, int64_t n_rows, int64_t n_cols, int64_t nnz,
                const int64_t *row_ptr, const int32_t *col, const void *val, lz_dtype dtype,
                const void *x, void *y);

/* ------------------------------------------------ tall-skinny dense kernels */
/* R = W^T W  (b x b, written to device R).  Replaces mm_tt_cublas
 * (utils/lib_utils.hpp:102-123) / tt::mm_tt (kernels/mm_tt.hpp:5-179).
 * Deterministic (fixed-order two-stage reduction, no float atomics). */
int lz_gram(lz_handle *h, int64_t n, int b, lz_dtype dtype, const void *W, int64_t ld, void *R);

/* R = 0.5 (W^T Q + Q^T W).  Replaces mm_tt2_cublas (lib_utils.hpp:164-202) /
 * tt2::mm_tt2 (kernels/mm_tt2.hpp:14-210). */
int lz_sym_cross_gram(lz_handle *h, int64_t n, int b, lz_dtype dtype, const void *W,
                      const void *Q, int64_t ld, void *R);

/* W = beta*W + alpha*Q*S  (S b x b device).  Replaces mm_cublas(beta, alpha, Q,
 * S, W) (lib_utils.hpp:28-51) / ts::mm_ts1, mm_ts2 (kernels/mm_ts.hpp:5-273).
 * beta == 0 never reads W (W may alias nothing; Q must not alias W). */
int lz_tsmm(lz_handle *h, int64_t n, int b, lz_dtype dtype, double beta, double alpha,
            const void *Q, const void *S, void *W, int64_t ld);

/* beta <- V sqrt|L| V^T, beta_inv <- V |L|^-1/2 V^T for the symmetric b x b G
 * (lower triangle read).  Replaces sqrtm_cusolver = cusolverDn{D,S}syevjBatched
 * + custom_mult2 (lib_utils.hpp:649-745) and sqrtm::My_sqrtm_cusolver
 * (kernels/my_sqrtm_cusolver.hpp:174-376).  One workgroup, parallel Jacobi.
 * G may alias beta.  b <= 32.  eigval (device, may be NULL) receives the
 * ascending eigenvalues of G. */
int lz_sqrtm_pair(lz_handle *h, int b, lz_dtype dtype, const void *G, void *beta,
                  void *beta_inv, void *eigval);

/* q[start + c] = Q(lc, c), c < b.  Replaces copy_row_to_vector
 * (methods/copy_functions.hpp:10-57). */
int lz_copy_row(lz_handle *h, int b, lz_dtype dtype, const void *Q, int64_t ld, lz_layout layout,
                int64_t lc, void *q, int64_t start);

/* ------------------------------------------------------------------ methods */
/* m steps of block Lanczos with symmetric-sqrtm normalisation, no
 * re-orthogonalisation.  Replaces block_lanczos_blas<T>(A, B, m, lc, q, alpha,
 * beta, Q0, Q1, W, args, eigen_val, cublasH, n_blocks, n_loads)
 * (methods/block_lanczos.hpp:88-167); same outputs:
 *   q[m*b]          row lc of Q_0..Q_{m-1}
 *   alpha[m*b*b]    alpha_j
 *   beta[(m+1)*b*b] beta_0 = sqrtm(B^T B), beta_j (j=1..m-1), beta_m = last inverse sqrt
 * B, Q0, Q1, W: n x b row-major (ld = b), device.  B is read only.  Q0/Q1/W
 * are workspace during the call (the reference passes them pre-set to B; their
 * input content is ignored here) and on return hold what the reference leaves
 * in them (block_lanczos.hpp:145,159,162): Q0 = Q1 = Q_{m-1} (the last
 * normalised Krylov block; Q1 is not written when m = 1) and W = the last
 * residual A Q_{m-1} - Q_{m-2} beta_{m-1} - Q_{m-1} alpha_{m-1} (unnormalised).
 * That costs one row-local pass per call; lz_set_final_state(h, 0) skips it
 * for callers that never read the three blocks (they are then scratch).
 * Fused device-resident iteration: no host synchronisation inside the steps;
 * every output stays on the device.  Before the first step one value is read
 * back (one host synchronisation): the b = 16 fp64 wavefront step's plan, the
 * b = 32 fp32 SpMM's stage choice.  At b = 16 fp64 the call also ends with
 * one, to read the device error word of the step kernels (LZ_E_DEVICE when one
 * of them abandoned a bounded wait).
 * The b = 16 fp64 step kernels keep one workgroup on every CU and their
 * workgroups wait on each other's progress: the launch is checked for
 * co-residency, and no kernel that itself waits on the solve's results may
 * run beside it on the device. */
int lz_block_lanczos(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr,
                     const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                     int64_t lc, const void *B, void *q, void *alpha, void *beta, void *Q0,
                     void *Q1, void *W);

/* Same iteration, reference op order with separate (unfused) kernels: the
 * structure of block_lanczos_blas one call per line.  For A/B measurement and
 * as a second GPU path for parity. */
int lz_block_lanczos_unfused(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr,
                             const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                             int64_t lc, const void *B, void *q, void *alpha, void *beta,
                             void *Q0, void *Q1, void *W);

/* Single-vector Lanczos.  Replaces vector_lanczos<T>(A, b, m, lc, q, alpha,
 * beta, q0, q1, w) (methods/vector_lanczos.hpp:8-67; the correct variant -- the
 * BLAS variant's axpy at :116 is a reference bug not reproduced).  alpha[m],
 * beta[m] are DEVICE arrays here (the reference keeps host arrays; copy them
 * back with one hipMemcpy after the call).  beta[0] = ||b||.  fp64 or fp32
 * (test_lanczos.cu:355 instantiates test_VectorLanczos<float>): fp32 storage,
 * SpMV products and sums in fp32, the dot/norm reductions accumulated in fp64
 * and rounded to fp32. */
int lz_vector_lanczos(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr,
                      const int32_t *col, const void *val, lz_dtype dtype, int m, int64_t lc,
                      const void *bvec, void *q, void *alpha, void *beta, void *q0, void *q1,
                      void *w);

/* Forward-Euler validation run U += dt*A*U, Nsteps times, then out[c] = U(lc,c).
 * Replaces ftdt_block (methods/fdtd.hpp:33-56).  U0 n x b row-major; U, D are
 * n x b buffers (U receives the final state, D is scratch).  Up to 2^18 rows each
 * step is one fused kernel (U and D ping-pong); the step loop is replayed from a
 * captured hipGraph of 256 steps (LZ_FDTD_GRAPH=0: launch every step). */
int lz_fdtd_block(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr,
                  const int32_t *col, const void *val, lz_dtype dtype, int b, const void *U0,
                  int64_t steps, double T_end, int64_t lc, void *U, void *D, void *out);

/* ------------------------------------------------------------ multi-GPU (RCCL)
 * Row-partitioned block Lanczos: rank g owns rows [row0, row0 + n_local) of A
 * and of every Krylov block.  New in this build (the reference is single-GPU).
 * lz_comm_unique_id fills 128 bytes on rank 0; the caller broadcasts them (any
 * transport) and every rank calls lz_comm_init. */
int lz_comm_unique_id(unsigned char out[128]);
int lz_comm_init(lz_handle *h, int nranks, int rank, const unsigned char id[128]);
int lz_comm_destroy(lz_handle *h);

/* Virtual ranks: an N-rank decomposition driven from ONE process on one
 * device, one host thread and one stream per rank (test and rehearsal
 * support; the reference has no multi-GPU code to mirror).  Every rank's
 * handle attaches to the group with lz_comm_init_local and then calls the
 * same entry points an RCCL rank calls (lz_halo_init, lz_block_lanczos_halo,
 * lz_block_lanczos_dist); the collectives meet at a host barrier and move
 * data with device copies on the calling rank's stream, ordered by events.
 * A rank that fails calls lz_comm_abort (or lz_local_group_abort) so that the
 * others return LZ_E_COMM instead of waiting; a barrier also gives up after
 * LZ_LOCAL_TIMEOUT_S seconds (default 300).  The group's state lives until
 * the last attached handle is finalized. */
typedef struct lz_local_group lz_local_group;  /* opaque */
int lz_local_group_create(int device, int nranks, lz_local_group **g);
int lz_local_group_destroy(lz_local_group *g);
int lz_local_group_abort(lz_local_group *g);
int lz_comm_init_local(lz_handle *h, lz_local_group *g, int rank);
/* Wake every rank of h's group blocked in a collective (local groups), or
 * ncclCommAbort h's RCCL communicator.  A distributed solve that fails after
 * issuing a collective does this itself.  An aborted RCCL communicator stays
 * unusable (every later collective returns LZ_E_COMM): lz_comm_destroy, then
 * lz_comm_init with a new unique id.  RCCL peers blocked in a collective with
 * an aborted rank return only once they abort too (or poll the communicator's
 * async error). */
int lz_comm_abort(lz_handle *h);
/* Test support: the interior row range [out[0], out[1]) whose pass 1 ran
 * beside the exchange in the handle's last distributed solve ({-1, -1}: the
 * solve ran unsplit). */
int lz_debug_last_split(lz_handle *h, int64_t out[2]);
/* Test support: out[0] = 1 when the handle's last distributed solve ran the
 * wavefront step (b = 16 fp64), out[1] = 1 when it also ran the requested rows'
 * pass 2 first and the halo exchange beside the rest of each step. */
int lz_debug_last_wf(lz_handle *h, int out[2]);

/* Test hook: the wavefront step's once-per-solve plan of a CSR operator (device
 * arrays), as lz_block_lanczos would make it for these rows. deps_out (device,
 * 2 * T int32: each tile's [lo, hi] pass-2 tile range) and col16_out (device,
 * nnz int16: pass 1's strip-relative columns) receive the plan's arrays; info
 * (host): [0] plan applies, [1] 16-bit columns valid, [2] T tiles, [3] rows per
 * tile, [4..7] the span words (max back / forward reach, max width, range
 * flags). nx, xoff: gather-source rows and the row of local row 0 (n, 0 on one
 * GPU). deps_out and info[4..7] are this call's plan whenever the plan kernel
 * ran (info[0] = 1: it also applies), zero otherwise; col16_out is this call's
 * 16-bit columns when info[1] = 1, zero otherwise. Never a stale earlier plan. */
int lz_debug_wf_plan(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr, const int32_t *col_idx,
                     int64_t nx, int64_t xoff, int32_t *deps_out, int16_t *col16_out, int32_t info[8]);

/* Distributed block Lanczos, all-gather form (the north star's exchange).
 * Every rank's slab is padded to n_pad rows (n_pad >= max rows per rank) and
 * ncclAllGather places rank g's slab at rows [g*n_pad, (g+1)*n_pad) of X_full,
 * so:
 *   - A_local: the rank's n_local rows in CSR whose columns are in the PADDED
 *     numbering (global row r of rank g -> g*n_pad + (r - row0_g); host helper
 *     lzh_remap_cols_padded of include/lz_host.h);
 *   - X_full: n_global x b row-major workspace with n_global == n_pad * nranks
 *     (checked), holding the all-gathered residual every iteration; the rank's
 *     own slot is where its residual is updated, so the all-gather is in place;
 *   - B_local, W: n_pad x b (rows past n_local are zero padding); W holds the
 *     previous residual W_{j-1}; Q0 and Q1 unused (may be NULL).
 * Any 1 <= b <= 32 (b = 1 is the single-vector recurrence,
 * methods/vector_lanczos.hpp:8-67, with alpha[m] / beta[m+1] scalars), fp64 or
 * fp32: b = 16 fp64 runs the fused passes, other shapes the SpMM plus the
 * fused dense passes.  Rows that reference only the rank's own rows run
 * their pass 1 (SpMM) while the all-gather is in flight on the handle's
 * exchange stream; the rest follow it (LZ_DIST_OVERLAP=0: exchange first).
 * lc_rank: the rank owning row lc (q written there only; other ranks' q
 * untouched).  Outputs alpha/beta identical on every rank.  Gather sources of
 * 2^24+ rows take the windowed fused pass (each strip's columns within 2^23
 * rows of its own padded row), else the 64-bit addressed one. */
int lz_block_lanczos_dist(lz_handle *h, int64_t n_local, int64_t n_pad, int64_t n_global,
                          int64_t nnz_local, const int64_t *row_ptr, const int32_t *col,
                          const void *val, lz_dtype dtype, int b, int m, int64_t lc_local,
                          int lc_rank, const void *B_local, void *q, void *alpha, void *beta,
                          void *Q0, void *Q1, void *W, void *X_full);

/* Halo-exchange variant: only the rows of other ranks that the
 * local CSR references move each step (grouped ncclSend/ncclRecv), instead of
 * the all-gather of every rank's slab.  Collective setup, every rank:
 *   lzh_halo_plan (liblz_host) on the local CSR with GLOBAL columns gives the
 *   compact columns, recv_counts[nranks] and halo_rows[n_halo] (host arrays);
 *   lz_halo_init(h, row0, n_local, recv_counts, halo_rows) exchanges the
 *   request lists over RCCL and keeps the send lists on the device.
 * A rank's Krylov blocks then live in X buffers of n_local + n_halo rows:
 * rows [0, n_local) its own, the rest the halo in plan order.  With one rank
 * (or no communicator) n_halo = 0 and no collective is issued. */
int lz_halo_init(lz_handle *h, int64_t row0, int64_t n_local, const int64_t *recv_counts,
                 const int32_t *halo_rows);
int lz_halo_sizes(lz_handle *h, int64_t *n_halo, int64_t *n_send);
/* fill rows [n_local, n_local + n_halo) of X (b columns, row-major, ld = b)
 * from their owners; rows [0, n_local) must hold this rank's block */
int lz_halo_exchange(lz_handle *h, lz_dtype dtype, int b, void *X);
/* Distributed block Lanczos over the halo plan; replaces the single-GPU
 * block_lanczos_blas (methods/block_lanczos.hpp:88-167) on a row partition.
 * col: compact numbering from lzh_halo_plan.  B_local: n_local x b; X0, X1:
 * (n_local + n_halo) x b workspaces (the residual alternates between them).
 * alpha/beta identical on every rank; q written on lc_rank only.  Shapes and
 * the interior / boundary overlap as lz_block_lanczos_dist. */
int lz_block_lanczos_halo(lz_handle *h, int64_t n_local, int64_t nnz_local, const int64_t *row_ptr,
                          const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                          int64_t lc_local, int lc_rank, const void *B_local, void *q, void *alpha,
                          void *beta, void *X0, void *X1);

#ifdef __cplusplus
}
#endif
#endif
