/* oracle/lz_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Lanczos hot path.  Used exclusively by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
 * checker / CPU baseline.  The product (liblz_hip.so) never calls it.
 *
 * Each function cites the reference file:line it restates (paths relative to
 * /root/reference/source).  Pinning: tests/test_oracle.py checks this oracle
 * against the reference's own host code compiled in place (oracle/_ref) and
 * against an independent numpy restatement; golden vectors under tests/golden
 * were produced by tests/golden/make_golden.py.
 */
#include "lz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_threads = 0;

int lzo_num_threads(void)
{
#ifdef _OPENMP
    if (g_threads <= 0) g_threads = omp_get_max_threads();
    return g_threads;
#else
    return 1;
#endif
}

void lzo_set_num_threads(int n)
{
    g_threads = n;
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#endif
}

static double lzo_wtime(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ------------------------------------------------------------------ SpMM */
void lzo_csr_spmm(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int b,
                  const double *X, int64_t ldx, double *Y, int64_t ldy, int col_major)
{
    int64_t r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < n; ++r) {
        for (int c = 0; c < b; ++c) {
            double acc = 0.0;
            for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
                const int64_t j = col[k];
                acc += val[k] * (col_major ? X[j + c * ldx] : X[j * ldx + c]);
            }
            if (col_major) Y[r + c * ldy] = acc;
            else Y[r * ldy + c] = acc;
        }
    }
}

void lzo_csr_spmm_f32(int64_t n, const int64_t *rp, const int32_t *col, const float *val, int b,
                      const float *X, int64_t ldx, float *Y, int64_t ldy)
{
    int64_t r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < n; ++r) {
        for (int c = 0; c < b; ++c) {
            float acc = 0.0f;
            for (int64_t k = rp[r]; k < rp[r + 1]; ++k) acc += val[k] * X[(int64_t)col[k] * ldx + c];
            Y[r * ldy + c] = acc;
        }
    }
}

/* ------------------------------------------------------------ eigen (Jacobi)
 * Cyclic Jacobi with the classic threshold strategy.  Independent of the
 * product's eigensolver (which is Householder + implicit QL).  Stands in for
 * cusolverDn{D,S}syevjBatched / syevd (utils/lib_utils.hpp:547-577,721-745). */
int lzo_sym_eig(int k, const double *Ain, double *eval, double *V)
{
    double *A = (double *)malloc((size_t)k * k * sizeof(double));
    if (!A) return -1;
    memcpy(A, Ain, (size_t)k * k * sizeof(double));
    /* symmetrise from the lower triangle, as syevj with CUBLAS_FILL_MODE_LOWER */
    for (int i = 0; i < k; ++i)
        for (int j = i + 1; j < k; ++j) A[i * k + j] = A[j * k + i];
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) V[i * k + j] = (i == j);
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                const double a = A[i * k + j] * A[i * k + j];
                tot += a;
                if (i != j) off += a;
            }
        if (off <= 1e-64 + 1e-34 * tot) break;
        for (int p = 0; p < k - 1; ++p)
            for (int qq = p + 1; qq < k; ++qq) {
                const double apq = A[p * k + qq];
                if (apq == 0.0) continue;
                const double app = A[p * k + p], aqq = A[qq * k + qq];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) /
                                 (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int r = 0; r < k; ++r) { /* A <- A J (columns p,q) */
                    const double arp = A[r * k + p], arq = A[r * k + qq];
                    A[r * k + p] = c * arp - s * arq;
                    A[r * k + qq] = s * arp + c * arq;
                }
                for (int r = 0; r < k; ++r) { /* A <- J^T A (rows p,q) */
                    const double apr = A[p * k + r], aqr = A[qq * k + r];
                    A[p * k + r] = c * apr - s * aqr;
                    A[qq * k + r] = s * apr + c * aqr;
                }
                A[p * k + qq] = A[qq * k + p] = 0.0;
                for (int r = 0; r < k; ++r) {
                    const double vrp = V[r * k + p], vrq = V[r * k + qq];
                    V[r * k + p] = c * vrp - s * vrq;
                    V[r * k + qq] = s * vrp + c * vrq;
                }
            }
    }
    for (int i = 0; i < k; ++i) eval[i] = A[i * k + i];
    /* sort ascending (selection sort; k is small) */
    for (int i = 0; i < k; ++i) {
        int mi = i;
        for (int j = i + 1; j < k; ++j)
            if (eval[j] < eval[mi]) mi = j;
        if (mi != i) {
            double t = eval[i]; eval[i] = eval[mi]; eval[mi] = t;
            for (int r = 0; r < k; ++r) {
                t = V[r * k + i]; V[r * k + i] = V[r * k + mi]; V[r * k + mi] = t;
            }
        }
    }
    free(A);
    return 0;
}

/* sqrtm_cusolver + custom_mult2, utils/lib_utils.hpp:649-694,721-745:
 * beta = V sqrt|l| V^T, beta_inv = V (1/sqrt|l|) V^T. */
int lzo_sqrtm_pair(int b, const double *G, double *beta, double *beta_inv)
{
    double ev[64], V[64 * 64];
    if (b > 64) return -1;
    lzo_sym_eig(b, G, ev, V);
    for (int r = 0; r < b; ++r)
        for (int c = 0; c < b; ++c) {
            double s1 = 0.0, s2 = 0.0;
            for (int i = 0; i < b; ++i) {
                const double sq = sqrt(fabs(ev[i]));
                s1 += V[r * b + i] * sq * V[c * b + i];
                s2 += V[r * b + i] * (1.0 / sq) * V[c * b + i];
            }
            beta[r * b + c] = s1;
            beta_inv[r * b + c] = s2;
        }
    return 0;
}

/* --------------------------------------------------- block Lanczos (f64/f32) */
#define REAL double
#define SFX _f64
#include "lz_oracle_tmpl.h"
#undef REAL
#undef SFX
#define REAL float
#define SFX _f32
#include "lz_oracle_tmpl.h"
#undef REAL
#undef SFX

int lzo_block_lanczos(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int b,
                      int m, int64_t lc, const double *B, double *q, double *alpha, double *beta)
{
    return block_lanczos_impl_f64(n, rp, col, val, b, m, lc, B, q, alpha, beta, NULL, NULL, NULL);
}

int lzo_block_lanczos_f32(int64_t n, const int64_t *rp, const int32_t *col, const float *val,
                          int b, int m, int64_t lc, const float *B, float *q, float *alpha,
                          float *beta)
{
    return block_lanczos_impl_f32(n, rp, col, val, b, m, lc, B, q, alpha, beta, NULL, NULL, NULL);
}

/* the same, plus the final Q0 (= Q1) and W blocks the reference leaves behind */
int lzo_block_lanczos_final(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int b,
                            int m, int64_t lc, const double *B, double *q, double *alpha, double *beta,
                            double *Qf, double *Wf)
{
    return block_lanczos_impl_f64(n, rp, col, val, b, m, lc, B, q, alpha, beta, NULL, Qf, Wf);
}

int lzo_block_lanczos_final_f32(int64_t n, const int64_t *rp, const int32_t *col, const float *val, int b,
                                int m, int64_t lc, const float *B, float *q, float *alpha, float *beta,
                                float *Qf, float *Wf)
{
    return block_lanczos_impl_f32(n, rp, col, val, b, m, lc, B, q, alpha, beta, NULL, Qf, Wf);
}

int lzo_block_lanczos_timed(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int b,
                            int m, int64_t lc, const double *B, double *q, double *alpha, double *beta,
                            double *t_each)
{
    return block_lanczos_impl_f64(n, rp, col, val, b, m, lc, B, q, alpha, beta, t_each, NULL, NULL);
}

/* ------------------------------------------------- single-vector Lanczos
 * vector_lanczos, methods/vector_lanczos.hpp:8-67 (the correct variant; the
 * BLAS variant's axpy at :116 updates q0 instead of w and is not restated). */
/* Deterministic parallel dot product: a fixed number of contiguous chunks, each
 * summed in order, the chunk sums added in chunk order -- the same bits for any
 * thread count (the single-vector oracle's reductions at n = 1e6, config C2). */
#define LZO_NCHUNK 256
static double dot_chunked(int64_t n, const double *x, const double *y)
{
    double part[LZO_NCHUNK];
#pragma omp parallel for schedule(static)
    for (int c = 0; c < LZO_NCHUNK; ++c) {
        const int64_t lo = n * c / LZO_NCHUNK, hi = n * (c + 1) / LZO_NCHUNK;
        double s = 0.0;
        for (int64_t i = lo; i < hi; ++i) s += x[i] * y[i];
        part[c] = s;
    }
    double s = 0.0;
    for (int c = 0; c < LZO_NCHUNK; ++c) s += part[c];
    return s;
}

/* y = a*y + b*x elementwise (order-free: parallel) */
static void axpby(int64_t n, double a, double *y, double b, const double *x)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) y[i] = a * y[i] + b * x[i];
}

static int vector_lanczos_impl(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int m,
                               int64_t lc, const double *bvec, double *q, double *alpha, double *beta,
                               double *t_each)
{
    double *q0 = (double *)malloc(n * sizeof(double));
    double *q1 = (double *)malloc(n * sizeof(double));
    double *w = (double *)malloc(n * sizeof(double));
    if (!q0 || !q1 || !w) return -2;
    beta[0] = sqrt(dot_chunked(n, bvec, bvec));           /* :20 */
    const double s0 = 1.0 / beta[0];
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) q0[i] = bvec[i] * s0; /* :23 */
    q[0] = q0[lc];                                        /* :26 */
    lzo_csr_spmm(n, rp, col, val, 1, q0, 1, w, 1, 0);     /* :29 */
    alpha[0] = dot_chunked(n, w, q0);                     /* :32 */
    axpby(n, 1.0, w, -alpha[0], q0);                      /* :35 */
    for (int j = 1; j < m; ++j) {
        const double t0 = lzo_wtime();
        beta[j] = sqrt(dot_chunked(n, w, w));             /* :43 */
        const double sj = 1.0 / beta[j];
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) q1[i] = w[i] * sj;  /* :46-47 */
        lzo_csr_spmm(n, rp, col, val, 1, q1, 1, w, 1, 0); /* :50 */
        axpby(n, 1.0, w, -beta[j], q0);                   /* :53 */
        alpha[j] = dot_chunked(n, w, q1);                 /* :56 */
        axpby(n, 1.0, w, -alpha[j], q1);                  /* :59 */
        double *t = q0; q0 = q1; q1 = t;                  /* :61 */
        q[j] = q0[lc];                                    /* :64 */
        if (t_each) t_each[j - 1] = lzo_wtime() - t0;
    }
    free(q0); free(q1); free(w);
    return 0;
}

int lzo_vector_lanczos(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int m,
                       int64_t lc, const double *bvec, double *q, double *alpha, double *beta)
{
    return vector_lanczos_impl(n, rp, col, val, m, lc, bvec, q, alpha, beta, NULL);
}

int lzo_vector_lanczos_timed(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int m,
                             int64_t lc, const double *bvec, double *q, double *alpha, double *beta, double *t_each)
{
    return vector_lanczos_impl(n, rp, col, val, m, lc, bvec, q, alpha, beta, t_each);
}

int lzo_block_lanczos_f32_timed(int64_t n, const int64_t *rp, const int32_t *col, const float *val, int b, int m,
                                int64_t lc, const float *B, float *q, float *alpha, float *beta, double *t_each)
{
    return block_lanczos_impl_f32(n, rp, col, val, b, m, lc, B, q, alpha, beta, t_each, NULL, NULL);
}

/* vector_lanczos<float> (methods/vector_lanczos.hpp:8-67 at T = float, as
 * test_lanczos.cu:355 instantiates it): float vectors, float SpMV sums in CSR
 * order; the norms and dots are accumulated in double and rounded to float
 * (the product's choice -- the reference's float reductions are device code);
 * the scale is 1./beta in double rounded to float (`mult_scalar(1./beta[j])`). */
int lzo_vector_lanczos_f32(int64_t n, const int64_t *rp, const int32_t *col, const float *val, int m,
                           int64_t lc, const float *bvec, float *q, float *alpha, float *beta)
{
    float *q0 = (float *)malloc(n * sizeof(float));
    float *q1 = (float *)malloc(n * sizeof(float));
    float *w = (float *)malloc(n * sizeof(float));
    if (!q0 || !q1 || !w) return -2;
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += (double)bvec[i] * bvec[i];
    beta[0] = (float)sqrt(s);                                          /* :20 */
    float sc = (float)(1.0 / (double)beta[0]);
    for (int64_t i = 0; i < n; ++i) q0[i] = bvec[i] * sc;              /* :23 */
    q[0] = q0[lc];                                                     /* :26 */
    lzo_csr_spmm_f32(n, rp, col, val, 1, q0, 1, w, 1);                 /* :29 */
    s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += (double)w[i] * q0[i];
    alpha[0] = (float)s;                                               /* :32 */
    for (int64_t i = 0; i < n; ++i) w[i] -= alpha[0] * q0[i];          /* :35 */
    for (int j = 1; j < m; ++j) {
        s = 0.0;
        for (int64_t i = 0; i < n; ++i) s += (double)w[i] * w[i];
        beta[j] = (float)sqrt(s);                                      /* :43 */
        sc = (float)(1.0 / (double)beta[j]);
        for (int64_t i = 0; i < n; ++i) q1[i] = w[i] * sc;             /* :46-47 */
        lzo_csr_spmm_f32(n, rp, col, val, 1, q1, 1, w, 1);             /* :50 */
        for (int64_t i = 0; i < n; ++i) w[i] -= beta[j] * q0[i];       /* :53 */
        s = 0.0;
        for (int64_t i = 0; i < n; ++i) s += (double)w[i] * q1[i];
        alpha[j] = (float)s;                                           /* :56 */
        for (int64_t i = 0; i < n; ++i) w[i] -= alpha[j] * q1[i];      /* :59 */
        float *t = q0; q0 = q1; q1 = t;                                /* :61 */
        q[j] = q0[lc];                                                 /* :64 */
    }
    free(q0); free(q1); free(w);
    return 0;
}

/* --------------------------------------------------------- T and results */
void lzo_assemble_T(int m, int b, const double *alpha, const double *beta, double *T)
{
    const int k = m * b;
    memset(T, 0, (size_t)k * k * sizeof(double));
    for (int blk = 0; blk < m; ++blk) {
        const double *a = alpha + (size_t)blk * b * b;
        for (int r = 0; r < b; ++r)
            for (int c = 0; c < b; ++c) T[(blk * b + r) * k + blk * b + c] = a[r * b + c];
        if (blk >= 1) {
            /* insert_subdiag_blocks, tridiagonal_matrix.hpp:32-54: beta_b at
             * (rows b-1, cols b) and its transpose at (rows b, cols b-1). */
            const double *bt = beta + (size_t)blk * b * b;
            for (int r = 0; r < b; ++r)
                for (int c = 0; c < b; ++c) {
                    T[((blk - 1) * b + r) * k + blk * b + c] = bt[r * b + c];
                    T[(blk * b + c) * k + (blk - 1) * b + r] = bt[r * b + c];
                }
        }
    }
}

int lzo_ritz_values(int m, int b, const double *alpha, const double *beta, double *ritz)
{
    const int k = m * b;
    double *T = (double *)malloc((size_t)k * k * sizeof(double));
    double *V = (double *)malloc((size_t)k * k * sizeof(double));
    if (!T || !V) return -2;
    lzo_assemble_T(m, b, alpha, beta, T);
    int rc = lzo_sym_eig(k, T, ritz, V);
    free(T); free(V);
    return rc;
}

/* test_lanczos.cu:272-286 with expm from expm_cusolver (lib_utils.hpp:542-590)
 * and dm::custom_mult (dense_kernels.hpp:52-78): expm(S) = V e^L V^T. */
int lzo_block_solution(int m, int b, double T_end, const double *alpha, const double *beta,
                       const double *q, double *solution)
{
    const int k = m * b;
    double *T = (double *)malloc((size_t)k * k * sizeof(double));
    double *V = (double *)malloc((size_t)k * k * sizeof(double));
    double *ev = (double *)malloc((size_t)k * sizeof(double));
    double *F = (double *)malloc((size_t)k * b * sizeof(double));
    if (!T || !V || !ev || !F) return -2;
    lzo_assemble_T(m, b, alpha, beta, T);
    for (int i = 0; i < k * k; ++i) T[i] *= T_end;                   /* :273 */
    lzo_sym_eig(k, T, ev, V);
    /* F1 = expm(T)[:, :b] */
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < b; ++c) {
            double s = 0.0;
            for (int i = 0; i < k; ++i) s += V[r * k + i] * exp(ev[i]) * V[c * k + i];
            F[r * b + c] = s;
        }
    /* F1 = F1 * beta[0]  (:281); solution = F1^T q  (:286) */
    for (int c = 0; c < b; ++c) {
        double s = 0.0;
        for (int r = 0; r < k; ++r) {
            double f = 0.0;
            for (int i = 0; i < b; ++i) f += F[r * b + i] * beta[i * b + c];
            s += f * q[r];
        }
        solution[c] = s;
    }
    free(T); free(V); free(ev); free(F);
    return 0;
}

int lzo_fdtd_block(int64_t n, const int64_t *rp, const int32_t *col, const double *val, int b,
                   const double *B, int64_t steps, double T_end, int64_t lc, double *out)
{
    const double dt = T_end / (double)steps;
    double *U = (double *)malloc((size_t)n * b * sizeof(double));
    double *D = (double *)malloc((size_t)n * b * sizeof(double));
    if (!U || !D) return -2;
    memcpy(U, B, (size_t)n * b * sizeof(double));
    for (int64_t s = 0; s < steps; ++s) {
        spmm_rm_f64(n, rp, col, val, b, U, D);                /* fdtd.hpp:48 */
        for (int64_t i = 0; i < n * b; ++i) U[i] += dt * D[i]; /* fdtd.hpp:49 */
    }
    for (int c = 0; c < b; ++c) out[c] = U[lc * b + c];
    free(U); free(D);
    return 0;
}
