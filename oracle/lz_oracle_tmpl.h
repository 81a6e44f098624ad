/* oracle/lz_oracle_tmpl.h -- TEST INFRASTRUCTURE ONLY.
 * Type-generic body of the oracle's block Lanczos, included by lz_oracle.c
 * once with REAL=double and once with REAL=float.  Requires REAL and SFX. */

#define CAT2_(a, b) a##b
#define CAT_(a, b) CAT2_(a, b)
#define FN(name) CAT_(name, SFX)

/* Y = A*X (row-major blocks) */
static void FN(spmm_rm)(int64_t n, const int64_t *rp, const int32_t *col, const REAL *val, int b,
                        const REAL *X, REAL *Y)
{
    int64_t r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < n; ++r) {
        REAL acc[64];
        for (int c = 0; c < b; ++c) acc[c] = 0;
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
            const REAL v = val[k];
            const REAL *x = X + (int64_t)col[k] * b;
            for (int c = 0; c < b; ++c) acc[c] += v * x[c];
        }
        REAL *y = Y + r * b;
        for (int c = 0; c < b; ++c) y[c] = acc[c];
    }
}

/* R = X^T Y (b x b, row-major), double accumulation per thread, fixed-order
 * combine: deterministic for a fixed thread count. */
static void FN(gram_rm)(int64_t n, int b, const REAL *X, const REAL *Y, double *R)
{
    const int nt = lzo_num_threads();
    double *part = (double *)calloc((size_t)nt * b * b, sizeof(double));
#pragma omp parallel num_threads(nt)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        double *P = part + (size_t)t * b * b;
        int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        for (int64_t r = lo; r < hi; ++r) {
            const REAL *x = X + r * b, *y = Y + r * b;
            for (int i = 0; i < b; ++i) {
                const double xi = x[i];
                for (int j = 0; j < b; ++j) P[i * b + j] += xi * (double)y[j];
            }
        }
    }
    for (int k = 0; k < b * b; ++k) R[k] = 0;
    for (int t = 0; t < nt; ++t)
        for (int k = 0; k < b * b; ++k) R[k] += part[(size_t)t * b * b + k];
    free(part);
}

/* W = s_w*W + s_q*Q*S  (S b x b row-major, given in double) */
static void FN(tsmm_rm)(int64_t n, int b, REAL s_w, REAL s_q, const REAL *Q, const double *S,
                        REAL *W)
{
    REAL Sr[64 * 64];
    for (int k = 0; k < b * b; ++k) Sr[k] = (REAL)S[k];
    int64_t r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < n; ++r) {
        REAL acc[64];
        const REAL *qr = Q + r * b;
        for (int j = 0; j < b; ++j) acc[j] = 0;
        for (int i = 0; i < b; ++i) {
            const REAL qi = qr[i];
            for (int j = 0; j < b; ++j) acc[j] += qi * Sr[i * b + j];
        }
        REAL *w = W + r * b;
        if (s_w == (REAL)0)
            for (int j = 0; j < b; ++j) w[j] = s_q * acc[j];
        else
            for (int j = 0; j < b; ++j) w[j] = s_w * w[j] + s_q * acc[j];
    }
}

/* block_lanczos_blas, methods/block_lanczos.hpp:104-166, op for op. */
/* Qf, Wf (optional, n x b): the state the reference leaves in Q0 (= Q1) and W
 * on return (:159, :162): Q_{m-1} and the last residual W_m. */
static int FN(block_lanczos_impl)(int64_t n, const int64_t *rp, const int32_t *col,
                                  const REAL *val, int b, int m, int64_t lc, const REAL *B,
                                  REAL *q, REAL *alpha, REAL *beta, double *t_each, REAL *Qf,
                                  REAL *Wf)
{
    if (b < 1 || b > 64 || m < 1 || n < 1) return -1;
    const size_t nb = (size_t)n * b, bb = (size_t)b * b;
    REAL *Q0 = (REAL *)malloc(nb * sizeof(REAL));
    REAL *Q1 = (REAL *)malloc(nb * sizeof(REAL));
    REAL *W = (REAL *)malloc(nb * sizeof(REAL));
    double G[64 * 64], Sq[64 * 64], Si[64 * 64], Al[64 * 64];
    if (!Q0 || !Q1 || !W) return -2;

    /* beta[0] = B'B ; sqrtm pair (block_lanczos.hpp:106-111) */
    FN(gram_rm)(n, b, B, B, G);
    lzo_sqrtm_pair(b, G, Sq, Si);
    if (beta) for (size_t k = 0; k < bb; ++k) beta[k] = (REAL)Sq[k];
    /* Q0 = B * beta_inv (:114) */
    FN(tsmm_rm)(n, b, 0, 1, B, Si, Q0);
    if (q) for (int c = 0; c < b; ++c) q[c] = Q0[lc * b + c];  /* (:118) */
    /* W = A*Q0 (:121) */
    FN(spmm_rm)(n, rp, col, val, b, Q0, W);
    /* alpha[0] = 0.5 (W'Q0 + Q0'W) (:124) */
    FN(gram_rm)(n, b, W, Q0, G);
    for (int i = 0; i < b; ++i)
        for (int j = 0; j < b; ++j) Al[i * b + j] = 0.5 * (G[i * b + j] + G[j * b + i]);
    if (alpha) for (size_t k = 0; k < bb; ++k) alpha[k] = (REAL)Al[k];
    /* W = W - Q0*alpha (:128) */
    FN(tsmm_rm)(n, b, 1, -1, Q0, Al, W);

    /* t_each[j - 1]: wall time of iteration j (the CPU baseline's samples) */
    for (int j = 1; j < m; ++j) {
        const double t0 = lzo_wtime();
        FN(gram_rm)(n, b, W, W, G);                                /* :137 */
        lzo_sqrtm_pair(b, G, Sq, Si);                              /* :142 */
        if (beta) for (size_t k = 0; k < bb; ++k) beta[j * bb + k] = (REAL)Sq[k];
        FN(tsmm_rm)(n, b, 0, 1, W, Si, Q1);                        /* :145 */
        FN(spmm_rm)(n, rp, col, val, b, Q1, W);                    /* :149 */
        FN(tsmm_rm)(n, b, 1, -1, Q0, Sq, W);                       /* :152 */
        FN(gram_rm)(n, b, W, Q1, G);                               /* :155 */
        for (int i = 0; i < b; ++i)
            for (int jj = 0; jj < b; ++jj)
                Al[i * b + jj] = 0.5 * (G[i * b + jj] + G[jj * b + i]);
        if (alpha) for (size_t k = 0; k < bb; ++k) alpha[j * bb + k] = (REAL)Al[k];
        FN(tsmm_rm)(n, b, 1, -1, Q1, Al, W);                       /* :159 */
        { REAL *t = Q0; Q0 = Q1; Q1 = t; }                         /* :162 */
        if (q) for (int c = 0; c < b; ++c) q[j * b + c] = Q0[lc * b + c]; /* :165 */
        if (t_each) t_each[j - 1] = lzo_wtime() - t0;
    }
    if (beta) for (size_t k = 0; k < bb; ++k) beta[(size_t)m * bb + k] = (REAL)Si[k];
    if (Qf) memcpy(Qf, Q0, nb * sizeof(REAL));
    if (Wf) memcpy(Wf, W, nb * sizeof(REAL));
    free(Q0); free(Q1); free(W);
    return 0;
}

#undef FN
#undef CAT_
#undef CAT2_
