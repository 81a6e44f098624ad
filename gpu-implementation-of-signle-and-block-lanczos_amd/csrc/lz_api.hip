// lz_api.hip -- the extern "C" boundary of liblz_hip.so (include/lz_hip.h)
// plus the device-resident Lanczos methods behind it.
#include <cstdarg>
#include <cstring>
#include <algorithm>
#include <utility>
#include <vector>

#include <type_traits>
#include "lz_comm.hpp"
#include "lz_common.hpp"
#include "lz_internal.hpp"
#include "lz_kernels.hpp"

namespace lz {

static thread_local char g_err[1024] = "";

int prof_begin(lz_handle *h, int cls)
{
    if (!h->prof || !((h->prof_mask >> cls) & 1u) || h->ev_used + 2 > h->ev_cap) return -1;
    const int idx = h->ev_used;
    if (hipEventRecord(h->ev_pool[idx], h->stream) != hipSuccess) return -1;
    h->ev_class[idx / 2] = cls;
    h->ev_used += 2;
    return idx;
}

int ensure_partials(lz_handle *h, size_t doubles)
{
    if (doubles <= h->partials_cap) return LZ_OK;
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    LZ_HIP_TRY(hipFree(h->partials));
    h->partials = nullptr;
    LZ_HIP_TRY(hipMalloc(&h->partials, doubles * sizeof(double)));
    h->partials_cap = doubles;
    return LZ_OK;
}

void prof_end(lz_handle *h, int idx)
{
    if (idx >= 0) (void)hipEventRecord(h->ev_pool[idx + 1], h->stream);
}

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// The wavefront step and the persistent pass 1 end a wait they would
// otherwise never leave by setting the device error word (lz_device_error);
// their results are then wrong.  The solve entry points that launch them clear
// the word on their stream first (a word an earlier call left behind is not
// this solve's) and read it once at the end (one host synchronisation per
// solve); a nonzero word fails the solve and stays readable by
// lz_device_error.
static int solve_begin(lz_handle *h)
{
    LZ_HIP_TRY(hipMemsetAsync(h->err_flag, 0, sizeof(int), h->stream));
    return LZ_OK;
}

static int solve_status(lz_handle *h)
{
    int e = 0;
    LZ_HIP_TRY(hipMemcpyAsync(&e, h->err_flag, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    if (e != 0) {
        set_error("device error word %d: a persistent kernel abandoned a bounded wait; the results are invalid "
                  "(lz_device_error reads and clears the word)", e);
        return LZ_E_DEVICE;
    }
    return LZ_OK;
}

static int check_csr(int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                     const void *val)
{
    LZ_ARG_CHECK(n >= 0 && nnz >= 0, "negative size");
    LZ_ARG_CHECK(rp != nullptr, "row_ptr is NULL");
    LZ_ARG_CHECK(nnz == 0 || (col != nullptr && val != nullptr), "col/val NULL");
    return LZ_OK;
}

template <typename T>
__global__ void k_axpy(int64_t n, T a, const T *__restrict__ x, T *__restrict__ y)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = fma(a, x[i], y[i]);
}

// One forward-Euler step Y = X + dt*A*X (fdtd.hpp:48-49 fused; X, Y distinct
// n x b row-major buffers).  Thread (r, c) sums row r in CSR order with fma
// and finishes with fma(dt, acc, X) -- the arithmetic of spmm_rm + k_axpy.
// The b threads of a row read the same col/val (one cache line) and
// b contiguous values of X per non-zero.
template <typename T>
__global__ void k_fdtd_step(int64_t nb, int b, const int64_t *__restrict__ rp,
                            const int32_t *__restrict__ col, const T *__restrict__ val, T dt,
                            const T *__restrict__ X, T *__restrict__ Y)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nb) return;
    const int64_t r = i / b;
    const int c = (int)(i - r * b);
    T acc = 0;
    for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k)
        acc = fma(val[k], X[(int64_t)col[k] * b + c], acc);
    Y[i] = fma(dt, acc, X[i]);
}

template <typename T>
static int axpy(lz_handle *h, int64_t n, T a, const T *x, T *y)
{
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), h->n_cu * 8));
    hipLaunchKernelGGL((k_axpy<T>), dim3(grid), dim3(256), 0, h->stream, n, a, x, y);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ---------------------------------------------------------- block Lanczos
// Reference op order, one kernel (or kernel pair) per reference call
// (methods/block_lanczos.hpp:104-166).  Any b <= 32, fp64 or fp32.
template <typename T>
static int block_lanczos_unfused(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                                 const T *val, int b, int m, int64_t lc, const T *B, T *q, T *alpha,
                                 T *beta, T *Q0, T *Q1, T *W)
{
    const int64_t bb = (int64_t)b * b;
    T *binv = beta + (int64_t)m * bb;  // the reference's beta[m]
    int P = 0;
    // beta[0] = sqrtm(B'B), beta[m] = inverse            (:106-111)
    LZ_TRY(gram_partials<T>(h, n, b, B, B, b, &P));
    LZ_TRY(sqrtm_pair<T>(h, b, nullptr, P, beta, binv, nullptr));
    LZ_TRY(tsmm<T>(h, n, b, T(0), T(1), B, binv, Q0, b));          // Q0 = B*beta_inv (:114)
    LZ_TRY(copy_row<T>(h, b, Q0, b, 0, lc, q));                     // (:118)
    LZ_TRY(spmm_rm<T>(h, n, nnz, rp, col, val, b, Q0, b, n, W, b));          // W = A*Q0 (:121)
    LZ_TRY(gram_partials<T>(h, n, b, W, Q0, b, &P));                 // alpha[0] (:124)
    LZ_TRY(gram_finish<T>(h, b, P, 1, alpha));
    LZ_TRY(tsmm<T>(h, n, b, T(1), T(-1), Q0, alpha, W, b));          // W -= Q0*alpha (:128)
    for (int j = 1; j < m; ++j) {
        T *bj = beta + j * bb, *aj = alpha + j * bb;
        LZ_TRY(gram_partials<T>(h, n, b, W, W, b, &P));              // (:137)
        LZ_TRY(sqrtm_pair<T>(h, b, nullptr, P, bj, binv, nullptr));  // (:142)
        LZ_TRY(tsmm<T>(h, n, b, T(0), T(1), W, binv, Q1, b));        // Q1 = W*beta_inv (:145)
        LZ_TRY(spmm_rm<T>(h, n, nnz, rp, col, val, b, Q1, b, n, W, b));      // W = A*Q1 (:149)
        LZ_TRY(tsmm<T>(h, n, b, T(1), T(-1), Q0, bj, W, b));         // W -= Q0*beta (:152)
        LZ_TRY(gram_partials<T>(h, n, b, W, Q1, b, &P));             // alpha[j] (:155)
        LZ_TRY(gram_finish<T>(h, b, P, 1, aj));
        LZ_TRY(tsmm<T>(h, n, b, T(1), T(-1), Q1, aj, W, b));         // W -= Q1*alpha (:159)
        std::swap(Q0, Q1);                                           // Q0 = Q1 (:162), no copy
        LZ_TRY(copy_row<T>(h, b, Q0, b, 0, lc, q + j * b));          // (:165)
    }
    // the pointer swaps leave Q_{m-1} in one buffer and Q_{m-2} in the other:
    // one copy gives the reference's Q0 = Q1 = Q_{m-1} on return
    if (m >= 2 && h->final_state)
        LZ_HIP_TRY(hipMemcpyAsync(Q1, Q0, sizeof(T) * (size_t)n * b, hipMemcpyDeviceToDevice, h->stream));
    return LZ_OK;
}

// Fused device-resident iteration, b = 16 fp64 (lz_fused.hip), Q-free: the
// normalised block Q_j = W_j beta_j^-1 is formed in registers where it is used
// (pass 1: the alpha slabs and the row probe; Q_j's other two uses fold into
// 16 x 16 products: Q_{j-1} beta_j = W_{j-1} (beta_{j-1}^-1 beta_j) in pass 1,
// Q_j alpha_j = W_j (beta_j^-1 alpha_j) in pass 2), so no pass writes or reads
// Q: A + 6 n b s bytes per step instead of A + 7 n b s.  Residual buffers:
// W_0 = B (read only); step j's output W' -> W'' goes to r0 at j = 0, r1 at
// j = 1 and from then on in place over W_{j-1} (row r read, then written, by
// the same wave).  residual_order: {r0, r1} = {W, Q1} for odd m, {Q1, W} for
// even m, so the last residual W_m is written into W itself and the post-call
// pass only forms Q0 = Q1 = W_{m-1} beta^-1 (in place over W_{m-1}, in Q1) --
// copying W_m over from Q1 cost C5's 10-step solve 2.56 GB.  The inverse square roots of two consecutive steps live in
// two scratch slots; beta[m] gets the last one, as the reference's.
// Once-per-solve set-up of pass 1: the strips' row orders and, for a gather
// source of 2^24+ rows, whether the windowed kernel applies.
struct Pass1Plan {
    const uint64_t *pairs = nullptr;
    int win = 0;
    const int16_t *col16 = nullptr;  // 16-bit strip-relative columns when every column is in reach
};
static int pass1_plan(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, int64_t nx,
                      int64_t row_off, Pass1Plan *pl)
{
    LZ_TRY(strip_pairs(h, n, rp, &pl->pairs));
    if (nx >= (1 << 24)) {
        bool ok = false;
        LZ_TRY(gather_window_ok(h, n, rp, col, nx, row_off, &ok));
        pl->win = ok ? 1 : 0;
    }
    if (nx < (1 << 24) || pl->win) LZ_TRY(col16_plan(h, n, nnz, rp, col, row_off, &pl->col16));
    return LZ_OK;
}

struct QfreeBufs {
    double *binv[2], *P;
    explicit QfreeBufs(lz_handle *h) : binv{h->scratch + 4 * 256, h->scratch + 5 * 256}, P(h->scratch + 6 * 256) {}
};

// B^T B's per-block slabs (b = 16 fp64) on the handle's side stream, forked
// from the main stream; h->ev_join is recorded behind them (the caller waits on
// it before the slabs are folded).
static int gram_beside(lz_handle *h, int64_t n, const double *B, int *P)
{
    LZ_HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
    LZ_HIP_TRY(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    std::swap(h->stream, h->side);  // gram_partials launches on h->stream
    const int rc = gram_partials<double>(h, n, 16, B, B, 16, P);
    std::swap(h->stream, h->side);
    LZ_TRY(rc);
    LZ_HIP_TRY(hipEventRecord(h->ev_join, h->side));
    return LZ_OK;
}

// The wavefront form of the same step (lz_wf.hip; default when it applies):
// one launch runs pass 2 of step j and pass 1 of step j + 1, then the sqrtm of
// G_{j+1} and the alpha kernel.  Buffers: Y_j in Q0 (every step, in place),
// V_0 = B (read only), V_1 in W, V_2 in Q1, then V_{j+1} over V_{j-1}.
static int block_lanczos_wf16(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                              const double *val, int m, int64_t lc, const double *B, double *q, double *alpha,
                              double *beta, double *Q0, double *Q1, double *W, const Pass1Plan &pl,
                              const WfPlan &wp, int Pg)
{
    constexpr int64_t bb = 256;
    (void)nnz;
    double *binv[2] = {h->scratch + 4 * 256, h->scratch + 5 * 256};
    double *P1 = h->scratch + 6 * 256, *P2 = h->scratch + 7 * 256;
    double *slab = h->scratch + 8 * 256;  // [S1 | S2 | G], 768
    int P = 0;
    const bool g0 = Pg < 0;  // beta_0's Gram from the first launch (wf_first_gram)
    // else B^T B's slabs (Pg of them) were made beside the plan (gram_beside)
    if (!g0) LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, Pg, beta, binv[0], nullptr));
    LZ_TRY(wf_reset16(h, n, wp));
    // Y_0 = A B, S1_0 = B^T Y_0 (g0: and G_0 = B^T B)
    LZ_TRY(wf_step16(h, n, rp, col, pl.col16, val, pl.pairs, wp, nullptr, nullptr, g0 ? B : nullptr, nullptr,
                     nullptr, nullptr, nullptr, B, Q0, 0, &P));
    if (g0) {  // beta_0, its inverse, alpha_0, P2 and q_0 in one kernel, as every later step's
        WfSlabs sl;
        sl.add(h->partials2, P);
        LZ_TRY(wf_fold16(h, sl, slab));
        WfAlpha wa;
        wa.part = slab;
        wa.P = 1;
        wa.alpha = alpha;
        wa.P2 = P2;
        wa.V = B;
        wa.lc = (lc >= 0 && lc < n) ? lc : -1;
        wa.qrow = q;
        LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, 1, beta, binv[0], nullptr, slab + 512, nullptr, nullptr, &wa));
    } else {
        LZ_TRY(alpha_wf16(h, h->partials2, P, binv[0], nullptr, alpha, P2, B, lc, n, q));
    }
    const double *Vm1 = nullptr, *V0 = B;
    for (int j = 0; j + 1 < m; ++j) {
        double *Vn = j == 0 ? W : j == 1 ? Q1 : const_cast<double *>(Vm1);
        LZ_TRY(wf_step16(h, n, rp, col, pl.col16, val, pl.pairs, wp, Q0, Vm1, V0, Vn, binv[j & 1], j ? P1 : nullptr,
                         P2, Vn, Q0, j + 1, &P));
        // the block slabs folded by 12 workgroups (one workgroup reading all
        // 1.5 MB took ~20 us), then beta_{j+1}, its inverse and P1 = beta_j^-1
        // beta_{j+1} from G, and (same launch) alpha_{j+1}, P2 and the row probe
        WfSlabs sl;
        sl.add(h->partials2, P);
        LZ_TRY(wf_fold16(h, sl, slab));
        WfAlpha wa;
        wa.part = slab;
        wa.P = 1;
        wa.alpha = alpha + (j + 1) * bb;
        wa.P2 = P2;
        wa.V = Vn;
        wa.lc = (lc >= 0 && lc < n) ? lc : -1;
        wa.qrow = q + (j + 1) * 16;
        LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, 1, beta + (j + 1) * bb, binv[(j + 1) & 1], nullptr, slab + 512,
                                  binv[j & 1], P1, &wa));
        Vm1 = V0;
        V0 = Vn;
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, binv[(m - 1) & 1], sizeof(double) * bb, hipMemcpyDeviceToDevice,
                              h->stream));
    // the reference's post-call state: W_m = Y_{m-1} beta^-1 - V_{m-2} P1 -
    // V_{m-1} P2 (the pass 2 a further step would run), Q0 = Q1 = V_{m-1} beta^-1
    // (Q1 untouched at m = 1, as the reference's).  The default shape: one
    // pass-2-only step launch whose updaters also store Q (QO; the LDS-DMA
    // streams of pass 2, 4 waves per CU); otherwise the MFMA strip kernel
    if (h->final_state) {
        if (wp.var == 111) {
            int Pq = 0;
            LZ_TRY(wf_step16(h, n, rp, col, pl.col16, val, pl.pairs, wp, Q0, Vm1, V0, W, binv[(m - 1) & 1],
                             Vm1 ? P1 : nullptr, P2, W, m >= 2 ? Q1 : nullptr, m, &Pq, -1, 0, 0, nullptr, nullptr,
                             Q0, true));
        } else {
            LZ_TRY(final_state<double>(h, n, 16, Q0, Vm1, V0, nullptr, binv[(m - 1) & 1], Vm1 ? P1 : nullptr, P2, W,
                                       Q0, m >= 2 ? Q1 : nullptr));
        }
    }
    return LZ_OK;
}

static int block_lanczos_fused16(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                                 const double *val, int m, int64_t lc, const double *B, double *q,
                                 double *alpha, double *beta, double *Q0, double *Q1, double *W)
{
    constexpr int64_t bb = 256;
    (void)Q0;
    QfreeBufs qb(h);
    int P = 0;
    Pass1Plan pl;
    // B^T B (beta_0's Gram): where the wavefront step will run with a shape
    // whose first launch sums it (wf_first_gram), there; otherwise on the side
    // stream while the once-per-solve plans (latency-bound passes over the
    // columns, each ending in a host sync) run on the main one, joined before
    // its sqrtm
    const bool g0 = wf_first_gram(n, nnz);
    if (!g0) LZ_TRY(gram_beside(h, n, B, &P));
    // every return from here on leaves the main stream behind the Gram (an early
    // error return too: the side stream's slabs must not race a later call)
    struct JoinSide {
        lz_handle *h;
        ~JoinSide() { (void)hipStreamWaitEvent(h->stream, h->ev_join, 0); }
    } join_side{h};
    {
        WfPlan wp;
        LZ_TRY(wf_plan16(h, n, nnz, rp, col, &wp));  // n < 2^24 only
        if (wp.ok) {
            LZ_TRY(strip_pairs(h, n, rp, &pl.pairs));
            pl.col16 = wp.col16;
            if (!g0) LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
            else if (wp.var != 111) LZ_TRY(gram_partials<double>(h, n, 16, B, B, 16, &P));  // (another shape)
            const bool first = g0 && wp.var == 111;
            return block_lanczos_wf16(h, n, nnz, rp, col, val, m, lc, B, q, alpha, beta, Q0, Q1, W, pl, wp,
                                      first ? -1 : P);
        }
    }
    if (g0) LZ_TRY(gram_partials<double>(h, n, 16, B, B, 16, &P));  // (the plan refused the wavefront)
    LZ_TRY(pass1_plan(h, n, nnz, rp, col, n, 0, &pl));
    LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
    LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, P, beta, qb.binv[0], nullptr));
    const double *in = B, *prev = nullptr;
    double *r0 = (m & 1) ? W : Q1, *r1 = (m & 1) ? Q1 : W;  // W_m lands in W (residual_order)
    for (int j = 0; j < m; ++j) {
        double *out = j == 0 ? r0 : j == 1 ? r1 : const_cast<double *>(prev);
        const double *bi = qb.binv[j & 1];
        LZ_TRY(fused_spmm16(h, n, rp, col, val, in, n, in, prev, out, bi, j ? qb.P : nullptr, lc, q + j * 16, &P,
                            pl.pairs, nnz, 0, pl.win, 0, pl.col16));
        // alpha_j and P2 = beta_j^-1 alpha_j in one kernel (P1 of this step is consumed)
        LZ_TRY(gram_finish<double>(h, 16, P, 1, alpha + j * bb, h->partials2, bi, qb.P));
        LZ_TRY(fused_update16(h, n, out, in, qb.P, &P));
        if (j + 1 < m)  // beta_{j+1}, its inverse and P1 = beta_j^-1 beta_{j+1}
            LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, P, beta + (j + 1) * bb, qb.binv[(j + 1) & 1], nullptr,
                                      nullptr, bi, qb.P));
        prev = in;
        in = out;
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, qb.binv[(m - 1) & 1], sizeof(double) * bb, hipMemcpyDeviceToDevice,
                              h->stream));
    if (h->final_state)  // W = W_m (in), Q0 = Q1 = W_{m-1} beta^-1 (prev)
        LZ_TRY(final_state<double>(h, n, 16, nullptr, nullptr, prev, in, qb.binv[(m - 1) & 1], nullptr, nullptr, W,
                                   Q0, m >= 2 ? Q1 : nullptr));
    return LZ_OK;
}

// Q-free iteration with the SpMM as its own launch (lz_fused32.hip): b = 32
// fp32 (BASELINE config C5) on MFMA passes, every other b <= 32 except 16-fp64
// (e.g. the reference driver's default N_COL = 4) on VALU passes.  The b = 16
// fp64 scheme above with the SpMM (the nnz-split tile kernel + long-tile queue
// that power-law rows need) writing Y into the API's Q0 buffer, then pass E
// and pass U: A + 9 n b s bytes per step against the reference order's
// A + 13 n b s.  The residual buffers rotate as in block_lanczos_fused16
// (B = W_0 read only, then r0, r1 -- W and Q1 in the order residual_order
// picks -- then in place).
// The b = 32 fp32 step in its beta^2 form (default; LZ_C5_B2=0 selects the
// pass-E form below): the SpMM's
// epilogue stores U = W' beta_j = A W_j - W_{j-1} M_j with M_j =
// beta_{j-1}^-1 G_j (G_j = W_j^T W_j, known before the step's sqrtm), so pass E
// shrinks to the slabs W_j^T U; alpha_j = sym(beta_j^-1 (W_j^T U) beta_j^-1),
// W'' = U beta_j^-1 - W_j beta_j^-1 alpha_j.  The sqrtm of G_{j+1} runs on the
// side stream beside the next SpMM, which needs only M_{j+1}.
static int block_lanczos_b2_32(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                               const float *val, int m, int64_t lc, const float *B, float *q, float *alpha,
                               float *beta, float *Q0, float *Q1, float *W)
{
    constexpr int b = 32;
    const int64_t bb = (int64_t)b * b;
    float *sc = reinterpret_cast<float *>(h->scratch + 4 * kMaxB * kMaxB);
    float *binv[2] = {sc, sc + bb}, *P2 = sc + 2 * bb, *M = sc + 3 * bb;
    float *U = Q0;
    // every return leaves the handle's stream behind the side stream's sqrtm
    // of the next step's G: an early error return too.  (beta_0's Gram and
    // sqrtm beside step 0's SpMM measured a wash: the SpMM paid the Gram's
    // bandwidth, profiles/r05zzs_c5_gram0_beside_ab.log)
    struct JoinSide {
        lz_handle *h;
        ~JoinSide() { (void)hipStreamWaitEvent(h->stream, h->ev_join, 0); }
    } join_side{h};
    int np = 0, cap = 768, lslot = -1;
    LZ_TRY(spmm_b2_stage(h, n, rp, &cap));  // (the solve's one host sync, before any of its work)
#ifndef LZ_B2_STEP0_QUEUES  // (measurement build: step 0 queues the list itself, as before round 5's end)
    LZ_TRY(spmm_b2_plan(h, n, rp, cap, &lslot));
#endif
    LZ_TRY(gram_partials<float>(h, n, b, B, B, b, &np));
    LZ_TRY(sqrtm_pair<float>(h, b, nullptr, np, beta, binv[0], nullptr));
    const float *in = B, *prev = nullptr;
    float *r0 = (m & 1) ? W : Q1, *r1 = (m & 1) ? Q1 : W;  // W_m lands in W (residual_order)
    for (int j = 0; j < m; ++j) {
        float *out = j == 0 ? r0 : j == 1 ? r1 : const_cast<float *>(prev);
        const float *bi = binv[j & 1];
        // the long-tile pass beside the tile pass, over the solve's list (from
        // step 1 on: C5 step 4.401-4.411 -> 4.381-4.385 ms; step 0 too since
        // the list is made up front; each tile computed as before)
#ifndef LZ_B2_STEP0_QUEUES
        LZ_TRY(spmm_rm_b2(h, n, nnz, rp, col, val, in, n, U, prev, j ? M : nullptr, lslot, nullptr, cap));
#else
        LZ_TRY(spmm_rm_b2(h, n, nnz, rp, col, val, in, n, U, prev, j ? M : nullptr, j ? lslot : -1,
                          j ? nullptr : &lslot, cap));
#endif
        if (j > 0) LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
        LZ_TRY(fused_el32(h, n, in, U, &np));
        // the one-workgroup kernels read 32 folded slabs, not the passes' 1024
        const int nf = fold_slabs_g(h, h->partials, np, (int)bb, 32);
        LZ_TRY(alpha_b2(h, h->partials2, nf, bi, alpha + j * bb, P2, in, lc, n, q + (int64_t)j * b));
        // the last step's pass UB also leaves the post-call Q0 = Q1 = W_j beta_j^-1
        // (from the W_j rows it holds; Q0 over U, Q1 over W_j, row by row): the
        // separate Q pass cost 0.89 ms a solve, this 0.65 (C5 step 4.289-4.294
        // -> 4.256-4.282 ms, profiles/r05zn_c5_ub_q_ab.log)
        const bool qlast = j + 1 == m && h->final_state;
        LZ_TRY(fused_ub32(h, n, U, in, bi, P2, out, &np, qlast ? Q0 : nullptr, qlast && m >= 2 ? Q1 : nullptr));
        if (j + 1 < m) {
            const int ng = fold_slabs_g(h, h->partials, np, (int)bb, 32);
            LZ_TRY(m_b2(h, h->partials2, ng, bi, M));  // M_{j+1} = beta_j^-1 G_{j+1}
            LZ_HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
            LZ_HIP_TRY(hipStreamWaitEvent(h->side, h->ev_fork, 0));
            hipStream_t main = h->stream;
            h->stream = h->side;
            // (from the 32 folded slabs m_b2 read: the same G bits, and the
            // one-workgroup kernel pulls 256 KB instead of the passes' 8 MB)
            const int rc = sqrtm_pair<float>(h, b, nullptr, ng, beta + (j + 1) * bb, binv[(j + 1) & 1], nullptr,
                                             h->partials2);
            h->stream = main;
            LZ_TRY(rc);
            LZ_HIP_TRY(hipEventRecord(h->ev_join, h->side));
        }
        prev = in;
        in = out;
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, binv[(m - 1) & 1], sizeof(float) * bb, hipMemcpyDeviceToDevice, h->stream));
    // (the post-call state: W = W_m is the last pass UB's output, in W by the
    // residual order, and that pass also wrote Q0 = Q1 = W_{m-1} beta^-1)
    return LZ_OK;
}

template <typename T>
static int block_lanczos_sep(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                             const T *val, int b, int m, int64_t lc, const T *B, T *q, T *alpha, T *beta, T *Q0,
                             T *Q1, T *W)
{
    if constexpr (std::is_same<T, float>::value) {  // default at b = 32; LZ_C5_B2=0: the form below
        const char *e = getenv("LZ_C5_B2");
        if (b == 32 && !(e && atoi(e) == 0) && spmm_b2_ok(n, nnz, n))
            return block_lanczos_b2_32(h, n, nnz, rp, col, val, m, lc, B, q, alpha, beta, Q0, Q1, W);
    }
    const int64_t bb = (int64_t)b * b;
    T *sc = reinterpret_cast<T *>(h->scratch + 4 * kMaxB * kMaxB);
    T *binv[2] = {sc, sc + bb}, *P = sc + 2 * bb;
    T *Y = Q0;
    int np = 0;
    LZ_TRY(gram_partials<T>(h, n, b, B, B, b, &np));
    LZ_TRY(sqrtm_pair<T>(h, b, nullptr, np, beta, binv[0], nullptr));
    const T *in = B, *prev = nullptr;
    T *r0 = (m & 1) ? W : Q1, *r1 = (m & 1) ? Q1 : W;  // W_m lands in W (residual_order)
    for (int j = 0; j < m; ++j) {
        T *out = j == 0 ? r0 : j == 1 ? r1 : const_cast<T *>(prev);
        const T *bi = binv[j & 1];
        // the SpMM gathers the unnormalised W_j: it needs no beta, so step j-1's
        // sqrtm runs beside it on the side stream; pass E waits for it
        LZ_TRY(spmm_rm<T>(h, n, nnz, rp, col, val, b, in, b, n, Y, b));
        if (j > 0) LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
        LZ_TRY(fused_e_sep<T>(h, n, b, Y, in, prev, out, bi, j ? P : nullptr, lc, q + (int64_t)j * b, &np));
        // alpha_j and P2 = beta_j^-1 alpha_j (this step's P1 is consumed)
        LZ_TRY(gram_finish<T>(h, b, np, 1, alpha + j * bb, h->partials, bi, P));
        LZ_TRY(fused_u_sep<T>(h, n, b, out, in, P, &np));
        if (j + 1 < m) {  // beta_{j+1}, its inverse and P1 = beta_j^-1 beta_{j+1}, on the side stream
            LZ_HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
            LZ_HIP_TRY(hipStreamWaitEvent(h->side, h->ev_fork, 0));
            hipStream_t main = h->stream;
            h->stream = h->side;
            const int rc = sqrtm_pair<T>(h, b, nullptr, np, beta + (j + 1) * bb, binv[(j + 1) & 1], nullptr, nullptr,
                                         bi, P);
            h->stream = main;
            LZ_TRY(rc);
            LZ_HIP_TRY(hipEventRecord(h->ev_join, h->side));
        }
        prev = in;
        in = out;
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, binv[(m - 1) & 1], sizeof(T) * bb, hipMemcpyDeviceToDevice, h->stream));
    if (h->final_state)  // W = W_m (in), Q0 = Q1 = W_{m-1} beta^-1 (prev)
        LZ_TRY(final_state<T>(h, n, b, nullptr, nullptr, prev, in, binv[(m - 1) & 1], nullptr, nullptr, W, Q0,
                              m >= 2 ? Q1 : nullptr));
    return LZ_OK;
}

// ------------------------------------------------------------------ FDTD
constexpr int64_t kFdtdGraph = 256;
constexpr int64_t kFdtdFusedRows = 1 << 18;

template <typename T>
static int fdtd_block(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const T *val,
                      int b, const T *U0, int64_t steps, double T_end, int64_t lc, T *U, T *D,
                      T *out)
{
    const T dt = (T)(T_end / (double)steps);   // fdtd.hpp:41
    LZ_HIP_TRY(hipMemcpyAsync(U, U0, sizeof(T) * n * b, hipMemcpyDeviceToDevice, h->stream));
    // Small systems (the driver's A(N) at N=10 has 6930 rows) are launch-bound:
    // one fused step kernel ping-ponging U <-> D.  Large ones take the tuned
    // SpMM then the axpy in place (D = A U, U += dt D).
    const bool fused = n <= kFdtdFusedRows;
    T *cur = U;
    auto step = [&]() -> int {
        if (fused) {
            T *nxt = cur == U ? D : U;
            const int64_t nb = n * b;
            hipLaunchKernelGGL((k_fdtd_step<T>), dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, h->stream,
                               nb, b, rp, col, val, dt, (const T *)cur, nxt);
            LZ_LAUNCH_CHECK();
            cur = nxt;
            return LZ_OK;
        }
        LZ_TRY(spmm_rm<T>(h, n, nnz, rp, col, val, b, U, b, n, D, b));    // fdtd.hpp:48
        return axpy<T>(h, n * b, dt, D, U);                           // fdtd.hpp:49
    };
    // The reference runs 10^6 steps of two small launches each: launch-bound.
    // After one eager step (it sizes every lazily grown workspace: nothing may
    // allocate inside a capture) kFdtdGraph steps are captured into a hipGraph
    // once and replayed; the remainder runs eagerly.  Same kernels, same order;
    // kFdtdGraph is even, so every replay starts from the same ping-pong buffer.
    const char *graph_env = getenv("LZ_FDTD_GRAPH");  // "0": eager loop (A/B)
    const bool use_graph = !(graph_env && graph_env[0] == '0');
    int64_t s = 0;
    LZ_TRY(step());
    ++s;
    if (use_graph && steps - s >= 2 * kFdtdGraph) {
        hipStream_t cap = nullptr;
        LZ_HIP_TRY(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
        const hipStream_t orig = h->stream;
        const bool prof = h->prof;
        h->stream = cap;
        h->prof = false;
        int rc = LZ_OK;
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        if (hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            set_error("fdtd: hipStreamBeginCapture failed");
            rc = LZ_E_HIP;
        } else {
            for (int64_t k = 0; k < kFdtdGraph && rc == LZ_OK; ++k) rc = step();
            const hipError_t e = hipStreamEndCapture(cap, &g);
            if (rc == LZ_OK && e != hipSuccess) {
                set_error("fdtd: hipStreamEndCapture: %s", hipGetErrorString(e));
                rc = LZ_E_HIP;
            }
        }
        h->stream = orig;
        h->prof = prof;
        if (rc == LZ_OK && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) {
            set_error("fdtd: hipGraphInstantiate failed");
            rc = LZ_E_HIP;
        }
        for (; rc == LZ_OK && steps - s >= kFdtdGraph; s += kFdtdGraph)
            if (hipGraphLaunch(ge, orig) != hipSuccess) {
                set_error("fdtd: hipGraphLaunch failed");
                rc = LZ_E_HIP;
            }
        if (ge) (void)hipGraphExecDestroy(ge);
        if (g) (void)hipGraphDestroy(g);
        (void)hipStreamDestroy(cap);
        LZ_TRY(rc);
    }
    for (; s < steps; ++s) LZ_TRY(step());
    if (cur != U)  // odd fused step count: the final state is in D
        LZ_HIP_TRY(hipMemcpyAsync(U, cur, sizeof(T) * n * b, hipMemcpyDeviceToDevice, h->stream));
    return copy_row<T>(h, b, U, b, 0, lc, out);                      // fdtd.hpp:52
}

// ------------------------------------------------------------ multi-GPU
// Row-partitioned iteration: rank g owns a contiguous row range
// of A and of every Krylov block.  Each step needs the rows of W_j its CSR
// references on other ranks (the exchange) and two b x b sums (all-reduces);
// the sqrtm is then computed redundantly on every rank.  Every collective goes
// through lz::Comm (lz_comm.hpp): RCCL between processes, or device copies
// between the virtual ranks of one process (the N-rank tests on one GPU).

int attach_comm(lz_handle *h, Comm *c)
{
    // the exchange stream and its events first; the communicator is attached
    // last, so a failure leaves the handle detached (and c deleted)
    hipStream_t xs = nullptr;
    hipEvent_t e1 = nullptr, e2 = nullptr, e3 = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&xs, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&e1, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&e2, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&e3, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (e3) (void)hipEventDestroy(e3);
        if (e2) (void)hipEventDestroy(e2);
        if (e1) (void)hipEventDestroy(e1);
        if (xs) (void)hipStreamDestroy(xs);
        delete c;
        set_error("attach_comm: exchange stream / events -> %s", hipGetErrorString(e));
        return LZ_E_HIP;
    }
    h->xstream = xs;
    h->ev_cx = e1;
    h->ev_xd = e2;
    h->ev_bd = e3;
    h->nranks = c->nranks;
    h->rank = c->rank;
    h->comm = c;
    return LZ_OK;
}

// Halo plan (lz_halo_init): each peer's requested rows are one contiguous run
// of the receiver's halo (ascending global row, so grouped by owner).
struct HaloPlan {
    int64_t n_local = 0, n_halo = 0, n_send = 0;
    // the rows peers request lie in [0, send_head) and [send_tail, n_local)
    // (the first / second half's extremes): the wavefront step's pass 2 of
    // their tiles runs first, so the exchange can overlap the rest of the step
    int64_t send_head = 0, send_tail = 0;
    std::vector<int64_t> soff, roff;  // nranks + 1 row offsets per peer
    int32_t *send_idx = nullptr;      // device: local rows to pack, grouped by peer
    void *sendbuf = nullptr;          // device: n_send packed rows
    size_t send_cap = 0;              // bytes
};

static void halo_free(lz_handle *h)
{
    if (!h->halo) return;
    HaloPlan *hp = static_cast<HaloPlan *>(h->halo);
    (void)hipFree(hp->send_idx);
    (void)hipFree(hp->sendbuf);
    delete hp;
    h->halo = nullptr;
}

static void detach_comm(lz_handle *h)
{
    halo_free(h);
    if (h->xstream) (void)hipStreamSynchronize(h->xstream);
    delete h->comm;
    h->comm = nullptr;
    if (h->ev_cx) (void)hipEventDestroy(h->ev_cx);
    if (h->ev_xd) (void)hipEventDestroy(h->ev_xd);
    if (h->ev_bd) (void)hipEventDestroy(h->ev_bd);
    if (h->xstream) (void)hipStreamDestroy(h->xstream);
    h->ev_cx = h->ev_xd = h->ev_bd = nullptr;
    h->xstream = nullptr;
    h->nranks = 1;
    h->rank = 0;
    h->grid_cap = 0;
}

// grow a device workspace; never inside the steps (it synchronises)
static int grow_ws(lz_handle *h, void **buf, size_t *cap, size_t bytes)
{
    if (bytes <= *cap) return LZ_OK;
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->xstream) LZ_HIP_TRY(hipStreamSynchronize(h->xstream));
    (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    LZ_HIP_TRY(hipMalloc(buf, bytes));
    *cap = bytes;
    return LZ_OK;
}

// rows idx[i] of X (rowb bytes each) packed one after another, V-sized pieces
template <typename V>
__global__ void k_halo_pack(int64_t ns, const int32_t *__restrict__ idx, const char *__restrict__ X, int64_t rowb,
                            V *__restrict__ out)
{
    const int64_t per = rowb / (int64_t)sizeof(V);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ns * per;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / per;
        out[t] = reinterpret_cast<const V *>(X + (int64_t)idx[r] * rowb)[t - r * per];
    }
}

// fill rows [n_local, n_local + n_halo) of X (rowb bytes per row) from their
// owners: pack the requested own rows, then one grouped point-to-point round
static int halo_exchange(lz_handle *h, HaloPlan &hp, void *X, size_t rowb, hipStream_t s)
{
    if (!h->comm || h->nranks == 1) return LZ_OK;
    LZ_ARG_CHECK(hp.send_cap >= (size_t)hp.n_send * rowb, "halo send buffer smaller than the plan (internal)");
    if (hp.n_send > 0) {
        const bool v16 = rowb % 16 == 0;
        const int64_t pieces = hp.n_send * (int64_t)(rowb / (v16 ? 16 : 4));
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(pieces, 256), (int64_t)h->n_cu * 4));
        if (v16)
            hipLaunchKernelGGL(k_halo_pack<uint4>, dim3(grid), dim3(256), 0, s, hp.n_send, hp.send_idx,
                               (const char *)X, (int64_t)rowb, (uint4 *)hp.sendbuf);
        else
            hipLaunchKernelGGL(k_halo_pack<uint32_t>, dim3(grid), dim3(256), 0, s, hp.n_send, hp.send_idx,
                               (const char *)X, (int64_t)rowb, (uint32_t *)hp.sendbuf);
        LZ_LAUNCH_CHECK();
    }
    std::vector<P2POp> ops;
    ops.reserve(h->nranks);
    char *sb = static_cast<char *>(hp.sendbuf), *xb = static_cast<char *>(X);
    for (int p = 0; p < h->nranks; ++p) {
        if (p == h->rank) continue;
        const size_t sc = (size_t)(hp.soff[p + 1] - hp.soff[p]) * rowb, rc = (size_t)(hp.roff[p + 1] - hp.roff[p]) * rowb;
        if (sc || rc)
            ops.push_back(P2POp{p, sb + hp.soff[p] * rowb, sc, xb + (hp.n_local + hp.roff[p]) * rowb, rc});
    }
    return h->comm->exchange(ops.data(), (int)ops.size(), s);
}

// Interior / boundary split of the local rows (once per solve): rows
// [i0, i1) reference only columns in [lo, hi) -- the rank's own rows of the
// gather source -- so their pass 1 (or SpMM) needs no exchanged row and runs
// while the exchange is in flight; rows [0, i0) and [i1, n) follow it.  i0 is
// the end of the last row in the first half that reaches outside, i1 the first
// such row in the second half (a banded partition's halo rows sit at both
// ends), both rounded outward to 16-row strips.
struct SplitPlan {
    bool on = false;
    int64_t i0 = 0, i1 = 0;
};

__global__ void k_span_init(int64_t n, unsigned long long *out)
{
    out[0] = 0;
    out[1] = (unsigned long long)n;
}

__global__ __launch_bounds__(256) void k_local_span(int64_t n, const int64_t *__restrict__ rp,
                                                    const int32_t *__restrict__ col, int64_t lo, int64_t hi,
                                                    unsigned long long *__restrict__ out)
{
    unsigned long long head = 0, tail = (unsigned long long)n;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        bool ext = false;
        for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k) {
            const int64_t c = col[k];
            ext |= (c < lo) | (c >= hi);
        }
        if (ext) {
            if (2 * r < n) head = head > (unsigned long long)(r + 1) ? head : (unsigned long long)(r + 1);
            else tail = tail < (unsigned long long)r ? tail : (unsigned long long)r;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long a = __shfl_xor(head, o, 64), t = __shfl_xor(tail, o, 64);
        head = a > head ? a : head;
        tail = t < tail ? t : tail;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], head);
        atomicMin(&out[1], tail);
    }
}

static int split_plan(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, int64_t lo, int64_t hi,
                      SplitPlan *sp)
{
    sp->on = false;
    const char *e = getenv("LZ_DIST_OVERLAP");  // "0": exchange, then the whole pass (A/B)
    if ((e && e[0] == '0') || !h->comm || h->nranks < 2 || n < 64) return LZ_OK;
    unsigned long long *d = reinterpret_cast<unsigned long long *>(h->scratch + 7 * kMaxB * kMaxB);
    hipLaunchKernelGGL(k_span_init, dim3(1), dim3(1), 0, h->stream, n, d);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)256), (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_local_span, dim3(grid), dim3(256), 0, h->stream, n, rp, col, lo, hi, d);
    LZ_LAUNCH_CHECK();
    unsigned long long hs[2] = {0, 0};
    LZ_HIP_TRY(hipMemcpyAsync(hs, d, sizeof(hs), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    const int64_t i0 = ceil_div((int64_t)hs[0], 16) * 16, i1 = ((int64_t)hs[1] / 16) * 16;
    // worth a second launch only when most rows are interior and some are not
    if (i1 - i0 >= n / 4 && (i0 > 0 || i1 < n)) {
        sp->on = true;
        sp->i0 = i0;
        sp->i1 = i1;
    }
    return LZ_OK;
}

enum { kFormHalo = 0, kFormAllgather = 1 };

static int dist_solve_wf16(lz_handle *h, int form, HaloPlan *hp, int64_t n, int64_t n_pad, int64_t nnz,
                           const int64_t *rp, const int32_t *col, const double *val, int m, int64_t lc,
                           const double *B, double *q, double *alpha, double *beta, double *X0, double *X1,
                           const WfPlan &wp, const SplitPlan &sp, bool g0);

// The distributed iteration, both exchange forms, any b <= 32, fp64 / fp32.
//   b = 16 fp64: the fused Q-free passes of block_lanczos_fused16 (pass 1 =
//     SpMM + epilogue, pass 2 update + Gram);
//   other b: the SpMM, then the VALU / MFMA passes E and U of block_lanczos_sep.
// Buffers (rows of b elements, row-major):
//   halo      X0, X1: n + n_halo rows; the residual alternates between them,
//             own rows first, then the halo; pass 1 gathers from one and writes
//             the other's own rows (W_{j-1} there, read then overwritten).
//   allgather X0 = X_full (n_pad * nranks rows; the rank's W_j lives in its own
//             slot), X1 = W (n_pad rows, W_{j-1}); pass 2 in its SWAP form
//             writes W_{j+1} into the slot and W_j into W, so the all-gather is
//             in place and moves only the peers' slabs.
// With a split plan the exchange of step j's result runs on the handle's
// exchange stream while pass 1 (or the SpMM) of step j+1 runs over the
// interior rows; the boundary rows follow once it has landed.  Issue order:
// pass 2 -> all-reduce -> sqrtm -> exchange (xstream) -> interior pass 1, so on
// one communicator the step's small all-reduces never queue behind the
// exchange.
template <typename T>
static int dist_solve_impl(lz_handle *h, int form, HaloPlan *hp, int64_t n, int64_t n_pad, int64_t nnz,
                           const int64_t *rp, const int32_t *col, const T *val, int b, int m, int64_t lc, const T *B,
                           T *q, T *alpha, T *beta, T *X0, T *X1)
{
    Comm *cm = h->comm;
    const bool ag = form == kFormAllgather;
    const bool f16 = std::is_same<T, double>::value && b == 16;
    const int64_t bb = (int64_t)b * b;
    const size_t rowb = sizeof(T) * (size_t)b;
    const int64_t nx = ag ? n_pad * h->nranks : n + (hp ? hp->n_halo : 0);
    const int64_t own_off = ag ? (int64_t)h->rank * n_pad : 0;
    double *slab = h->scratch;  // the reduced b x b slab (fp64), all-reduced in place
    T *sc = reinterpret_cast<T *>(h->scratch + 4 * kMaxB * kMaxB);
    T *binv[2] = {sc, sc + bb}, *P = sc + 2 * bb;
    T *own = X0 + own_off * b;  // allgather: this rank's slot of X_full
    // ---- once per solve (before any step: these may synchronise).  Every
    // set-up step that can fail runs before the solve's first collective, the
    // ranks' vote below: a rank whose set-up failed still joins it, with
    // ok = 0, so every rank returns an error instead of its peers waiting in a
    // collective this rank never issues.
    int prc = h->dbg_setup_fail;  // lz_debug_fail_next_setup (test support), consumed here
    h->dbg_setup_fail = 0;
    if (prc != LZ_OK) set_error("set-up failure forced by lz_debug_fail_next_setup");
    T *Y = nullptr;
    if (prc == LZ_OK && !f16) {
        prc = grow_ws(h, &h->ybuf, &h->ybuf_cap, (size_t)std::max<int64_t>(n, 1) * rowb);
        Y = static_cast<T *>(h->ybuf);
    }
    if (prc == LZ_OK && !ag && hp && cm && h->nranks > 1)
        prc = grow_ws(h, &hp->sendbuf, &hp->send_cap, (size_t)std::max<int64_t>(hp->n_send, 1) * rowb);
    // the wavefront step when it applies (LZ_PASS_WF=0: the two passes).  The
    // all-gather form takes it at one rank, where its exchange moves nothing:
    // at N > 1 the all-gather (the whole block from every peer; ~4.2 ms at C4
    // on 8 GPUs) outlasts the step's compute, and the two-pass
    // step hides the interior rows' pass 1 under it where the wavefront step,
    // which needs the exchange between its pass 2 and the boundary tiles'
    // pass 1, could hide nothing.  LZ_AG_WF=1 / 0 forces it on / off (tests).
    const char *agw = getenv("LZ_AG_WF");
    const bool ag_wf = agw ? agw[0] == '1' : h->nranks == 1;
    const bool try_wf = std::is_same<T, double>::value && f16 && (!ag || ag_wf);
    WfPlan wp;
    bool g0 = false;  // beta_0's Gram from the first launch: the default shape (XO 1, dist_solve_wf16)
    if (prc == LZ_OK && try_wf) {
        prc = wf_plan16(h, n, nnz, rp, col, &wp, nx, own_off);
        g0 = wp.var == 111;
    }
    Pass1Plan pl;
    SplitPlan sp;
    // the plans of the step form this rank expects (the vote may still turn
    // the wavefront form down: then the two-pass plan follows the vote)
    auto plan_twopass = [&]() -> int {
        if (f16) LZ_TRY(pass1_plan(h, n, nnz, rp, col, nx, own_off, &pl));
        if (!f16 || fused16_direct(nx, pl.win)) LZ_TRY(split_plan(h, n, rp, col, own_off, own_off + n, &sp));
        return LZ_OK;
    };
    bool planned_twopass = false;
    if (prc == LZ_OK && try_wf && wp.ok) prc = split_plan(h, n, rp, col, own_off, own_off + n, &sp);
    if (prc == LZ_OK && !(try_wf && wp.ok)) {
        prc = plan_twopass();
        planned_twopass = true;
    }
    // ---- the vote: set-up ok on every rank, and (b = 16 fp64) the wavefront
    // form and the first-launch Gram only where every rank can take them
    // (their collectives must match)
    if (cm && h->nranks > 1) {
        double v[3] = {prc == LZ_OK ? 1.0 : 0.0, wp.ok ? 1.0 : 0.0, g0 ? 1.0 : 0.0};
        LZ_HIP_TRY(hipMemcpyAsync(slab, v, sizeof(v), hipMemcpyHostToDevice, h->stream));
        LZ_TRY(cm->allreduce_sum(slab, 3, h->stream));
        LZ_HIP_TRY(hipMemcpyAsync(v, slab, sizeof(v), hipMemcpyDeviceToHost, h->stream));
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        if (v[0] != (double)h->nranks) {
            if (prc == LZ_OK) {
                set_error("a peer rank failed its set-up of this distributed solve (%d of %d ok)", (int)v[0],
                          h->nranks);
                prc = LZ_E_STATE;
            }
            return prc;
        }
        wp.ok = v[1] == (double)h->nranks;
        g0 = v[2] == (double)h->nranks;
    } else if (prc != LZ_OK) {
        return prc;
    }
    if constexpr (std::is_same<T, double>::value) {
        if (try_wf) {
            h->last_wf = wp.ok ? 1 : 0;
            h->last_wf_pre = 0;
            if (wp.ok) {
                h->last_split[0] = sp.on ? sp.i0 : -1;
                h->last_split[1] = sp.on ? sp.i1 : -1;
                return dist_solve_wf16(h, form, hp, n, n_pad, nnz, rp, col, val, m, lc, B, q, alpha, beta, X0, X1,
                                       wp, sp, g0);
            }
        }
    }
    h->last_wf = h->last_wf_pre = 0;
    // (only where a peer turned the wavefront form down after this rank planned it)
    if (!planned_twopass) LZ_TRY(plan_twopass());
    h->last_split[0] = sp.on ? sp.i0 : -1;
    h->last_split[1] = sp.on ? sp.i1 : -1;
    const bool reduce = cm && (ag || h->nranks > 1);
    auto allreduce = [&]() -> int { return reduce ? cm->allreduce_sum(slab, (size_t)bb, h->stream) : LZ_OK; };
    // step jj's buffers
    auto gsrc = [&](int jj) -> T * { return ag ? X0 : (jj & 1 ? X1 : X0); };       // gather source, W_jj in own rows
    auto wj = [&](int jj) -> T * { return ag ? own : gsrc(jj); };                   // W_jj's own rows
    auto wn = [&](int jj) -> T * { return ag ? X1 : (jj & 1 ? X0 : X1); };          // W' / W'' (own rows)
    // pass 1 (b = 16: fused) or the SpMM (other b) of step jj over rows [r0, r1)
    int nslab = 0;  // b = 16: folded slabs written so far this step (at h->partials2)
    auto pass1 = [&](int jj, int64_t r0, int64_t r1) -> int {
        if (r1 <= r0) return LZ_OK;
        const int64_t nnz_r = (int64_t)((double)nnz * (double)(r1 - r0) / (double)n);  // same kernel shape as the whole
        if (!f16)
            return spmm_rm<T>(h, r1 - r0, nnz_r, rp + r0, col, val, b, gsrc(jj), b, nx, Y + r0 * b, b);
        if constexpr (std::is_same<T, double>::value) {
            const int64_t lcr = (lc >= r0 && lc < r1) ? lc - r0 : -1;
            int np = 0;
            LZ_TRY(fused_spmm16(h, r1 - r0, rp + r0, col, val, gsrc(jj), nx, wj(jj) + r0 * 16,
                                jj ? wn(jj) + r0 * 16 : nullptr, wn(jj) + r0 * 16, binv[jj & 1], jj ? P : nullptr, lcr,
                                q + (int64_t)jj * 16, &np, pl.pairs + r0 / 16, nnz_r, own_off + r0, pl.win, nslab,
                                pl.col16));
            nslab += np;
        }
        return LZ_OK;
    };
    // the exchange that completes step jj's gather source (W_jj in own rows)
    auto exchange = [&](int jj, hipStream_t s) -> int {
        if (ag) return cm->allgather(own, X0, (size_t)n_pad * rowb, s);
        return hp ? halo_exchange(h, *hp, gsrc(jj), rowb, s) : LZ_OK;
    };
    // ---- beta_0 from the global Gram of B, W_0 = B into the gather source
    int np = 0;
    LZ_TRY(gram_partials<T>(h, n, b, B, B, b, &np));
    LZ_TRY(gram_finish<double>(h, b, np, 0, slab));
    LZ_TRY(allreduce());
    LZ_TRY(sqrtm_pair<T>(h, b, nullptr, 1, beta, binv[0], nullptr, slab));
    if (ag) {
        LZ_TRY(cm->allgather(B, X0, (size_t)n_pad * rowb, h->stream));
    } else {
        LZ_HIP_TRY(hipMemcpyAsync(X0, B, (size_t)n * rowb, hipMemcpyDeviceToDevice, h->stream));
        LZ_TRY(exchange(0, h->stream));
    }
    bool interior_done = false;  // step j's interior rows already ran beside the exchange
    for (int j = 0; j < m; ++j) {
        const T *bi = binv[j & 1];
        if (interior_done) {
            LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_xd, 0));
            LZ_TRY(pass1(j, 0, sp.i0));
            LZ_TRY(pass1(j, sp.i1, n));
        } else {
            nslab = 0;
            LZ_TRY(pass1(j, 0, n));
        }
        if (f16) {
            LZ_TRY(gram_finish<double>(h, 16, nslab, 0, slab, h->partials2));
        } else {
            LZ_TRY(fused_e_sep<T>(h, n, b, Y, wj(j), j ? wn(j) : nullptr, wn(j), bi, j ? P : nullptr, lc,
                                  q + (int64_t)j * b, &np));
            LZ_TRY(gram_finish<double>(h, b, np, 0, slab));
        }
        LZ_TRY(allreduce());
        // alpha_j and P2 = beta_j^-1 alpha_j (this step's P1 is consumed)
        LZ_TRY(gram_finish<T>(h, b, 1, 1, alpha + j * bb, slab, bi, P));
        if constexpr (std::is_same<T, double>::value) {
            if (f16) {
                if (ag) LZ_TRY(fused_update16_swap(h, n, X1, own, P, &np));
                else LZ_TRY(fused_update16(h, n, wn(j), wj(j), P, &np));
            }
        }
        if (!f16) {
            if (ag) LZ_TRY(fused_u_swap_sep<T>(h, n, b, X1, own, P, &np));
            else LZ_TRY(fused_u_sep<T>(h, n, b, wn(j), wj(j), P, &np));
        }
        interior_done = false;
        if (j + 1 < m) {
            LZ_TRY(gram_finish<double>(h, b, np, 0, slab));
            LZ_TRY(allreduce());
            // beta_{j+1}, its inverse and P1 = beta_j^-1 beta_{j+1}
            LZ_TRY(sqrtm_pair<T>(h, b, nullptr, 1, beta + (j + 1) * bb, binv[(j + 1) & 1], nullptr, slab, bi, P));
            if (sp.on) {
                LZ_HIP_TRY(hipEventRecord(h->ev_cx, h->stream));
                LZ_HIP_TRY(hipStreamWaitEvent(h->xstream, h->ev_cx, 0));
                LZ_TRY(exchange(j + 1, h->xstream));
                LZ_HIP_TRY(hipEventRecord(h->ev_xd, h->xstream));
                nslab = 0;
                LZ_TRY(pass1(j + 1, sp.i0, sp.i1));
                interior_done = true;
            } else {
                LZ_TRY(exchange(j + 1, h->stream));
            }
        }
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, binv[(m - 1) & 1], sizeof(T) * bb, hipMemcpyDeviceToDevice, h->stream));
    if (cm) LZ_TRY(cm->fence(h->stream));  // no peer reads this rank's buffers after the call
    return LZ_OK;
}

// The wavefront step (lz_wf.hip) on a row-partitioned rank, b = 16 fp64.
// Halo form, per step:
//   1. pass 2 of the tiles holding rows peers request (the first and last
//      ones of a banded slab): a pass-2-only launch;
//   2. the halo exchange of V_{j+1} on the exchange stream, beside
//   3. the step launch: pass 2 of the other tiles + pass 1 of the interior
//      tiles (their columns are own rows);
//   4. pass 1 of the boundary tiles (head, tail) once the halo has landed;
// then the slab sets [S1 | S2 | G] of the launches are folded and summed over
// the ranks in ONE 768-double all-reduce, and one sqrtm launch makes beta,
// P1 and alpha, P2, q.  Without a split (or with the requested rows spread
// over the slab) steps 1 and 2 are the step launch's pass 2 and a serial
// exchange.  V_0 = B copied into X0 (with its halo); V_{j+1} over V_{j-1} in
// X1, X0, ...; Y (own rows) in the handle's workspace.
// All-gather form: X0 = X_full (n_pad * N rows), the rank's slot at rank *
// n_pad holds V_j; X1 = W (n_pad rows) holds V_{j-1}: the step launch's pass 2
// writes V_{j+1} into the slot and V_j into W (SW), then the in-place
// all-gather, then the boundary tiles.
static int dist_solve_wf16(lz_handle *h, int form, HaloPlan *hp, int64_t n, int64_t n_pad, int64_t nnz,
                           const int64_t *rp, const int32_t *col, const double *val, int m, int64_t lc,
                           const double *B, double *q, double *alpha, double *beta, double *X0, double *X1,
                           const WfPlan &wp, const SplitPlan &sp, bool g0)
{
    Comm *cm = h->comm;
    constexpr int64_t bb = 256;
    const size_t rowb = 128;
    const bool ag = form == kFormAllgather;
    const int64_t nx = ag ? n_pad * h->nranks : n + (hp ? hp->n_halo : 0);
    const int64_t own_off = ag ? (int64_t)h->rank * n_pad : 0;
    const int64_t T = ceil_div(n, (int64_t)wp.tr);
    double *slab = h->scratch;  // [S1 | S2 | G], all-reduced in place
    double *sc = h->scratch + 4 * kMaxB * kMaxB;
    double *binv[2] = {sc, sc + bb}, *P1 = sc + 2 * bb, *P2 = sc + 3 * bb;
    (void)nnz;
    LZ_ARG_CHECK(wp.xoff == own_off, "wavefront plan for another slot (internal)");
    LZ_TRY(grow_ws(h, &h->ybuf, &h->ybuf_cap, (size_t)std::max<int64_t>(n, 1) * rowb));
    double *Y = static_cast<double *>(h->ybuf);
    const uint64_t *pairs = nullptr;
    LZ_TRY(strip_pairs(h, n, rp, &pairs));
    double *slot = X0 + own_off * 16;  // all-gather: this rank's rows of X_full
    // interior pass-1 tiles: inside the split plan's interior rows (every tile
    // when no column leaves the rank's rows)
    const bool exch = h->nranks > 1 && (ag || (hp && hp->n_halo > 0));
    int64_t t0 = 0, t1 = T;
    if (exch) {
        t0 = t1 = 0;
        if (sp.on) {
            t0 = ceil_div(sp.i0, (int64_t)wp.tr);
            t1 = std::min<int64_t>(T, sp.i1 / wp.tr);
            if (t1 <= t0) t0 = t1 = 0;
        }
    }
    // halo form: pass 2 of the requested rows' tiles first, the exchange
    // beside the rest of the step (LZ_DIST_OVERLAP=0 turns the split off too)
    int64_t sh = 0, st = T;
    bool pre = false;
    if (!ag && exch && sp.on && hp->n_send > 0) {
        sh = ceil_div(hp->send_head, (int64_t)wp.tr);
        st = std::max(sh, hp->send_tail / wp.tr);
        pre = st - sh >= T / 4;
    }
    h->last_wf_pre = pre ? 1 : 0;
    const bool reduce = cm && h->nranks > 1;
    auto allreduce = [&](size_t cnt) -> int { return reduce ? cm->allreduce_sum(slab, cnt, h->stream) : LZ_OK; };
    auto exchange = [&](double *X, hipStream_t s) -> int {
        if (ag) return cm ? cm->allgather(slot, X0, (size_t)n_pad * rowb, s) : LZ_OK;
        return hp ? halo_exchange(h, *hp, X, rowb, s) : LZ_OK;
    };
    const int64_t lcl = (lc >= 0 && lc < n) ? lc : -1;
    // ---- beta_0 from the global Gram of B: g0 (every rank on the default
    // shape), summed by the first launch's consumers
    // and all-reduced with its S1; otherwise a Gram, its own all-reduce and
    // sqrtm first.  V_0 = B with its halo / in every slot
    LZ_ARG_CHECK(!g0 || wp.var == 111, "beta_0's Gram in the first launch: the default shape only (internal)");
    if (!g0) {
        int np = 0;
        LZ_TRY(gram_partials<double>(h, n, 16, B, B, 16, &np));
        LZ_TRY(gram_finish<double>(h, 16, np, 0, slab));
        LZ_TRY(allreduce(bb));
        LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, 1, beta, binv[0], nullptr, slab));
    }
    if (ag) {
        if (cm) LZ_TRY(cm->allgather(B, X0, (size_t)n_pad * rowb, h->stream));
        else LZ_HIP_TRY(hipMemcpyAsync(slot, B, (size_t)n * rowb, hipMemcpyDeviceToDevice, h->stream));
    } else {
        LZ_HIP_TRY(hipMemcpyAsync(X0, B, (size_t)n * rowb, hipMemcpyDeviceToDevice, h->stream));
        LZ_TRY(exchange(X0, h->stream));
    }
    LZ_TRY(wf_reset16(h, n, wp));
    // ---- Y_0 = A V_0 (pass 1 only, every tile; g0: and G_0), alpha_0
    int G = 0;
    LZ_TRY(wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, nullptr, nullptr, g0 ? X0 : nullptr, nullptr, nullptr,
                     nullptr, nullptr, X0, Y, 0, &G, nx, 0, T, h->partials2));
    {
        WfSlabs sl;
        sl.add(h->partials2, G);
        LZ_TRY(wf_fold16(h, sl, slab));
    }
    LZ_TRY(allreduce(3 * bb));
    if (g0) {  // beta_0, its inverse, alpha_0, P2 and q_0 in one kernel
        WfAlpha wa;
        wa.part = slab;
        wa.P = 1;
        wa.alpha = alpha;
        wa.P2 = P2;
        wa.V = ag ? slot : X0;
        wa.lc = lcl;
        wa.qrow = q;
        LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, 1, beta, binv[0], nullptr, slab + 2 * bb, nullptr, nullptr, &wa));
    } else {
        LZ_TRY(alpha_wf16(h, slab, 1, binv[0], nullptr, alpha, P2, ag ? slot : X0, lcl, n, q));
    }
    const double *Vm1 = nullptr, *V0 = ag ? slot : X0;
    // all-gather form at N > 1: V_{j+1} into the slot over V_j, V_j into X1 (=
    // W) over V_{j-1}, so the slot can be all-gathered in place.  At one rank
    // there is no all-gather: V_{j+1} goes over V_{j-1}, alternating between
    // X_full and W as in the halo form (no V_j copy).
    const bool sw = ag && h->nranks > 1;
    for (int j = 0; j + 1 < m; ++j) {
        double *Vn = sw ? slot : ((j & 1) ? X0 : X1);
        double *Vg = sw ? X0 : Vn;
        const double *Vprev = sw ? (j ? X1 : nullptr) : Vm1;
        double *Vsave = sw ? X1 : nullptr;
        WfSlabs sl;
        double *part = h->partials2;
        int Gp = 0, Gk = 0, G1 = 0, G2 = 0;
        if (pre) {  // pass 2 of the requested rows' tiles, then their exchange beside the step launch
            const int64_t qa[4] = {0, sh, st, T};
            LZ_TRY(wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, Y, Vprev, V0, Vn, binv[j & 1],
                             j ? P1 : nullptr, P2, Vg, Y, j + 1, &Gp, nx, 0, 0, part, qa, Vsave));
            sl.add(part, Gp);
            part += 3 * (int64_t)Gp * 256;
            LZ_HIP_TRY(hipEventRecord(h->ev_cx, h->stream));
            LZ_HIP_TRY(hipStreamWaitEvent(h->xstream, h->ev_cx, 0));
            LZ_TRY(exchange(Vn, h->xstream));
            LZ_HIP_TRY(hipEventRecord(h->ev_xd, h->xstream));
        }
        // the step launch: pass 2 (the other tiles) + pass 1 of the interior tiles
        const int64_t qk[4] = {pre ? sh : 0, pre ? st : T, T, T};
        LZ_TRY(wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, Y, Vprev, V0, Vn, binv[j & 1], j ? P1 : nullptr,
                         P2, Vg, Y, j + 1, &Gk, nx, t0, t1, part, qk, Vsave));
        sl.add(part, Gk);
        part += 3 * (int64_t)Gk * 256;
        if (exch) {
            // V_{j+1}'s halo rows / peers' slots, then pass 1 of the boundary
            // tiles: [0, t0) on the handle's stream and [t1, T) beside it on the
            // exchange stream (two short launches of a few dozen blocks each,
            // with no waits inside: run one after the other they cost a launch
            // ramp and tail more per step)
            if (pre) LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_xd, 0));
            else LZ_TRY(exchange(Vn, h->stream));
            const bool two = t0 > 0 && t1 < T;
            if (two) LZ_HIP_TRY(hipEventRecord(h->ev_cx, h->stream));
            LZ_TRY(wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, nullptr, Vg, Y, 0, &G1, nx, 0, t0, part));
            sl.add(part, G1);
            part += 3 * (int64_t)G1 * 256;
            if (two) {
                LZ_HIP_TRY(hipStreamWaitEvent(h->xstream, h->ev_cx, 0));
                std::swap(h->stream, h->xstream);  // wf_step16 launches on h->stream
                const int rc = wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, nullptr, nullptr, nullptr, nullptr,
                                         nullptr, nullptr, nullptr, Vg, Y, 0, &G2, nx, t1, T, part);
                std::swap(h->stream, h->xstream);
                LZ_TRY(rc);
                LZ_HIP_TRY(hipEventRecord(h->ev_bd, h->xstream));
                LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_bd, 0));
            } else {
                LZ_TRY(wf_step16(h, n, rp, col, wp.col16, val, pairs, wp, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 nullptr, nullptr, Vg, Y, 0, &G2, nx, t1, T, part));
            }
            sl.add(part, G2);
        }
        LZ_TRY(wf_fold16(h, sl, slab));
        LZ_TRY(allreduce(3 * bb));
        WfAlpha wa;
        wa.part = slab;
        wa.P = 1;
        wa.alpha = alpha + (j + 1) * bb;
        wa.P2 = P2;
        wa.V = Vn;
        wa.lc = lcl;
        wa.qrow = q + (j + 1) * 16;
        LZ_TRY(sqrtm_pair<double>(h, 16, nullptr, 1, beta + (j + 1) * bb, binv[(j + 1) & 1], nullptr, slab + 2 * bb,
                                  binv[j & 1], P1, &wa));
        Vm1 = V0;
        V0 = Vn;
    }
    LZ_HIP_TRY(hipMemcpyAsync(beta + m * bb, binv[(m - 1) & 1], sizeof(double) * bb, hipMemcpyDeviceToDevice,
                              h->stream));
    if (cm) LZ_TRY(cm->fence(h->stream));  // no peer reads this rank's buffers after the call
    return LZ_OK;
}

// The distributed solve itself; the extern "C" wrappers decide on an abort
// (dist_fail).
template <typename T>
static int dist_solve(lz_handle *h, int form, HaloPlan *hp, int64_t n, int64_t n_pad, int64_t nnz, const int64_t *rp,
                      const int32_t *col, const T *val, int b, int m, int64_t lc, const T *B, T *q, T *alpha, T *beta,
                      T *X0, T *X1)
{
    LZ_TRY(solve_begin(h));
    int rc = dist_solve_impl<T>(h, form, hp, n, n_pad, nnz, rp, col, val, b, m, lc, B, q, alpha, beta, X0, X1);
    if (rc == LZ_OK) rc = solve_status(h);
    return rc;
}

}  // namespace lz

using namespace lz;

// A distributed call that fails aborts the handle's communicator when that can
// release a peer.  A virtual-rank group: always -- its abort wakes every rank
// waiting at the host barrier at once (they would otherwise wait until the
// barrier timeout), and the group is a test / rehearsal harness.  RCCL: only
// once this call has issued a collective (Comm::issued moved).  ncclCommAbort
// is permanent -- the caller then destroys the communicator (lz_comm_destroy)
// and initialises a new one with a new unique id -- and RCCL peers blocked in a
// collective return only when they poll ncclCommGetAsyncError or abort
// themselves, so a failure before the first collective (arguments, workspace
// growth, the plans) leaves the communicator usable, and the caller fails every
// rank alike or calls lz_comm_abort.  (Inside the solve, a set-up failure
// joins the ranks' vote -- the solve's first collective -- with ok = 0, so its
// peers return LZ_E_STATE rather than wait; dist_solve_impl.  Argument errors
// the wrappers report before any work are the caller's to make rank-uniform.)
// (LZ_E_DEVICE comes from the status read after the solve's closing fence: no
// peer waits on this rank then, and the communicator stays usable.)
static int dist_fail(lz_handle *h, int rc, uint64_t issued0)
{
    if (rc != LZ_OK && rc != LZ_E_DEVICE && h && h->comm &&
        (h->comm->abort_wakes_peers() || h->comm->issued != issued0))
        h->comm->abort();
    return rc;
}

static uint64_t comm_issued(const lz_handle *h) { return h && h->comm ? h->comm->issued : 0; }

#define LZ_HANDLE_CHECK(h)                                                          \
    do {                                                                            \
        if (!(h)) {                                                                 \
            set_error("handle is NULL");                                           \
            return LZ_E_STATE;                                                      \
        }                                                                           \
        LZ_HIP_TRY(hipSetDevice((h)->device));                                      \
    } while (0)

extern "C" {

const char *lz_last_error(void) { return g_err; }
const char *lz_version(void) { return "lz_hip 0.1 gfx950"; }

int lz_device_ok(int device)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// allocate the handle's workspaces; on any failure the caller frees the
// partly built handle with lz_finalize (no leak on an error path)
static int init_handle(lz_handle *h, int device)
{
    h->device = device;
    hipDeviceProp_t prop;
    LZ_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s, liblz_hip.so is built for gfx950 only", device, prop.gcnArchName);
        return LZ_E_HIP;
    }
    h->n_cu = prop.multiProcessorCount;
    h->partials_cap = (size_t)kMaxPartials * kMaxB * kMaxB;
    LZ_HIP_TRY(hipMalloc(&h->partials, sizeof(double) * h->partials_cap));
    LZ_HIP_TRY(hipMalloc(&h->partials2, sizeof(double) * (256 * kMaxB * kMaxB + 4096 * 256)));
    LZ_HIP_TRY(hipMalloc(&h->scratch, sizeof(double) * 8 * kMaxB * kMaxB));
    LZ_HIP_TRY(hipMalloc(&h->err_flag, 64));
    // (every fill below is stream-ordered and waited for here: later work runs
    // on whatever stream lz_set_stream names, which need not order against the
    // null stream a plain hipMemset uses)
    LZ_HIP_TRY(hipMemsetAsync(h->err_flag, 0, 64, h->stream));
    LZ_HIP_TRY(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
    LZ_HIP_TRY(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    LZ_HIP_TRY(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
    if (const char *pz = getenv("LZ_POISON"); pz && pz[0] == '1') {  // test support: NaN-filled workspaces
        LZ_HIP_TRY(hipMemsetAsync(h->partials, 0xFF, sizeof(double) * h->partials_cap, h->stream));
        LZ_HIP_TRY(hipMemsetAsync(h->partials2, 0xFF, sizeof(double) * (256 * kMaxB * kMaxB + 4096 * 256), h->stream));
        LZ_HIP_TRY(hipMemsetAsync(h->scratch, 0xFF, sizeof(double) * 8 * kMaxB * kMaxB, h->stream));
    }
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    return LZ_OK;
}

int lz_init(int device, lz_handle **out)
{
    LZ_ARG_CHECK(out != nullptr, "out handle pointer is NULL");
    *out = nullptr;
    int count = 0;
    LZ_HIP_TRY(hipGetDeviceCount(&count));
    LZ_ARG_CHECK(device >= 0 && device < count, "device index");
    LZ_HIP_TRY(hipSetDevice(device));
    lz_handle *h = new lz_handle();
    const int rc = init_handle(h, device);
    if (rc != LZ_OK) {
        lz_finalize(h);
        return rc;
    }
    *out = h;
    return LZ_OK;
}

int lz_finalize(lz_handle *h)
{
    if (!h) return LZ_OK;
    (void)hipSetDevice(h->device);
    detach_comm(h);
    (void)hipFree(h->pairs);
    (void)hipFree(h->longq);
    (void)hipFree(h->cm_buf);
    (void)hipFree(h->ybuf);
    (void)hipFree(h->c16buf);
    (void)hipFree(h->wf_deps);
    (void)hipFree(h->wf_flags);
    (void)hipFree(h->fnz_colf);
    (void)hipFree(h->fnz_trow);
    if (h->ev_pool) {
        for (int i = 0; i < h->ev_cap; ++i) (void)hipEventDestroy(h->ev_pool[i]);
        delete[] h->ev_pool;
    }
    (void)hipFree(h->partials);
    (void)hipFree(h->partials2);
    (void)hipFree(h->scratch);
    (void)hipFree(h->err_flag);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->ev_lfork) (void)hipEventDestroy(h->ev_lfork);
    if (h->ev_ljoin) (void)hipEventDestroy(h->ev_ljoin);
    if (h->lstream) (void)hipStreamDestroy(h->lstream);
    if (h->side) (void)hipStreamDestroy(h->side);
    for (hipStream_t s : {h->pf_sg, h->pf_sp})
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    for (hipEvent_t e : {h->ev_pff, h->ev_pfg, h->ev_pfp})
        if (e) (void)hipEventDestroy(e);
    (void)hipFree(h->pf_ctl);
    delete h;
    return LZ_OK;
}

int lz_device_error(lz_handle *h, int *code)
{
    LZ_ARG_CHECK(h && code, "null argument");
    int c = 0;
    LZ_HIP_TRY(hipMemcpyAsync(&c, h->err_flag, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipMemsetAsync(h->err_flag, 0, sizeof(int), h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    *code = c;
    return LZ_OK;
}

int lz_debug_set_device_error(lz_handle *h, int code)
{
    LZ_HANDLE_CHECK(h);
    LZ_HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h->err_flag), code, 1, h->stream));
    return LZ_OK;
}

int lz_debug_fail_next_setup(lz_handle *h, int code)
{
    LZ_HANDLE_CHECK(h);
    h->dbg_setup_fail = code;
    return LZ_OK;
}

__global__ __launch_bounds__(1024) void k_poison_lds(uint32_t pattern)
{
    constexpr int kWords = 160 * 1024 / 4;
    __shared__ uint32_t lds[kWords];
    volatile uint32_t *v = lds;
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) v[i] = pattern;
}

int lz_debug_poison_lds(lz_handle *h, uint32_t pattern)
{
    LZ_HANDLE_CHECK(h);
    hipLaunchKernelGGL(k_poison_lds, dim3(h->n_cu * 4), dim3(1024), 0, h->stream, pattern);
    LZ_LAUNCH_CHECK();
    // and the handle's slab / scratch workspaces (nothing may read them before writing)
    const int byte = (int)(pattern & 0xFF);
    LZ_HIP_TRY(hipMemsetAsync(h->partials, byte, sizeof(double) * h->partials_cap, h->stream));
    LZ_HIP_TRY(hipMemsetAsync(h->partials2, byte, sizeof(double) * (256 * kMaxB * kMaxB + 4096 * 256), h->stream));
    LZ_HIP_TRY(hipMemsetAsync(h->scratch, byte, sizeof(double) * 8 * kMaxB * kMaxB, h->stream));
    return LZ_OK;
}

int lz_prof_enable_mask(lz_handle *h, unsigned class_mask)
{
    LZ_HANDLE_CHECK(h);
    if (class_mask && !h->ev_pool) {
        h->ev_cap = 8192;
        h->ev_pool = new hipEvent_t[h->ev_cap];
        for (int i = 0; i < h->ev_cap; ++i) LZ_HIP_TRY(hipEventCreate(&h->ev_pool[i]));
    }
    h->prof = class_mask != 0;
    h->prof_mask = class_mask;
    h->ev_used = 0;
    return LZ_OK;
}

int lz_prof_enable(lz_handle *h, int on) { return lz_prof_enable_mask(h, on ? ~0u : 0u); }

int lz_prof_read(lz_handle *h, int cls, double *ms_total, int *count)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(ms_total && count, "NULL outputs");
    *ms_total = 0.0;
    *count = 0;
    if (!h->ev_pool || h->ev_used == 0) return LZ_OK;
    LZ_HIP_TRY(hipEventSynchronize(h->ev_pool[h->ev_used - 1]));
    for (int i = 0; i < h->ev_used; i += 2) {
        if (h->ev_class[i / 2] != cls) continue;
        float ms = 0.f;
        LZ_HIP_TRY(hipEventElapsedTime(&ms, h->ev_pool[i], h->ev_pool[i + 1]));
        *ms_total += ms;
        *count += 1;
    }
    return LZ_OK;
}

int lz_set_final_state(lz_handle *h, int on)
{
    LZ_HANDLE_CHECK(h);
    h->final_state = on ? 1 : 0;
    return LZ_OK;
}

int lz_set_stream(lz_handle *h, void *stream)
{
    LZ_HANDLE_CHECK(h);
    h->stream = reinterpret_cast<hipStream_t>(stream);
    return LZ_OK;
}

int lz_csr_spmm(lz_handle *h, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *rp,
                const int32_t *col, const void *val, lz_dtype dtype, int b, const void *X,
                int64_t ldx, lz_layout layout, void *Y, int64_t ldy)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(check_csr(n_rows, nnz, rp, col, val));
    LZ_ARG_CHECK(b >= 1 && b <= kMaxB, "b in [1,64]");
    LZ_ARG_CHECK(X && Y, "X/Y NULL");
    if (layout == LZ_ROW_MAJOR) {
        LZ_ARG_CHECK(ldx >= b && ldy >= b, "row-major ld >= b");
        if (dtype == LZ_F64)
            return spmm_rm<double>(h, n_rows, nnz, rp, col, (const double *)val, b, (const double *)X,
                                   ldx, n_cols, (double *)Y, ldy);
        return spmm_rm<float>(h, n_rows, nnz, rp, col, (const float *)val, b, (const float *)X, ldx,
                              n_cols, (float *)Y, ldy);
    }
    LZ_ARG_CHECK(ldx >= n_cols && ldy >= n_rows, "column-major ld >= rows");
    if (dtype == LZ_F64)
        return spmm_cm<double>(h, n_rows, nnz, rp, col, (const double *)val, b, (const double *)X, ldx, n_cols,
                               (double *)Y, ldy);
    return spmm_cm<float>(h, n_rows, nnz, rp, col, (const float *)val, b, (const float *)X, ldx, n_cols,
                          (float *)Y, ldy);
}

int lz_to_row_major(lz_handle *h, int64_t rows, int b, lz_dtype dtype, const void *X, int64_t ldx, void *Y)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(X && Y && X != Y, "to_row_major: X, Y distinct, not NULL");
    if (dtype == LZ_F64) return to_row_major<double>(h, rows, b, (const double *)X, ldx, (double *)Y);
    return to_row_major<float>(h, rows, b, (const float *)X, ldx, (float *)Y);
}

int lz_to_col_major(lz_handle *h, int64_t rows, int b, lz_dtype dtype, const void *X, void *Y, int64_t ldy)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(X && Y && X != Y, "to_col_major: X, Y distinct, not NULL");
    if (dtype == LZ_F64) return to_col_major<double>(h, rows, b, (const double *)X, ldy, (double *)Y);
    return to_col_major<float>(h, rows, b, (const float *)X, ldy, (float *)Y);
}

int lz_csr_spmv(lz_handle *h, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *rp,
                const int32_t *col, const void *val, lz_dtype dtype, const void *x, void *y)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(check_csr(n_rows, nnz, rp, col, val));
    LZ_ARG_CHECK(x && y, "x/y NULL");
    (void)n_cols;
    if (dtype == LZ_F64)
        return spmv<double>(h, n_rows, rp, col, (const double *)val, (const double *)x,
                            (double *)y, nnz);
    return spmv<float>(h, n_rows, rp, col, (const float *)val, (const float *)x, (float *)y, nnz);
}

int lz_gram(lz_handle *h, int64_t n, int b, lz_dtype dtype, const void *W, int64_t ld, void *R)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(W && R && b >= 1 && b <= kMaxB && ld >= b && n >= 0, "gram args");
    int P = 0;
    if (dtype == LZ_F64) {
        LZ_TRY(gram_partials<double>(h, n, b, (const double *)W, (const double *)W, ld, &P));
        return gram_finish<double>(h, b, P, 0, (double *)R);
    }
    LZ_TRY(gram_partials<float>(h, n, b, (const float *)W, (const float *)W, ld, &P));
    return gram_finish<float>(h, b, P, 0, (float *)R);
}

int lz_sym_cross_gram(lz_handle *h, int64_t n, int b, lz_dtype dtype, const void *W, const void *Q,
                      int64_t ld, void *R)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(W && Q && R && b >= 1 && b <= kMaxB && ld >= b && n >= 0, "cross gram args");
    int P = 0;
    if (dtype == LZ_F64) {
        LZ_TRY(gram_partials<double>(h, n, b, (const double *)W, (const double *)Q, ld, &P));
        return gram_finish<double>(h, b, P, 1, (double *)R);
    }
    LZ_TRY(gram_partials<float>(h, n, b, (const float *)W, (const float *)Q, ld, &P));
    return gram_finish<float>(h, b, P, 1, (float *)R);
}

int lz_tsmm(lz_handle *h, int64_t n, int b, lz_dtype dtype, double beta, double alpha,
            const void *Q, const void *S, void *W, int64_t ld)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(Q && S && W && Q != W, "tsmm pointers (Q must not alias W)");
    if (dtype == LZ_F64)
        return tsmm<double>(h, n, b, beta, alpha, (const double *)Q, (const double *)S,
                            (double *)W, ld);
    return tsmm<float>(h, n, b, (float)beta, (float)alpha, (const float *)Q, (const float *)S,
                       (float *)W, ld);
}

int lz_sqrtm_pair(lz_handle *h, int b, lz_dtype dtype, const void *G, void *beta, void *beta_inv,
                  void *eigval)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(G && b >= 1 && b <= 32, "sqrtm args");
    if (dtype == LZ_F64)
        return sqrtm_pair<double>(h, b, (const double *)G, 0, (double *)beta, (double *)beta_inv,
                                  (double *)eigval);
    return sqrtm_pair<float>(h, b, (const float *)G, 0, (float *)beta, (float *)beta_inv,
                             (float *)eigval);
}

int lz_copy_row(lz_handle *h, int b, lz_dtype dtype, const void *Q, int64_t ld, lz_layout layout,
                int64_t lc, void *q, int64_t start)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(Q && q && b >= 1 && b <= kMaxB && lc >= 0, "copy_row args");
    if (dtype == LZ_F64)
        return copy_row<double>(h, b, (const double *)Q, ld, layout == LZ_COL_MAJOR, lc,
                                (double *)q + start);
    return copy_row<float>(h, b, (const float *)Q, ld, layout == LZ_COL_MAJOR, lc,
                           (float *)q + start);
}

static int block_args(int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                      const void *val, int b, int m, int64_t lc, const void *B, void *q,
                      void *alpha, void *beta, void *Q0, void *Q1, void *W)
{
    LZ_TRY(check_csr(n, nnz, rp, col, val));
    LZ_ARG_CHECK(n >= 1, "n >= 1");
    LZ_ARG_CHECK(b >= 1 && b <= 32, "block Lanczos supports 1 <= b <= 32");
    LZ_ARG_CHECK(m >= 1, "m >= 1");
    LZ_ARG_CHECK(lc >= 0 && lc < n, "lc must be a row index");
    LZ_ARG_CHECK(B && q && alpha && beta && Q0 && Q1 && W, "NULL buffer");
    LZ_ARG_CHECK(Q0 != Q1 && Q0 != W && Q1 != W && B != Q0 && B != Q1 && B != W,
                 "B, Q0, Q1, W must be distinct buffers");
    return LZ_OK;
}

int lz_block_lanczos_unfused(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp,
                             const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                             int64_t lc, const void *B, void *q, void *alpha, void *beta, void *Q0,
                             void *Q1, void *W)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(block_args(n, nnz, rp, col, val, b, m, lc, B, q, alpha, beta, Q0, Q1, W));
    if (dtype == LZ_F64)
        return block_lanczos_unfused<double>(h, n, nnz, rp, col, (const double *)val, b, m, lc,
                                             (const double *)B, (double *)q, (double *)alpha,
                                             (double *)beta, (double *)Q0, (double *)Q1,
                                             (double *)W);
    return block_lanczos_unfused<float>(h, n, nnz, rp, col, (const float *)val, b, m, lc,
                                        (const float *)B, (float *)q, (float *)alpha,
                                        (float *)beta, (float *)Q0, (float *)Q1, (float *)W);
}

int lz_block_lanczos(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                     const void *val, lz_dtype dtype, int b, int m, int64_t lc, const void *B,
                     void *q, void *alpha, void *beta, void *Q0, void *Q1, void *W)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(block_args(n, nnz, rp, col, val, b, m, lc, B, q, alpha, beta, Q0, Q1, W));
    if (dtype == LZ_F64 && b == 16) {
        LZ_TRY(solve_begin(h));
        LZ_TRY(block_lanczos_fused16(h, n, nnz, rp, col, (const double *)val, m, lc, (const double *)B, (double *)q,
                                     (double *)alpha, (double *)beta, (double *)Q0, (double *)Q1, (double *)W));
        return solve_status(h);
    }
    if (dtype == LZ_F64)
        return block_lanczos_sep<double>(h, n, nnz, rp, col, (const double *)val, b, m, lc, (const double *)B,
                                         (double *)q, (double *)alpha, (double *)beta, (double *)Q0, (double *)Q1,
                                         (double *)W);
    return block_lanczos_sep<float>(h, n, nnz, rp, col, (const float *)val, b, m, lc, (const float *)B, (float *)q,
                                    (float *)alpha, (float *)beta, (float *)Q0, (float *)Q1, (float *)W);
}

int lz_vector_lanczos(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                      const void *val, lz_dtype dtype, int m, int64_t lc, const void *bvec,
                      void *q, void *alpha, void *beta, void *q0, void *q1, void *w)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(check_csr(n, nnz, rp, col, val));
    LZ_ARG_CHECK(n >= 1 && m >= 1 && lc >= 0 && lc < n, "vector Lanczos sizes");
    LZ_ARG_CHECK(bvec && q && alpha && beta && q0 && q1 && w, "NULL buffer");
    LZ_ARG_CHECK(bvec != q0 && bvec != q1 && bvec != w && q0 != q1 && q0 != w && q1 != w,
                 "b, q0, q1, w must be distinct buffers");
    if (dtype == LZ_F64)
        return vector_lanczos_dev<double>(h, n, nnz, rp, col, (const double *)val, m, lc,
                                          (const double *)bvec, (double *)q, (double *)alpha,
                                          (double *)beta, (double *)q0, (double *)q1, (double *)w);
    return vector_lanczos_dev<float>(h, n, nnz, rp, col, (const float *)val, m, lc, (const float *)bvec,
                                     (float *)q, (float *)alpha, (float *)beta, (float *)q0, (float *)q1,
                                     (float *)w);
}

int lz_fdtd_block(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                  const void *val, lz_dtype dtype, int b, const void *U0, int64_t steps,
                  double T_end, int64_t lc, void *U, void *D, void *out)
{
    LZ_HANDLE_CHECK(h);
    LZ_TRY(check_csr(n, nnz, rp, col, val));
    LZ_ARG_CHECK(steps >= 1 && lc >= 0 && lc < n && U0 && U && D && out, "fdtd args");
    if (dtype == LZ_F64)
        return fdtd_block<double>(h, n, nnz, rp, col, (const double *)val, b, (const double *)U0, steps,
                                  T_end, lc, (double *)U, (double *)D, (double *)out);
    return fdtd_block<float>(h, n, nnz, rp, col, (const float *)val, b, (const float *)U0, steps,
                             T_end, lc, (float *)U, (float *)D, (float *)out);
}

int lz_comm_init(lz_handle *h, int nranks, int rank, const unsigned char id[128])
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks && id, "comm args");
    LZ_ARG_CHECK(h->comm == nullptr, "handle already has a communicator (lz_comm_destroy first)");
    Comm *c = nullptr;
    LZ_TRY(make_rccl_comm(nranks, rank, id, &c));
    return attach_comm(h, c);
}

int lz_debug_last_split(lz_handle *h, int64_t out[2])
{
    LZ_ARG_CHECK(h && out, "NULL argument");
    out[0] = h->last_split[0];
    out[1] = h->last_split[1];
    return LZ_OK;
}

int lz_debug_last_wf(lz_handle *h, int out[2])
{
    LZ_ARG_CHECK(h && out, "NULL argument");
    out[0] = h->last_wf;
    out[1] = h->last_wf_pre;
    return LZ_OK;
}

int lz_debug_wf_plan(lz_handle *h, int64_t n, int64_t nnz, const int64_t *row_ptr, const int32_t *col_idx,
                     int64_t nx, int64_t xoff, int32_t *deps_out, int16_t *col16_out, int32_t info[8])
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(row_ptr && col_idx && deps_out && col16_out && info, "NULL argument");
    lz::WfPlan wp;
    LZ_TRY(lz::wf_plan16(h, n, nnz, row_ptr, col_idx, &wp, nx, xoff));
    const int64_t T = wp.tr > 0 ? lz::ceil_div(n, (int64_t)wp.tr) : 0;
    // outputs only from this call's plan (never a stale earlier one): deps and
    // spans when the plan kernel ran, the 16-bit columns when they were kept;
    // zero-filled otherwise (the caller sized deps_out for T = n / 16 + 2 tiles)
    int sp[4] = {0, 0, 0, 0};
    if (wp.planned && T > 0) {
        LZ_HIP_TRY(hipMemcpyAsync(deps_out, h->wf_deps, sizeof(int32_t) * 2 * (size_t)T, hipMemcpyDeviceToDevice,
                                  h->stream));
        LZ_HIP_TRY(hipMemcpyAsync(sp, h->err_flag + 12, sizeof(sp), hipMemcpyDeviceToHost, h->stream));
    } else if (T > 0) {
        LZ_HIP_TRY(hipMemsetAsync(deps_out, 0, sizeof(int32_t) * 2 * (size_t)T, h->stream));
    }
    if (nnz > 0) {
        if (wp.col16)
            LZ_HIP_TRY(hipMemcpyAsync(col16_out, wp.col16, sizeof(int16_t) * (size_t)nnz, hipMemcpyDeviceToDevice,
                                      h->stream));
        else
            LZ_HIP_TRY(hipMemsetAsync(col16_out, 0, sizeof(int16_t) * (size_t)nnz, h->stream));
    }
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    info[0] = wp.ok ? 1 : 0;
    info[1] = wp.col16 ? 1 : 0;
    info[2] = (int32_t)T;
    info[3] = wp.tr;
    for (int i = 0; i < 4; ++i) info[4 + i] = sp[i];
    return LZ_OK;
}

int lz_comm_destroy(lz_handle *h)
{
    LZ_HANDLE_CHECK(h);
    detach_comm(h);
    return LZ_OK;
}

static int dist_args(lz_handle *h, lz_dtype dtype, int b, int m)
{
    LZ_ARG_CHECK(dtype == LZ_F64 || dtype == LZ_F32, "dtype");
    LZ_ARG_CHECK(b >= 1 && b <= 32, "distributed block Lanczos: 1 <= b <= 32");
    LZ_ARG_CHECK(m >= 1, "m >= 1");
    (void)h;
    return LZ_OK;
}

static int lz_block_lanczos_dist_impl(lz_handle *h, int64_t n_local, int64_t n_pad, int64_t n_global,
                          int64_t nnz_local, const int64_t *rp, const int32_t *col,
                          const void *val, lz_dtype dtype, int b, int m, int64_t lc_local,
                          int lc_rank, const void *B_local, void *q, void *alpha, void *beta,
                          void *Q0, void *Q1, void *W, void *X_full)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(h->comm != nullptr, "lz_comm_init first");
    LZ_TRY(check_csr(n_local, nnz_local, rp, col, val));
    LZ_TRY(dist_args(h, dtype, b, m));
    LZ_ARG_CHECK(n_local >= 1 && n_pad >= n_local && n_pad * h->nranks == n_global,
                 "dist sizes: n_pad >= n_local >= 1 and n_global == n_pad * nranks (padded numbering)");
    LZ_ARG_CHECK(B_local && q && alpha && beta && W && X_full, "NULL buffer");
    LZ_ARG_CHECK(W != X_full && B_local != X_full && B_local != W, "B_local, W, X_full must be distinct");
    (void)Q0;
    (void)Q1;
    const int64_t lc = (lc_rank == h->rank) ? lc_local : -1;
    if (dtype == LZ_F64)
        return dist_solve<double>(h, kFormAllgather, nullptr, n_local, n_pad, nnz_local, rp, col, (const double *)val, b,
                                  m, lc, (const double *)B_local, (double *)q, (double *)alpha, (double *)beta,
                                  (double *)X_full, (double *)W);
    return dist_solve<float>(h, kFormAllgather, nullptr, n_local, n_pad, nnz_local, rp, col, (const float *)val, b, m,
                             lc, (const float *)B_local, (float *)q, (float *)alpha, (float *)beta, (float *)X_full,
                             (float *)W);
}

int lz_block_lanczos_dist(lz_handle *h, int64_t n_local, int64_t n_pad, int64_t n_global,
                          int64_t nnz_local, const int64_t *rp, const int32_t *col,
                          const void *val, lz_dtype dtype, int b, int m, int64_t lc_local,
                          int lc_rank, const void *B_local, void *q, void *alpha, void *beta,
                          void *Q0, void *Q1, void *W, void *X_full)
{
    const uint64_t issued0 = comm_issued(h);
    const int rc = lz_block_lanczos_dist_impl(h, n_local, n_pad, n_global, nnz_local, rp, col, val, dtype, b, m,
                                              lc_local, lc_rank, B_local, q, alpha, beta, Q0, Q1, W, X_full);
    return dist_fail(h, rc, issued0);
}

static int halo_init_impl(lz_handle *h, int64_t row0, int64_t n_local, const int64_t *recv_counts,
                          const int32_t *halo_rows)
{
    LZ_ARG_CHECK(n_local >= 0 && row0 >= 0 && recv_counts, "halo args");
    const int nr = h->nranks;
    LZ_ARG_CHECK(nr == 1 || h->comm != nullptr, "lz_comm_init first");
    LZ_ARG_CHECK(recv_counts[h->rank] == 0, "recv_counts[rank] must be 0 (own rows are not halo)");
    halo_free(h);
    HaloPlan *hp = new HaloPlan();
    h->halo = hp;
    hp->n_local = n_local;
    hp->roff.assign(nr + 1, 0);
    hp->soff.assign(nr + 1, 0);
    for (int p = 0; p < nr; ++p) {
        LZ_ARG_CHECK(recv_counts[p] >= 0, "negative recv count");
        hp->roff[p + 1] = hp->roff[p] + recv_counts[p];
    }
    hp->n_halo = hp->roff[nr];
    LZ_ARG_CHECK(hp->n_halo == 0 || halo_rows, "halo_rows is NULL");
    LZ_ARG_CHECK(n_local + hp->n_halo < (1LL << 31), "n_local + n_halo must fit int32 columns");
    if (nr == 1) return LZ_OK;
    Comm *cm = h->comm;
    // 1. counts: rank p tells rank q how many of q's rows it needs
    int64_t *dcnt = nullptr;
    LZ_HIP_TRY(hipMalloc(&dcnt, sizeof(int64_t) * 2 * nr));
    std::vector<int64_t> scnt(nr, 0);
    int rc = LZ_OK;
    do {
        // (stream-ordered: a plain hipMemset / pageable hipMemcpy need not be
        // done, or ordered, before a non-blocking stream's exchange reads them)
        if (hipMemcpyAsync(dcnt, recv_counts, sizeof(int64_t) * nr, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
            hipMemsetAsync(dcnt + nr, 0, sizeof(int64_t) * nr, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess) {
            set_error("lz_halo_init: staging counts failed");
            rc = LZ_E_HIP;
            break;
        }
        std::vector<P2POp> ops;
        for (int p = 0; p < nr; ++p)
            if (p != h->rank) ops.push_back(P2POp{p, dcnt + p, sizeof(int64_t), dcnt + nr + p, sizeof(int64_t)});
        rc = cm->exchange(ops.data(), (int)ops.size(), h->stream);
        if (rc != LZ_OK) break;
        if (hipStreamSynchronize(h->stream) != hipSuccess ||
            hipMemcpyAsync(scnt.data(), dcnt + nr, sizeof(int64_t) * nr, hipMemcpyDeviceToHost, h->stream) !=
                hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess) {
            set_error("lz_halo_init: reading counts failed");
            rc = LZ_E_HIP;
        }
    } while (0);
    if (rc == LZ_OK) rc = cm->fence(h->stream);  // peers are done reading dcnt
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(dcnt);
    if (rc != LZ_OK) return rc;
    for (int p = 0; p < nr; ++p) {
        LZ_ARG_CHECK(scnt[p] >= 0 && scnt[p] <= n_local, "peer requested more rows than this rank owns");
        hp->soff[p + 1] = hp->soff[p] + scnt[p];
    }
    hp->n_send = hp->soff[nr];
    // 2. the request lists (global rows) travel to their owners
    int32_t *dreq = nullptr;
    LZ_HIP_TRY(hipMalloc(&dreq, sizeof(int32_t) * std::max<int64_t>(1, hp->n_halo)));
    LZ_HIP_TRY(hipMalloc(&hp->send_idx, sizeof(int32_t) * std::max<int64_t>(1, hp->n_send)));
    std::vector<int32_t> sidx(hp->n_send);
    do {
        if (hp->n_halo &&
            (hipMemcpyAsync(dreq, halo_rows, sizeof(int32_t) * hp->n_halo, hipMemcpyHostToDevice, h->stream) !=
                 hipSuccess ||
             hipStreamSynchronize(h->stream) != hipSuccess)) {
            set_error("lz_halo_init: staging requests failed");
            rc = LZ_E_HIP;
            break;
        }
        std::vector<P2POp> ops;
        for (int p = 0; p < nr; ++p) {
            if (p == h->rank) continue;
            const int64_t sc = hp->soff[p + 1] - hp->soff[p], rcv = hp->roff[p + 1] - hp->roff[p];
            if (sc || rcv)
                ops.push_back(P2POp{p, dreq + hp->roff[p], sizeof(int32_t) * (size_t)rcv, hp->send_idx + hp->soff[p],
                                    sizeof(int32_t) * (size_t)sc});
        }
        rc = cm->exchange(ops.data(), (int)ops.size(), h->stream);
        if (rc != LZ_OK) break;
        if (hipStreamSynchronize(h->stream) != hipSuccess ||
            (hp->n_send && (hipMemcpyAsync(sidx.data(), hp->send_idx, sizeof(int32_t) * hp->n_send,
                                           hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                            hipStreamSynchronize(h->stream) != hipSuccess))) {
            set_error("lz_halo_init: reading requests failed");
            rc = LZ_E_HIP;
        }
    } while (0);
    if (rc == LZ_OK) rc = cm->fence(h->stream);  // peers are done reading dreq
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(dreq);
    if (rc != LZ_OK) return rc;
    // 3. global -> local row; every requested row must be ours
    hp->send_head = 0;
    hp->send_tail = n_local;
    for (int64_t i = 0; i < hp->n_send; ++i) {
        const int64_t g = (int64_t)sidx[i] - row0;
        LZ_ARG_CHECK(g >= 0 && g < n_local, "a peer requested a row this rank does not own");
        sidx[i] = (int32_t)g;
        if (2 * g < n_local) hp->send_head = std::max(hp->send_head, g + 1);
        else hp->send_tail = std::min(hp->send_tail, g);
    }
    if (hp->n_send) {
        LZ_HIP_TRY(hipMemcpyAsync(hp->send_idx, sidx.data(), sizeof(int32_t) * hp->n_send, hipMemcpyHostToDevice,
                                  h->stream));
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));  // sidx is a local
    }
    return LZ_OK;
}

int lz_halo_init(lz_handle *h, int64_t row0, int64_t n_local, const int64_t *recv_counts,
                 const int32_t *halo_rows)
{
    LZ_HANDLE_CHECK(h);
    const uint64_t issued0 = comm_issued(h);
    const int rc = halo_init_impl(h, row0, n_local, recv_counts, halo_rows);
    if (rc != LZ_OK) halo_free(h);  // never leave a half-built plan behind
    return dist_fail(h, rc, issued0);  // a peer blocked in the same set-up must not wait for this rank
}

int lz_halo_sizes(lz_handle *h, int64_t *n_halo, int64_t *n_send)
{
    LZ_ARG_CHECK(h && h->halo, "lz_halo_init first");
    const HaloPlan *hp = static_cast<const HaloPlan *>(h->halo);
    if (n_halo) *n_halo = hp->n_halo;
    if (n_send) *n_send = hp->n_send;
    return LZ_OK;
}

int lz_halo_exchange(lz_handle *h, lz_dtype dtype, int b, void *X)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(h->halo, "lz_halo_init first");
    LZ_ARG_CHECK((dtype == LZ_F64 || dtype == LZ_F32) && b >= 1 && b <= kMaxB && X, "halo exchange args");
    HaloPlan &hp = *static_cast<HaloPlan *>(h->halo);
    const size_t rowb = (size_t)b * (dtype == LZ_F64 ? 8 : 4);
    if (h->comm && h->nranks > 1) LZ_TRY(grow_ws(h, &hp.sendbuf, &hp.send_cap, (size_t)std::max<int64_t>(hp.n_send, 1) * rowb));
    LZ_TRY(halo_exchange(h, hp, X, rowb, h->stream));
    // after the fence no peer still reads this rank's send buffer: the next
    // call may repack (or, at a larger b, reallocate) it.  (Inside the solves
    // the step's all-reduces order the exchanges; they fence once at the end.)
    return h->comm ? h->comm->fence(h->stream) : LZ_OK;
}

static int lz_block_lanczos_halo_impl(lz_handle *h, int64_t n_local, int64_t nnz_local, const int64_t *rp,
                          const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                          int64_t lc_local, int lc_rank, const void *B_local, void *q, void *alpha,
                          void *beta, void *X0, void *X1)
{
    LZ_HANDLE_CHECK(h);
    LZ_ARG_CHECK(h->halo, "lz_halo_init first");
    HaloPlan &hp = *static_cast<HaloPlan *>(h->halo);
    LZ_TRY(check_csr(n_local, nnz_local, rp, col, val));
    LZ_ARG_CHECK(n_local == hp.n_local, "n_local differs from lz_halo_init");
    LZ_TRY(dist_args(h, dtype, b, m));
    LZ_ARG_CHECK(n_local >= 1, "sizes");
    LZ_ARG_CHECK(B_local && q && alpha && beta && X0 && X1 && X0 != X1, "NULL / aliased buffer");
    const int64_t lc = (lc_rank == h->rank) ? lc_local : -1;
    if (dtype == LZ_F64)
        return dist_solve<double>(h, kFormHalo, &hp, n_local, n_local, nnz_local, rp, col, (const double *)val, b, m,
                                  lc, (const double *)B_local, (double *)q, (double *)alpha, (double *)beta,
                                  (double *)X0, (double *)X1);
    return dist_solve<float>(h, kFormHalo, &hp, n_local, n_local, nnz_local, rp, col, (const float *)val, b, m, lc,
                             (const float *)B_local, (float *)q, (float *)alpha, (float *)beta, (float *)X0,
                             (float *)X1);
}

int lz_block_lanczos_halo(lz_handle *h, int64_t n_local, int64_t nnz_local, const int64_t *rp,
                          const int32_t *col, const void *val, lz_dtype dtype, int b, int m,
                          int64_t lc_local, int lc_rank, const void *B_local, void *q, void *alpha,
                          void *beta, void *X0, void *X1)
{
    const uint64_t issued0 = comm_issued(h);
    const int rc = lz_block_lanczos_halo_impl(h, n_local, nnz_local, rp, col, val, dtype, b, m, lc_local, lc_rank,
                                              B_local, q, alpha, beta, X0, X1);
    return dist_fail(h, rc, issued0);
}

}  // extern "C"
