// lz_internal.hpp -- internal (C++) entry points between the .hip units.
#pragma once
#include "lz_common.hpp"

namespace lz {

// ---- sparse (lz_spmm.hip)
template <typename T>
int spmm_rm(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy,
            bool ycm = false);  // nx: rows of X; ycm: Y column-major (leading dimension ldy), b >= 2
template <typename T>
int spmm_cm(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy);  // nx: rows of X
// column-major rows x b (ld >= rows) -> row-major rows x b (ld = b)
template <typename T>
int to_row_major(lz_handle *h, int64_t rows, int b, const T *src, int64_t ld, T *dst);
template <typename T>
int spmv(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, const T *x,
         T *y, int64_t nnz_hint);

// ---- dense (lz_dense.hip)
// partial b x b products of X^T Y, one slab per workgroup, into h->partials;
// returns the number of slabs in *nparts.
template <typename T>
int gram_partials(lz_handle *h, int64_t n, int b, const T *X, const T *Y, int64_t ld, int *nparts);
// reduce nparts slabs (fixed order); mode 0: R = sum, mode 1: R = 0.5 (S + S^T);
// L != null: also LR = L * R (b x b)
template <typename T>
int gram_finish(lz_handle *h, int b, int nparts, int mode, T *R, const double *slabs = nullptr,
                const T *L = nullptr, T *LR = nullptr);
// The wavefront step's alpha products (lz_wf.hip), folded into the sqrtm
// launch: S1, S2 = sums of the P slabs at part, part + 256 P; alpha =
// sym(binv (S1 binv - S2 P1)), P2 = binv alpha, qrow = V[lc] binv (lc < 0: none)
struct WfAlpha {
    const double *part = nullptr;
    int P = 0;
    double *alpha = nullptr, *P2 = nullptr;
    const double *V = nullptr;
    int64_t lc = -1;
    double *qrow = nullptr;
};
// symmetric square root pair of G (device double b x b) or, when nparts > 0,
// of the sum of the nparts slabs in h->partials.  L != null (b in {8,16,32}):
// also LB = L * beta.  wa (b = 16): also the wavefront alpha products with
// binv = beta_inv and P1 = LB.
template <typename T>
int sqrtm_pair(lz_handle *h, int b, const T *G, int nparts, T *beta, T *beta_inv, T *eig,
               const double *slabs = nullptr, const T *L = nullptr, T *LB = nullptr,
               const WfAlpha *wa = nullptr);
// W = sw*W + sq*Q*S
template <typename T>
int tsmm(lz_handle *h, int64_t n, int b, T sw, T sq, const T *Q, const T *S, T *W, int64_t ld);
template <typename T>
int copy_row(lz_handle *h, int b, const T *Q, int64_t ld, int col_major, int64_t lc, T *q);
// the reference's post-call state (block_lanczos.hpp:145,159,162): Q0 (and Q1
// when non-null) = Vq binv; W = Y binv - Vp P1 - Vq P2 (Y != null; Vp may be
// null) or W = Wm.  Row-local: inputs may alias outputs.  b <= 32.
template <typename T>
int final_state(lz_handle *h, int64_t n, int b, const T *Y, const T *Vp, const T *Vq, const T *Wm, const T *binv,
                const T *P1, const T *P2, T *Wout, T *Q0, T *Q1);
// row-major rows x b (ld b) -> column-major with leading dimension ld >= rows
template <typename T>
int to_col_major(lz_handle *h, int64_t rows, int b, const T *src, int64_t ld, T *dst);

// ---- fused block-Lanczos passes, b = 16 fp64 (lz_fused.hip)
// Q-free form: Q_j = W_j beta_j^-1 is formed in registers wherever it is used
// and never stored.
// Pass 1: Y = A*Wg; Q_j[r] = Wown[r]*binv; Wn[r] = Y[r]*binv - Wprev[r]*P1
// (P1 = beta_{j-1}^-1 beta_j, so Wprev[r]*P1 = Q_{j-1}[r] beta_j; none at j = 0);
// slabs of Q_j^T Wn; row probe of Q_j.  nx: rows of Wg.  Wown: the rows r of Wg
// this rank owns (== Wg single-GPU).  Wprev may be the Wn buffer (in place).
int fused_spmm16(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col,
                 const double *val, const double *Wg, int64_t nx, const double *Wown, const double *Wprev,
                 double *Wn, const double *binv, const double *P1, int64_t lc, double *qrow, int *nparts,
                 const uint64_t *pairs, int64_t nnz, int64_t row_off, int win, int slab_off = 0,
                 const int16_t *col16 = nullptr);
// col16 (col16_plan, once per solve): the columns as int16 offsets from each
// 16-row strip's own row (row_off + strip start); nullptr: 32-bit columns.
// Stages 2 B per column instead of 4 (A: 10 B per nonzero instead of 12).
int col16_plan(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, int64_t row_off,
               const int16_t **out);
// slab_off: this launch's folded slabs go to h->partials2 + slab_off * 256 (a
// pass split over row ranges writes its launches' slabs side by side); the
// 64-bit fallback (gather source past 2^24 rows, no window) needs slab_off 0.
// Whether the buffer-addressed kernels (slab per block, at most n_cu) apply:
bool fused16_direct(int64_t nx, int win);
// gather source of 2^24+ rows: does every strip's column set fit its window?
// (row_off: X row of local row 0; synchronises the stream once)
int gather_window_ok(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, int64_t nx, int64_t row_off,
                     bool *ok);
// per-16-row-strip row order by length for fused_spmm16's `pairs` (once per solve)
int strip_pairs(lz_handle *h, int64_t n, const int64_t *rp, const uint64_t **out);
// Pass 2: Wn <- Wn - Wcur*P2 (P2 = beta_j^-1 alpha_j, so Wcur*P2 = Q_j alpha_j);
// slabs of Wn^T Wn.
int fused_update16(lz_handle *h, int64_t n, double *Wn, const double *Wcur, const double *P2,
                   int *nparts);
int fused_update16_swap(lz_handle *h, int64_t n, double *Wn, double *Xown, const double *alpha, int *nparts);
// C = A*B, 16 x 16 row-major fp64, on the stream
int mm16(lz_handle *h, const double *A, const double *B, double *C);

// ---- wavefront step, b = 16 fp64, one GPU (lz_wf.hip): pass 2 of step j and
// pass 1 of step j + 1 in one launch (see the file header)
struct WfPlan {
    bool ok = false;       // the wavefront step applies (n < 2^24, narrow column spans)
    int hback = 0, hfwd = 0;  // max tiles a tile's columns reach below / above it
    int nc = 12, tr = 192;    // consumers per block, rows per tile (16 nc)
    int var = 0;              // measurement shape (LZ_WF_SHAPE 104 / 111), 0: the standard ones
    const int16_t *col16 = nullptr;  // pass 1's 16-bit columns (made in the same pass), or null
    int64_t xoff = 0;         // gather-source row of local row 0 (the all-gather form's slot)
    bool planned = false;     // the plan kernel ran (deps and spans are this call's)
};
// once per solve: per-tile dependency ranges and the 16-bit columns in one pass
// over the CSR columns; synchronises the stream once
bool wf_first_gram(int64_t n, int64_t nnz);
int wf_plan16(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, WfPlan *pl,
              int64_t nx = -1, int64_t xoff = 0);
// (nx: rows of the gather source -- a rank's own + halo rows, or the all-gather
// form's n_pad * N -- default n; xoff: its row of local row 0; 2^24+ rows are
// read through per-strip windows, checked here)
// zero the pass-2 flags (start of a solve; epochs 1, 2, ... follow)
int wf_reset16(lz_handle *h, int64_t n, const WfPlan &pl);
// P2 == nullptr: pass 1 only (Y = A Vg, S1 slabs).  Otherwise V_{j+1} = Yj binv
// - Vprev P1 - Vj P2 into Vout (== Vg; P1 == nullptr: no Vprev term), Y_{j+1}
// = A Vout into Yo (may be Yj).  Slabs at h->partials2: S1 [0, G), S2 [G, 2G),
// G [2G, 3G) of 256 doubles, *nparts = G.
int wf_step16(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const int16_t *col16,
              const double *val, const uint64_t *pairs, const WfPlan &pl, const double *Yj, const double *Vprev,
              const double *Vj, double *Vout, const double *binv, const double *P1, const double *P2,
              const double *Vg, double *Yo, int epoch, int *nparts, int64_t nx = -1, int64_t p1a = 0,
              int64_t p1b = -1, double *part = nullptr, const int64_t *q = nullptr, double *Vsave = nullptr,
              bool qo = false);
// (qo: the one-GPU solve's post-call state -- a pass-2-only launch, Q =
// V_j beta^-1 also stored into Vsave and, when not null, Yo; the default shape
// only, else LZ_E_ARG)
// (nx: rows of Vg, default n; pass 1 over tiles [p1a, p1b), default all; slabs
// at part, default h->partials2; q: pass-2 tiles [q[0], q[1]) u [q[2], q[3]),
// default all -- two ranges only without pass-1 tiles; Vout = Vg + 16 xoff;
// Vsave: pass 2 also stores V_j's rows there (the all-gather form), 111 / wide
// shapes only)
// one step's slab sets (set t: [S1 | S2 | G] of g[t] block slabs at p[t]);
// wf_fold16: out[0..768) = [S1 | S2 | G] summed over every set, in order
struct WfSlabs {
    static constexpr int kMax = 6;
    const double *p[kMax] = {};
    int g[kMax] = {};
    int k = 0;
    void add(const double *ptr, int nslab)
    {
        p[k] = ptr;
        g[k] = nslab;
        ++k;
    }
};
int wf_fold16(lz_handle *h, const WfSlabs &sl, double *out);
// alpha = sym(binv (S1 binv - S2 P1)) (P1 == nullptr: no S2 term), P2 = binv alpha,
// q = V[lc] binv; S1, S2 = the sums of the P slabs at part, part + 256 P
int alpha_wf16(lz_handle *h, const double *part, int P, const double *binv, const double *P1, double *alpha,
               double *P2, const double *V, int64_t lc, int64_t n, double *qrow);

// ---- Q-free dense passes, b = 32 fp32 (lz_fused32.hip), around a separate SpMM Y = A W_j
// pass E: Q_j = Wj binv (registers); Wn = Y binv - Wprev P1 (P1 == null: no
// Wprev term); slabs (32 x 32 doubles, one per block, *nparts <= 2 n_cu) of
// Q_j^T Wn in h->partials; row probe.  Wprev may alias Wn.
int fused_e32(lz_handle *h, int64_t n, const float *Y, const float *Wj, const float *Wprev, float *Wn,
              const float *binv, const float *P1, int64_t lc, float *qrow, int *nparts);
// pass U: Wn <- Wn - Wj P2; slabs of Wn^T Wn
int fused_u32(lz_handle *h, int64_t n, float *Wn, const float *Wj, const float *P2, int *nparts);
// C5 beta^2 step (lz_fused32.hip, lz_dense.hip, lz_spmm.hip)
int fused_el32(lz_handle *h, int64_t n, const float *Wj, const float *U, int *nparts);
int fused_ub32(lz_handle *h, int64_t n, const float *U, const float *Wj, const float *binv, const float *P2,
               float *Wn, int *nparts, float *Qa = nullptr,
               float *Qb = nullptr);
int alpha_b2(lz_handle *h, const double *part, int P, const float *binv, float *alpha, float *P2, const float *Wj,
             int64_t lc, int64_t n, float *qrow);
int m_b2(lz_handle *h, const double *part, int P, const float *binv, float *M);
bool spmm_b2_ok(int64_t n, int64_t nnz, int64_t nx);
int fold_slabs_g(lz_handle *h, const double *part, int64_t P, int bb, int G);  // -> slab count at h->partials2
// plan_slot >= 0: the long-tile list an earlier call of the solve queued (its
// *slot_out), the long-tile pass beside the main kernel (launch_seg)
// cap: the CSR stage (768 or 1024 entries), one per solve (spmm_b2_stage):
// a solve's planned calls must use the stage its first call queued with
int spmm_rm_b2(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const float *val,
               const float *X, int64_t nx, float *Y, const float *Wp, const float *Mm, int plan_slot = -1,
               int *slot_out = nullptr, int cap = 768);
int spmm_b2_stage(lz_handle *h, int64_t n, const int64_t *rp, int *cap);  // host sync
// the long-tile list for that stage, before the solve's first SpMM: every call
// of the solve then runs planned (plan_slot = *slot)
int spmm_b2_plan(lz_handle *h, int64_t n, const int64_t *rp, int cap, int *slot);
// the same two passes at any b <= 32, fp64 or fp32 (b = 32 fp32: the MFMA kernels above;
// otherwise VALU kernels); slabs of b x b doubles in h->partials
template <typename T>
int fused_e_sep(lz_handle *h, int64_t n, int b, const T *Y, const T *Wj, const T *Wprev, T *Wn, const T *binv,
                const T *P1, int64_t lc, T *qrow, int *nparts);
template <typename T>
int fused_u_sep(lz_handle *h, int64_t n, int b, T *Wn, const T *Wj, const T *P2, int *nparts);
// the same pass in SWAP form (VALU, any b <= 32): Xown <- W' - Xown P2, Wn <- Xown (old)
template <typename T>
int fused_u_swap_sep(lz_handle *h, int64_t n, int b, T *Wn, T *Xown, const T *P2, int *nparts);

// fp64 scalar helpers for the vector Lanczos (lz_fused.hip)
template <typename T>
int vector_lanczos_dev(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                       const T *val, int m, int64_t lc, const T *b, T *q, T *alpha, T *beta, T *q0,
                       T *q1, T *w);

}  // namespace lz
