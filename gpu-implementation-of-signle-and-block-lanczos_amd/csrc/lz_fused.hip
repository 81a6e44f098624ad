// lz_fused.hip -- fused block-Lanczos passes (b = 16, fp64) and the fused
// single-vector Lanczos passes, gfx950.
//
// The reference iteration (methods/block_lanczos.hpp:131-166) is seven
// library calls per step, moving ~A + 13 n*b*8 bytes.  Here one step is two
// streaming passes plus two one-workgroup kernels (the Q-free form: the
// residual blocks W_j are kept unnormalised, Q_j is never stored):
//
//   pass 1  k_fused_pp16     Y = A*W_j (gather),  Q_j[r] = W_j[r]*beta_j^-1,
//                            W'[r] = Y[r]*beta_j^-1 - W_{j-1}[r]*P1,
//                            slabs of Q_j^T W' (folded per block in LDS),
//                            row probe                     (A + 3 n*b*8 bytes)
//   finish  k_gram_finish    alpha_j = 0.5 (M + M^T), P2 = beta_j^-1 alpha_j
//   pass 2  k_fused_update16 W' -= W_j*P2, slabs of W'^T W'        (3 n*b*8)
//   finish  k_sqrtm_b        beta_{j+1}, beta_{j+1}^-1 = sqrtm(W'^T W'),
//                            P1 = beta_j^-1 beta_{j+1}
// (k_fused_spmm16, one 128-row tile per block, is the 64-bit-addressed
// fallback for gather sources no 32-bit window covers.)
//
// using A*(W*beta^-1) = (A*W)*beta^-1, so Q_j exists only in registers of the
// SpMM epilogue.  W' overwrites W_{j-1} in place (row r is read and written by
// the same wave); the residual alternates between the W and Q1 buffers.  All
// epilogue products run on v_mfma_f64_16x16x4_f64 (see lz_dense.hip for the
// operand layouts).
#include <cstring>
#include <type_traits>
#include "lz_common.hpp"
#include "lz_internal.hpp"
#include "lz_kernels.hpp"

namespace lz {

// load a 16 x 16 row-major fp64 tile starting at row r0 into the wave's LDS
// tile (row stride 17) and return the MFMA A-operand fragments
// a[kc] = tile[l & 15][4 kc + (l >> 4)].
__device__ __forceinline__ void tile_to_aop(double *T, const double *__restrict__ src, int64_t r0,
                                            int64_t n, int lane, double a[4])
{
    const int64_t row = r0 + (lane >> 2);
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if (row < n) {
        const double2 *s2 = reinterpret_cast<const double2 *>(src + row * 16 + 4 * (lane & 3));
        const double2 x = s2[0], y = s2[1];
        v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) T[(lane >> 2) * 17 + 4 * (lane & 3) + i] = v[i];
    wave_lds_sync();
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) a[kc] = T[(lane & 15) * 17 + 4 * kc + (lane >> 4)];
    wave_lds_sync();
}

// the same in two halves: global -> registers (issue early), registers -> LDS
// -> A operands (later)
__device__ __forceinline__ void tile_load(const double *__restrict__ src, int64_t r0, int64_t n,
                                          int lane, double v[4])
{
    const int64_t row = r0 + (lane >> 2);
    v[0] = v[1] = v[2] = v[3] = 0.0;
    if (row < n) {
        const double2 *s2 = reinterpret_cast<const double2 *>(src + row * 16 + 4 * (lane & 3));
        const double2 x = s2[0], y = s2[1];
        v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
    }
}

__device__ __forceinline__ void tile_regs_to_aop(double *T, const double v[4], int lane, double a[4])
{
#pragma unroll
    for (int i = 0; i < 4; ++i) T[(lane >> 2) * 17 + 4 * (lane & 3) + i] = v[i];
    wave_lds_sync();
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) a[kc] = T[(lane & 15) * 17 + 4 * kc + (lane >> 4)];
    wave_lds_sync();
}

// sum the 8 waves' 16x16 accumulators of the workgroup into its slab
__device__ __forceinline__ void wg_slab(double (*red)[256], d4_t acc, int lane, int w,
                                        double *__restrict__ part)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
    __syncthreads();
    if (threadIdx.x < 256) {
        double s = 0.0;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) s += red[ww][threadIdx.x];
        part[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
    }
}

// One 128-row tile per block (8 waves x 16 rows), XCD remap (xcd_remap), so
// the tiles in flight on an XCD stay a narrow window of rows and the banded X
// gather hits that XCD's L2.  The tile's (col, val) range is staged through LDS
// with coalesced loads; each group of 8 lanes (16 B each = one 128-B X row)
// owns rows 16w+g and 16w+g+8 and issues 8 independent X gathers per step.
// The per-block 16x16 slab of Q_j^T W' goes to part[tile]; lz_fused.hip's
// k_slab_reduce1 folds the slabs in fixed order.
constexpr int kFusedRows = 128, kFusedCap = 2048;
#ifdef LZ_FUSED_PROBE
// per-block phase records of k_fused_spmm16 (scripts/probe/fused_probe.hip):
// staging, gather, epilogue cycles, start and end realtime stamps, XCC id
__device__ long long *lz_fused_probe;
#define LZ_PROBE_T(v) const long long v = clock64()
#else
#define LZ_PROBE_T(v)
#endif

template <bool BUF>
__global__ __launch_bounds__(512, 4) void k_fused_spmm16(
    int64_t n, const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ Wg, int64_t nx,
    const double *__restrict__ Wown, const double *Qbuf,
    double *Wn, const double *__restrict__ binv, const double *__restrict__ beta,
    int64_t lc, double *__restrict__ qrow, double *__restrict__ part)
{
    __shared__ double tile[8][16 * 17];
    __shared__ double red[8][256];
    __shared__ int32_t cs[kFusedCap + 8];
    __shared__ double vs[kFusedCap + 8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane >> 3, p = lane & 7;
    double *T = tile[w];
    const bool has_prev = beta != nullptr;
    double bi_op[4], nb_op[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
        const int idx = (4 * kc + (lane >> 4)) * 16 + (lane & 15);
        bi_op[kc] = binv[idx];
        nb_op[kc] = has_prev ? -beta[idx] : 0.0;
    }
    LZ_PROBE_T(t_start);
#ifdef LZ_FUSED_PROBE
    const long long w_start = wall_clock64();
    long long t_staged = 0;
#endif
    const int64_t u = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t rb = u * kFusedRows;
    const int64_t rend = (rb + kFusedRows < n) ? rb + kFusedRows : n;
    const int64_t kA = rp[rb], kB = rp[rend];
    const int64_t r0 = rb + 16 * w;  // this wave's 16-row tile
    int64_t k0[2], k1[2];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int64_t row = r0 + g + 8 * rr;
        k0[rr] = row < n ? rp[row] : kB;
        k1[rr] = row < n ? rp[row + 1] : kB;
    }
    const double *Xp = Wg + 2 * p;
    // X through a buffer resource (BUF: X < 2 GiB, columns < 2^24): 32-bit
    // offsets, out-of-range offset = masked load (returns 0, no traffic)
    __amdgpu_buffer_rsrc_t xr;
    if constexpr (BUF)
        xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Wg), (short)0,
                                               (int)(nx * 128), 0x00020000);
    const uint32_t lane_off = 16u * (uint32_t)p;
    // the epilogue's own-row tiles (W rows and Q_{j-1} rows) are fetched now so
    // their HBM latency overlaps the gather
    double wv[4], qv[4] = {0.0, 0.0, 0.0, 0.0};
    tile_load(Wown, r0, n, lane, wv);
    if (has_prev) tile_load(Qbuf, r0, n, lane, qv);
    double y[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    for (int64_t c0 = kA; c0 < kB; c0 += kFusedCap) {  // block-uniform
        const int64_t c1 = (c0 + kFusedCap < kB) ? c0 + kFusedCap : kB;
        if (c0 != kA) __syncthreads();
        {  // the chunk's run in one batch of loads, then LDS (+ 8 finite slack slots)
            constexpr int SPT = kFusedCap / 512;
            int32_t ct[SPT];
            double vt[SPT];
#pragma unroll
            for (int q = 0; q < SPT; ++q) {
                const int64_t k = c0 + threadIdx.x + 512 * q;
                ct[q] = k < c1 ? col[k] : 0;
                vt[q] = k < c1 ? val[k] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < SPT; ++q) {
                if (c0 + threadIdx.x + 512 * q < c1) {
                    cs[threadIdx.x + 512 * q] = ct[q];
                    vs[threadIdx.x + 512 * q] = vt[q];
                }
            }
            if (threadIdx.x < 8) {
                cs[c1 - c0 + threadIdx.x] = 0;
                vs[c1 - c0 + threadIdx.x] = 0.0;
            }
        }
        __syncthreads();
#ifdef LZ_FUSED_PROBE
        if (c0 == kA) t_staged = clock64();
#endif
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int a = (int)((k0[rr] > c0 ? k0[rr] : c0) - c0);
            const int e = (int)((k1[rr] < c1 ? k1[rr] : c1) - c0);
            double a0 = y[rr][0], a1 = y[rr][1];
            for (int kb = a; kb < e; kb += 8) {  // group-uniform
                const int cnt = e - kb;
                int32_t cc[8];
                double vv[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    cc[t] = cs[kb + t];
                    vv[t] = vs[kb + t];
                }
                double2 xs[8];
                if constexpr (BUF) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const uint32_t off =
                            t < cnt ? __umul24((unsigned)cc[t], 128u) + lane_off : 0x80000000u;
                        const auto u4 = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
                        __builtin_memcpy(&xs[t], &u4, 16);
                    }
#pragma unroll
                    for (int t = 0; t < 8; ++t) {  // masked entries: x == 0, v finite
                        a0 = fma(vv[t], xs[t].x, a0);
                        a1 = fma(vv[t], xs[t].y, a1);
                    }
                } else {
#pragma unroll
                    for (int t = 0; t < 8; ++t)
                        if (t < cnt) xs[t] = *reinterpret_cast<const double2 *>(Xp + (int64_t)cc[t] * 16);
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        if (t < cnt) {
                            a0 = fma(vv[t], xs[t].x, a0);
                            a1 = fma(vv[t], xs[t].y, a1);
                        }
                    }
                }
            }
            y[rr][0] = a0;
            y[rr][1] = a1;
        }
    }
    LZ_PROBE_T(t_gathered);
    d4_t macc = {0.0, 0.0, 0.0, 0.0};
    if (r0 < n) {  // wave-uniform
        // ---- Y tile -> A operands
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            T[(g + 8 * rr) * 17 + 2 * p] = y[rr][0];
            T[(g + 8 * rr) * 17 + 2 * p + 1] = y[rr][1];
        }
        wave_lds_sync();
        double ya[4], wa[4], qa[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) ya[kc] = T[(lane & 15) * 17 + 4 * kc + (lane >> 4)];
        wave_lds_sync();
        tile_regs_to_aop(T, wv, lane, wa);
        if (has_prev) tile_regs_to_aop(T, qv, lane, qa);
        // ---- epilogue products on the matrix cores
        d4_t q1 = {0.0, 0.0, 0.0, 0.0}, wn = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) q1 = mfma16(wa[kc], bi_op[kc], q1);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) wn = mfma16(ya[kc], bi_op[kc], wn);
        if (has_prev) {
#pragma unroll
            for (int kc = 0; kc < 4; ++kc) wn = mfma16(qa[kc], nb_op[kc], wn);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + (lane >> 4) + 4 * r;
            if (row < n) {
                Wn[r0 * 16 + 64 * r + lane] = wn[r];
                if (row == lc) qrow[lane & 15] = q1[r];
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) macc = mfma16(q1[r], wn[r], macc);
    }
    // slab of this tile, indexed by tile (row order): fixed-order reduction later
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = macc[r];
    __syncthreads();
    if (threadIdx.x < 256) {
        double sum = 0.0;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) sum += red[ww][threadIdx.x];
        part[u * 256 + threadIdx.x] = sum;
    }
#ifdef LZ_FUSED_PROBE
    if (threadIdx.x == 0) {
        const long long t_end = clock64();
        long long *rec = lz_fused_probe + 8 * (int64_t)blockIdx.x;
        rec[0] = t_staged - t_start;
        rec[1] = t_gathered - t_staged;
        rec[2] = t_end - t_gathered;
        rec[3] = w_start;
        rec[4] = wall_clock64();
        rec[5] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_ID2-ish (unused)
    }
#endif
}

// First-level fixed-order fold of P slabs (bb doubles each) into gridDim.x
// slabs: block q sums slabs [q*P/G, (q+1)*P/G) in order.
__global__ __launch_bounds__(256) void k_slab_reduce1(const double *__restrict__ part, int64_t P,
                                                      int bb, double *__restrict__ out)
{
    const int64_t G = gridDim.x, q = blockIdx.x;
    const int64_t s0 = q * P / G, s1 = (q + 1) * P / G;
    for (int e = threadIdx.x; e < bb; e += 256) {
        double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        int64_t s = s0;
        for (; s + 7 < s1; s += 8) {
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] += part[(s + i) * bb + e];
        }
        for (; s < s1; ++s) a[0] += part[s * bb + e];
        out[q * bb + e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
}

// Fold P slabs of bb doubles to G slabs at h->partials2 (block q sums slabs
// [q P / G, (q + 1) P / G) in order): the C5 beta^2 step's 1024 pass slabs
// to 32 before a one-workgroup kernel reads them.
int fold_slabs_g(lz_handle *h, const double *part, int64_t P, int bb, int G)
{
    const int g = (int)std::min<int64_t>(P, G);
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_slab_reduce1, dim3((unsigned)g), dim3(256), 0, h->stream, part, P, bb, h->partials2);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return g;
}

// Fold P slabs of bb (<= 256) doubles to <= 256 slabs at h->partials2 in one
// fixed-order level: block q sums slabs [q P / G, (q + 1) P / G) in order
// (G = min(P, 256); at C3 3,584 pass-1 slabs, 14 per block).  Returns the
// folded count.  (A copy-only first level of <= 4096 blocks was measured
// here before: one launch and 7 MB more per step for nothing.)
static int fold_slabs(lz_handle *h, const double *part, int64_t P, int bb, int *nout)
{
    const int g = (int)std::min<int64_t>(P, 256);
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_slab_reduce1, dim3((unsigned)g), dim3(256), 0, h->stream, part, P, bb, h->partials2);
    *nout = g;
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// SWAP (the all-gather form, lz_api.hip block_lanczos_dist16): Q is this
// rank's slot of the all-gathered block.  W'' goes there (the next all-gather
// is in place) and W_j, the next step's W_{j-1}, goes to Wn over W' -- one
// 1.28 GB write more than the in-place pass, one slab copy (read + write) less
// inside the all-gather.  Each row is read, then written, by the same wave.
template <bool REV, int NW = 8, bool SWAP = false>
__global__ __launch_bounds__(64 * NW) void k_fused_update16(int64_t n, double *__restrict__ Wn,
                                                        std::conditional_t<SWAP, double, const double> *__restrict__ Q,
                                                        const double *__restrict__ alpha,
                                                        double *__restrict__ part)
{
    __shared__ double red[NW][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // permuted contraction order (as k_fused_pp16): step kc, lane l contracts
    // over k = 4 (l >> 4) + kc, so a lane's A operands are 32 contiguous bytes
    // of one W_j row -- two 16-B loads, no LDS transpose
    double na_op[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) na_op[kc] = -alpha[(4 * (lane >> 4) + kc) * 16 + (lane & 15)];
    d4_t gacc = {0.0, 0.0, 0.0, 0.0};
    const int64_t ntile = ceil_div(n, 16);
    XcdSched s(ceil_div(ntile, NW));
    // REV: walk this block's units last-first.  Pass 1 writes Q_j and W' first
    // row to last, so the rows it wrote last are still in the MALL (256 MB)
    // when a reversed pass 2 starts; pass 2's last-written W'' rows (the first
    // rows) are in turn the first the next pass 1 gathers.
    const int64_t cnt = s.begin < s.end ? (s.end - s.begin + s.step - 1) / s.step : 0;
    auto row0 = [&](int64_t k) { return (s.begin + (REV ? cnt - 1 - k : k) * s.step) * (16 * NW) + 16 * w; };
    // one tile ahead in registers: the W' (accumulator layout) and Q rows of
    // tile k+1 are in flight while tile k is computed (vmcnt is in order, so
    // tile k's wait does not cover them)
    auto fetch = [&](int64_t k, d4_t &a, double qv[4]) {
        const int64_t r0 = row0(k);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + (lane >> 4) + 4 * r;
            a[r] = (k < cnt && row < n) ? Wn[r0 * 16 + 64 * r + lane] : 0.0;
        }
        qv[0] = qv[1] = qv[2] = qv[3] = 0.0;
        const int64_t row = r0 + (lane & 15);
        if (k < cnt && row < n) {  // qv[kc] = W_j[r0 + (l & 15)][4 (l >> 4) + kc]
            const double2 *p2 = reinterpret_cast<const double2 *>(Q + row * 16 + 4 * (lane >> 4));
            const double2 x = p2[0], y = p2[1];
            qv[0] = x.x; qv[1] = x.y; qv[2] = y.x; qv[3] = y.y;
        }
    };
    d4_t acc_n;
    double qv_n[4];
    fetch(0, acc_n, qv_n);
    for (int64_t k = 0; k < cnt; ++k) {
        const int64_t r0 = row0(k);
        d4_t acc = acc_n;
        double qv[4] = {qv_n[0], qv_n[1], qv_n[2], qv_n[3]};
        fetch(k + 1, acc_n, qv_n);
        if (r0 >= n) continue;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) acc = mfma16(qv[kc], na_op[kc], acc);
        double *dst = Wn;
        if constexpr (SWAP) {
            dst = Q;
            const int64_t row = r0 + (lane & 15);
            if (row < n) {
                double2 *p2 = reinterpret_cast<double2 *>(Wn + row * 16 + 4 * (lane >> 4));
                p2[0] = make_double2(qv[0], qv[1]);
                p2[1] = make_double2(qv[2], qv[3]);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + (lane >> 4) + 4 * r;
            if (row < n) dst[r0 * 16 + 64 * r + lane] = acc[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) gacc = mfma16(acc[r], acc[r], gacc);
    }
    // the waves' accumulators summed in wave order into the block's slab
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = gacc[r];
    __syncthreads();
    if (threadIdx.x < 256) {
        double sum = 0.0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sum += red[ww][threadIdx.x];
        part[(int64_t)blockIdx.x * 256 + threadIdx.x] = sum;
    }
}

// ---------------------------------------------------------------------------
// Wave-specialised persistent pass 1 (the k_spmm_ws structure, lz_spmm.hip,
// plus the fused epilogue).  One block per CU: a LOADER wave streams, per tile
// of 16*NC rows, the tile's row pointers and CSR run into a ring of FW_K LDS
// stages with LDS-DMA (a fixed number of DMA instructions per tile, so "the
// previous tile has landed" is a compile-time vmcnt); NC CONSUMER waves (one
// 16-row strip each) gather X from L2 (8 loads in flight per lane), load their
// own W rows (L2-resident: just gathered by neighbouring tiles), run the MFMA
// epilogue, store Q_j and W', and accumulate Q_j^T W' in registers across
// their tiles -- one 16x16 slab per consumer wave, no block barrier after the
// first.  The consumers' memory waits never cover the CSR stream.
//   QREG (default build): the stage holds only the CSR run, so three stages
//     fit; each consumer loads its Q_{j-1} strip into registers at the start
//     of its tile and releases the stage right after its gather.  Measured
//     1.87 ms against 1.94 ms for the Q-in-stage form at C3.
//   !QREG: Q_{j-1} strips also land in the stage (chunk-column order, slot
//     c4*16 + r); a consumer reuses its strip as the XOR-swizzled transpose
//     scratch and releases the stage after the epilogue.
//   NL > 1: NL loader waves stage alternate tiles, each publishing its tile as
//     soon as it lands.
// The stage layout (FwCfg), kPairPad and fw_sw are in lz_kernels.hpp.

// Per 16-row strip: the strip's rows sorted by length (ties by row), packed
// as 16 nibbles (nibble i = row of rank i; rows past n have length 0).
// Computed once per solve; k_fused_pp16 pairs rank g with rank 15 - g so each
// lane group's two-row list is a long row plus a short one.  (C3 rows: 10 +-
// 2.2 nnz; a wave steps as long as its longest list: 3.48 steps per strip for
// the rows (g, g+8), 3.03 for the ranked pairs, 3.00 ideal.)
__global__ __launch_bounds__(256) void k_strip_pairs(int64_t n, const int64_t *__restrict__ rp,
                                                     uint64_t *__restrict__ out)
{
    // kPairPad strips past the last one get the order of 16 empty rows (the
    // identity): the last tile's trailing strips lie past n, and a consumer
    // must still write every row of its parked Y tile (rows of length 0)
    const int64_t ns = (n + 15) / 16 + kPairPad;
    for (int64_t st = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; st < ns;
         st += (int64_t)gridDim.x * blockDim.x) {
        uint32_t key[16];
        const int64_t r0 = st * 16;
        // the strip's 17 row pointers first, all in flight at once (clamped
        // indices: no per-load branch for the compiler to serialise on)
        int64_t rv[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) rv[i] = rp[r0 + i < n ? r0 + i : n];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t len = r0 + i < n ? rv[i + 1] - rv[i] : 0;
            key[i] = ((uint32_t)(len < (1 << 27) ? len : (1 << 27)) << 4) | (uint32_t)i;
        }
#pragma unroll
        for (int i = 1; i < 16; ++i)  // insertion sort, ascending
#pragma unroll
            for (int j = i; j > 0; --j) {
                const uint32_t a = key[j - 1], b = key[j];
                key[j - 1] = a < b ? a : b;
                key[j] = a < b ? b : a;
            }
        uint64_t w = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) w |= (uint64_t)(key[i] & 15) << (4 * i);
        out[st] = w;
    }
}

int strip_pairs(lz_handle *h, int64_t n, const int64_t *rp, const uint64_t **out)
{
    const int64_t ns = ceil_div(n, (int64_t)16) + kPairPad;
    if ((size_t)ns > h->pairs_cap) {
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        (void)hipFree(h->pairs);
        h->pairs = nullptr;
        LZ_HIP_TRY(hipMalloc(&h->pairs, sizeof(uint64_t) * (size_t)ns));
        h->pairs_cap = (size_t)ns;
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ns, (int64_t)256), (int64_t)h->n_cu * 4));
    hipLaunchKernelGGL(k_strip_pairs, dim3(grid), dim3(256), 0, h->stream, n, rp, h->pairs);
    LZ_LAUNCH_CHECK();
    *out = h->pairs;
    return LZ_OK;
}


// ---------------------------------------------------------------------------
// Pipelined wave-specialised pass 1.  Timelines of k_fused_ws16
// (scripts/probe/tl_probe.hip) show two serialisations: a single loader
// publishes a stage only after issuing the next one (so a stage's readiness
// waits on the slowest consumer), and each consumer runs gather -> epilogue ->
// gather with nothing in flight during its epilogue.  Here
// - NL loader waves stage tiles l, l + NL, ... (CSR run only), each publishing
//   its tile as soon as it lands (its own vmcnt(0));
// - a consumer issues the first gather step of strip i, THEN runs the epilogue
//   of strip i-1 (its Y tile parked in LDS, its W / Q_{j-1} rows loaded into
//   registers after strip i-1's gather), so the epilogue hides the first
//   gather round trip;
// WIN: the gather source has 2^24 rows or more (X >= 2 GiB: past a 32-bit
//   buffer offset); each strip gathers through a window of kWinRows rows
//   centred on its own row (row_off + s0; a once-per-solve check,
//   gather_window_ok, proved every column of the strip lies inside it), so the
//   buffer-addressed gather keeps working at any n (BASELINE config C4: 40M
//   rows on one GPU, or the all-gathered block at N >= 2).
template <int NC, int CAP, int K, int NL, bool WIN = false, bool C16 = false>
__global__ __launch_bounds__(64 * (NC + NL)) void k_fused_pp16(
    int64_t n, const int64_t *__restrict__ rp, const int32_t *__restrict__ col, const int16_t *__restrict__ col16,
    const double *__restrict__ val, const double *__restrict__ Wg, int64_t nx,
    const double *__restrict__ Wown, const double *Qbuf, double *Wn,
    const double *__restrict__ binv, const double *__restrict__ beta, int64_t lc,
    double *__restrict__ qrow, double *__restrict__ part, int *__restrict__ err,
    const uint64_t *__restrict__ pairs, int64_t row_off)
{
    constexpr bool BP = true;
    using CT = typename std::conditional<C16, int16_t, int32_t>::type;
    using C = FwCfg<NC, CAP, true, BP, CT>;
    constexpr int TR = C::TR;
#ifdef LZ_WS_PROBE
    const int dbg = lz_ws_dbg;  // timing masks: bit 0 skips the Q_{j-1} loads, bit 1 the W loads
#else
    constexpr int dbg = 0;
#endif
    __shared__ typename C::Stage st[K];
    __shared__ double scr[NC][256];  // per consumer: the parked Y tile (swizzled)
    __shared__ double ops[2][256];      // beta^-1, -beta in MFMA B-operand order
    __shared__ int ready[K], done[K], slabs_in;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool has_prev = beta != nullptr;
    if (threadIdx.x < K) {
        ready[threadIdx.x] = -1;
        done[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) slabs_in = 0;
    // B operands in a permuted contraction order: MFMA step kc, lane l contracts
    // over k = 4 (l >> 4) + kc (not 4 kc + (l >> 4)), so every A operand a lane
    // needs is 4 contiguous doubles of one row -- two 16-B loads instead of
    // four 8-B loads for the W row tiles (C = M B is unchanged: the same k
    // permutation on both operands)
    for (int e = threadIdx.x; e < 256; e += blockDim.x) {
        const int kc = e >> 6, l = e & 63;
        const int idx = (4 * (l >> 4) + kc) * 16 + (l & 15);
        ops[0][e] = binv[idx];
        ops[1][e] = has_prev ? -beta[idx] : 0.0;
    }
    __syncthreads();  // the only block barrier
    const int64_t T = ceil_div(n, (int64_t)TR);
    int64_t begin, end, kb, KB;
    {
        const int64_t G = gridDim.x, b = blockIdx.x;
        if (G < 8) {
            begin = 0; end = T; kb = b; KB = G;
        } else {
            const int64_t x = b & 7;
            begin = T * x / 8;
            end = T * (x + 1) / 8;
            kb = b >> 3;
            KB = (G - x + 7) >> 3;
        }
    }
    const int64_t nt = (end - begin - kb + KB - 1) / KB > 0 ? (end - begin - kb + KB - 1) / KB : 0;
    auto tile_r0 = [&](int64_t i) { return (begin + kb + i * KB) * TR; };
    if (w < NL) {
        // ------------------------------------------------------------ loaders
        __builtin_amdgcn_s_setprio(3);
        const int64_t nnz = rp[n];
        for (int64_t i = w; i < nt; i += NL) {
            const int s = (int)(i % K);
            const int64_t r0 = tile_r0(i), r1 = (r0 + TR < n) ? r0 + TR : n;
            const int64_t kA = rp[r0];
            if (i >= K) {
                long spin = 0;
                const uint32_t da = ws_lds_addr(&done[s]);
                while (ws_lds_read(da) < NC * (int)(i / K) && ++spin < kWsSpin) __builtin_amdgcn_s_sleep(1);
                if (spin >= kWsSpin) { *err = 3; break; }
            }
            WS_TL(i, 0);
            const int64_t ca = kA & ~(int64_t)(C::CPP - 1), va = kA & ~(int64_t)1;
            // buffer range checks are per dword: with 2-B columns the last dword may
            // hold one real column and one past nnz, so the range ends on a dword
            // boundary (col16_plan allocates that slack)
            const int64_t cb = ((nnz - ca) * (int64_t)sizeof(CT) + 3) & ~(int64_t)3, vb = (nnz - va) * 8;
            const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int64_t *>(rp + r0), (short)0,
                                                              (int)((r1 - r0 + 1) * 8), 0x00020000);
            const CT *cbase = C16 ? reinterpret_cast<const CT *>(col16) : reinterpret_cast<const CT *>(col);
            const auto cr = __builtin_amdgcn_make_buffer_rsrc(const_cast<CT *>(cbase + ca), (short)0,
                                                              (int)(cb < 0x7fffffff ? cb : 0x7fffffff), 0x00020000);
            const auto vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(val + va), (short)0,
                                                              (int)(vb < 0x7fffffff ? vb : 0x7fffffff), 0x00020000);
            ws_dma(rr, st[s].rp, C::RP_PIECES, lane);
            ws_dma(cr, st[s].col, C::COL_PIECES, lane);
            ws_dma(vr, st[s].val, C::VAL_PIECES, lane);
            if constexpr (BP) {  // the tile's strips' row orders (past the last strip: identity)
                const int64_t s0i = r0 / 16, ns = (n + 15) / 16 + kPairPad;
                const auto pr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(pairs + s0i), (short)0,
                                                                  (int)((ns - s0i) * 8), 0x00020000);
                ws_dma(pr, st[s].pr, C::PR_PIECES, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) ws_lds_write(ws_lds_addr(&ready[s]), (int)i);
            WS_TL(i, 1);
        }
        return;
    }
    // -------------------------------------------------------------- consumers
    const int cw = w - NL;
    // The SQ favours older (lower-numbered) waves at equal priority: measured
    // per-consumer strip times rise ~35 % from the first to the last consumer,
    // and every tile waits for its slowest consumer.  Later consumers get a
    // higher issue priority (the loaders keep the highest).
#ifdef LZ_WS_PROBE
    if (!(lz_ws_dbg & 16))
#endif
    {
        const int pr = (cw * 3) / NC;
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    }
    __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Wg), (short)0, (int)(WIN ? kWinRows * 128 : nx * 128),
                                          0x00020000);
    uint32_t wb = 0;  // WIN: first row of the strip's gather window
    double *S0 = scr[cw];
    d4_t macc = {0.0, 0.0, 0.0, 0.0};
    // the pending strip's W_j and W_{j-1} rows, loaded straight into MFMA
    // A-operand order (permuted contraction, see ops: two 16-B loads per lane),
    // so the epilogue needs no LDS transpose for them
    double wa[4] = {0.0, 0.0, 0.0, 0.0}, qa[4] = {0.0, 0.0, 0.0, 0.0};
    auto aop_load = [&](const double *src, int64_t s0, double a[4]) {
        const int rows = (int)(n - s0 < 16 ? (n - s0 > 0 ? n - s0 : 0) : 16);  // strips past n: none
        const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(src + (s0 < n ? s0 : 0) * 16), (short)0,
                                                         rows * 128, 0x00020000);
        // a[kc] = M[l & 15][4 (l >> 4) + kc]: 32 contiguous bytes per lane
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(
                r, (uint32_t)((lane & 15) * 128 + (lane >> 4) * 32 + hh * 16), 0, 0);
            __builtin_memcpy(&a[2 * hh], &u, 16);
        }
    };
    int64_t s0p = -1;  // strip whose epilogue is pending
#ifdef LZ_WS_PROBE
    long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PP_T(v) const long long v = clock64()
#else
#define PP_T(v)
#endif
    // epilogue of the pending strip: Y parked in S0 (swizzled), W/Q rows in wv/qv
    auto epilogue = [&]() {
        const int ar = lane & 15;
        double ya[4];
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) ya[kc] = S0[fw_sw(ar, 4 * (lane >> 4) + kc)];
        d4_t q1 = {0.0, 0.0, 0.0, 0.0}, wn = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) q1 = mfma16(wa[kc], ops[0][64 * kc + lane], q1);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) wn = mfma16(qa[kc], ops[1][64 * kc + lane], wn);  // qa == 0 if !has_prev
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) wn = mfma16(ya[kc], ops[0][64 * kc + lane], wn);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = s0p + (lane >> 4) + 4 * r;
            if (row < n) {
                Wn[s0p * 16 + 64 * r + lane] = wn[r];
                if (row == lc) qrow[lane & 15] = q1[r];
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) macc = mfma16(q1[r], wn[r], macc);
    };
    for (int64_t i = 0; i < nt; ++i) {
        const int s = (int)(i % K);
        const int64_t r0 = tile_r0(i);
        const int64_t s0 = r0 + 16 * cw;
        const int g = lane >> 3, p = lane & 7;
        const uint32_t lane_off = 16u * p;
        if constexpr (WIN) {  // the strip's window: kWinRows rows centred on it
            const int64_t hi = nx - kWinRows > 0 ? nx - kWinRows : 0;
            int64_t b0 = s0 + row_off - kWinRows / 2;
            b0 = b0 < 0 ? 0 : (b0 > hi ? hi : b0);
            wb = (uint32_t)b0;
            xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Wg + b0 * 16), (short)0, (int)(kWinRows * 128),
                                                   0x00020000);
        }
        long spin = 0;
        PP_T(ta);
        while (__hip_atomic_load(&ready[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)i &&
               ++spin < kWsSpin)
            __builtin_amdgcn_s_sleep(1);
        if (spin >= kWsSpin) { *err = 4; break; }
        PP_T(tb);
        WS_TL(i, 2 + 2 * cw);
        asm volatile("" ::: "memory");
        typename C::Stage &S = st[s];
        const int64_t kA = S.rp[0];
        const int co = (int)(kA & (C::CPP - 1)), vo = (int)(kA & 1);
        const int nrow = (int)(n - r0 < TR ? n - r0 : TR);
        const int runlen = (int)(S.rp[nrow] - kA);
        // the group's two rows of the strip: g and g + 8, or (BP) the rows of
        // length rank g and 15 - g (a long row plus a short one: a wave steps
        // as long as its longest list)
        int ra = g, rb = g + 8;
        if constexpr (BP) {
            const uint64_t pw = S.pr[cw];
            ra = (int)(pw >> (4 * g)) & 15;
            rb = (int)(pw >> (4 * (15 - g))) & 15;
        }
        const int lra = 16 * cw + ra, lrb = 16 * cw + rb;
        const int o0 = lra < nrow ? (int)(S.rp[lra] - kA) : 0;
        const int len0 = lra < nrow ? (int)(S.rp[lra + 1] - kA) - o0 : 0;
        const int o1 = lrb < nrow ? (int)(S.rp[lrb] - kA) : 0;
        const int len1 = lrb < nrow ? (int)(S.rp[lrb + 1] - kA) - o1 : 0;
        const int cnt = len0 + len1;
        double y[4] = {0.0, 0.0, 0.0, 0.0};
        if (runlen <= CAP) {  // tile-uniform
            const CT *cp = S.col + co;
            // C16: a column is stored as its offset from the strip's first row in
            // the gather source's numbering (row_off + s0); fold the window base in
            const uint32_t cb16 = C16 ? (uint32_t)(s0 + row_off) - wb : 0u;
            const double *vp = S.val + vo;
            auto slot = [&](int ff) {
                const int o = ff < len0 ? o0 + ff : o1 + (ff - len0);
                return ff < cnt ? o : o0;
            };
            auto issue = [&](int f, double2 *xs) {
                int32_t c[8];
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) c[tt] = cp[slot(f + tt)];
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) {
                    const uint32_t off =
                        f + tt < cnt ? __umul24(C16 ? (unsigned)c[tt] + cb16 : (unsigned)c[tt] - wb, 128u) + lane_off
                                     : 0x80000000u;
                    const auto u4 = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
                    __builtin_memcpy(&xs[tt], &u4, 16);
                }
            };
            auto fmas = [&](int f, const double2 *xs) {
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) {
                    const double v = vp[slot(f + tt)];
                    if (f + tt < len0) {
                        y[0] = fma(v, xs[tt].x, y[0]);
                        y[1] = fma(v, xs[tt].y, y[1]);
                    } else {  // masked entries: x == 0, v finite
                        y[2] = fma(v, xs[tt].x, y[2]);
                        y[3] = fma(v, xs[tt].y, y[3]);
                    }
                }
            };
            double2 xs[8];
            PP_T(tc);
            issue(0, xs);  // step 0 for every lane (masked past cnt)
            PP_T(td);
            if (s0p >= 0) epilogue();
            PP_T(te);
            fmas(0, xs);
            PP_T(tf);
            for (int f = 8; f < cnt; f += 8) {  // group-uniform
                issue(f, xs);
                fmas(f, xs);
            }
            PP_T(tg);
#ifdef LZ_WS_PROBE
            ph[1] += tc - tb; ph[2] += td - tc; ph[3] += te - td; ph[4] += tf - te; ph[5] += tg - tf;
#endif
        } else {  // long run (rare): epilogue first, then gather from global
            if (s0p >= 0) epilogue();
            ws_gather(col + kA, val + kA, o0, len0, o1, cnt, xr, lane_off, y, wb);
        }
        // the CSR stage is no longer read by this wave
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&done[s], 1);
        // park Y (swizzled) and fetch this strip's W and Q_{j-1} rows for its
        // epilogue, which runs behind the next strip's first gather step
        S0[fw_sw(ra, 2 * p)] = y[0];
        S0[fw_sw(ra, 2 * p + 1)] = y[1];
        S0[fw_sw(rb, 2 * p)] = y[2];
        S0[fw_sw(rb, 2 * p + 1)] = y[3];
        if (!(dbg & 2)) aop_load(Wown, s0, wa);
        if (has_prev && !(dbg & 1)) aop_load(Qbuf, s0, qa);
        s0p = s0;
        wave_lds_sync();
        WS_TL(i, 3 + 2 * cw);
#ifdef LZ_WS_PROBE
        {
            PP_T(th);
            ph[0] += tb - ta;
            ph[6] += th - ta;
        }
#endif
    }
#ifdef LZ_WS_PROBE
    if (cw == 0 && lane == 0)
        for (int j = 0; j < 7; ++j) lz_ws_probe[8 * blockIdx.x + j] = ph[j];
    if (cw == 0 && lane == 0) lz_ws_probe[8 * blockIdx.x + 7] = nt;
#endif
    if (s0p >= 0) epilogue();
    // the block's NC consumer slabs folded into one at part[blockIdx.x] by the
    // last consumer to finish (an LDS counter; the loaders have exited), in
    // k_slab_reduce1's order for NC slabs -- the launch that folded them is gone
#pragma unroll
    for (int r = 0; r < 4; ++r) S0[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = macc[r];
    int arrived = 0;
    if (lane == 0) arrived = __hip_atomic_fetch_add(&slabs_in, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    arrived = __shfl(arrived, 0, 64);
    if (arrived == NC - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        double *slab = part + (int64_t)blockIdx.x * 256;
        for (int e = lane; e < 256; e += 64) {
            double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
            int sl = 0;
            for (; sl + 7 < NC; sl += 8) {
#pragma unroll
                for (int i = 0; i < 8; ++i) a[i] += scr[sl + i][e];
            }
            for (; sl < NC; ++sl) a[0] += scr[sl][e];
            slab[e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        }
    }
}

// C = A * B, 16 x 16 row-major fp64 (the per-step P1 = beta_{j-1}^-1 beta_j and
// P2 = beta_j^-1 alpha_j of the Q-free iteration, lz_api.hip)
__global__ __launch_bounds__(256) void k_mm16(const double *__restrict__ A, const double *__restrict__ B,
                                              double *__restrict__ C)
{
    __shared__ double a[256], b[256];
    const int t = threadIdx.x;
    a[t] = A[t];
    b[t] = B[t];
    __syncthreads();
    const int i = t >> 4, j = t & 15;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s = fma(a[i * 16 + k], b[k * 16 + j], s);
    C[t] = s;
}

int mm16(lz_handle *h, const double *A, const double *B, double *C)
{
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_mm16, dim3(1), dim3(256), 0, h->stream, A, B, C);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// Once per solve, when the gather source has 2^24 rows or more: does every
// column of every 16-row strip fall inside the strip's kWinRows window
// (k_fused_pp16<..., WIN>)?  One pass over col, one host read-back.
__global__ __launch_bounds__(256) void k_window_check(int64_t n, const int64_t *__restrict__ rp,
                                                      const int32_t *__restrict__ col, int64_t nx,
                                                      int64_t row_off, int *__restrict__ bad)
{
    const int64_t hi = nx - kWinRows > 0 ? nx - kWinRows : 0;
    int out = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t b0 = (r & ~(int64_t)15) + row_off - kWinRows / 2;
        b0 = b0 < 0 ? 0 : (b0 > hi ? hi : b0);
        for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k) {
            const int64_t d = (int64_t)col[k] - b0;
            out |= (d < 0) | (d >= kWinRows);
        }
    }
    if (out) atomicOr(bad, 1);
}

int gather_window_ok(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, int64_t nx, int64_t row_off,
                     bool *ok)
{
    int *flag = h->err_flag + 8;  // err_flag[0] is the device error word
    LZ_HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), h->stream));
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)256), (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_window_check, dim3(grid), dim3(256), 0, h->stream, n, rp, col, nx, row_off, flag);
    LZ_LAUNCH_CHECK();
    int bad = 1;
    LZ_HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    *ok = bad == 0;
    return LZ_OK;
}

// Pass 1 (Q-free).  Qbuf: W_{j-1} (own rows; may be the same buffer as Wn, row
// r is read before it is written by the same wave), beta: P1 =
// beta_{j-1}^-1 beta_j (or null at j = 0).  k_fused_pp16 in one of two
// shapes by mean row length: 14 consumers x 16 rows with a 2376-entry stage
// (C3: 10 nnz/row) or 10 consumers with 4400 entries (C4: 25 nnz/row), both
// one 1024 / 768-thread block per CU.  Gather sources past 2^24 rows use the
// windowed instantiation when every strip's columns fit its window
// (gather_window_ok), else the 64-bit tile kernel.
bool fused16_direct(int64_t nx, int win) { return nx < (1 << 24) || win; }

// Pass 1's 16-bit columns (once per solve): col16[k] = col[k] - (first row of
// row r's 16-row strip + row_off), the strip's own row in the gather source's
// numbering; a column out of int16 reach sets *bad.
__global__ __launch_bounds__(256) void k_col16(int64_t n, const int64_t *__restrict__ rp,
                                               const int32_t *__restrict__ col, int64_t row_off,
                                               int16_t *__restrict__ col16, int *__restrict__ bad)
{
    int out = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t base = (r & ~(int64_t)15) + row_off;
        for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k) {
            const int64_t d = (int64_t)col[k] - base;
            out |= (d < -32768) | (d > 32767);
            col16[k] = (int16_t)d;
        }
    }
    if (out) atomicOr(bad, 1);
}

int col16_plan(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, int64_t row_off,
               const int16_t **out)
{
    *out = nullptr;
    const char *e = getenv("LZ_PASS1_C16");  // "0": 32-bit columns (A/B); read per call
    if ((e && e[0] == '0') || n <= 0 || nnz <= 0) return LZ_OK;
    const size_t bytes = (size_t)nnz * 2 + 16;  // + the dword the kernel's range may end in
    if (bytes > h->c16_cap) {
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        (void)hipFree(h->c16buf);
        h->c16buf = nullptr;
        h->c16_cap = 0;
        LZ_HIP_TRY(hipMalloc(&h->c16buf, bytes));
        h->c16_cap = bytes;
    }
    int *flag = h->err_flag + 9;
    LZ_HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), h->stream));
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)256), (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_col16, dim3(grid), dim3(256), 0, h->stream, n, rp, col, row_off,
                       static_cast<int16_t *>(h->c16buf), flag);
    LZ_LAUNCH_CHECK();
    int bad = 1;
    LZ_HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    if (!bad) *out = static_cast<const int16_t *>(h->c16buf);
    return LZ_OK;
}

int fused_spmm16(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const double *val,
                 const double *Wg, int64_t nx, const double *Wown, const double *Qbuf, double *Wn,
                 const double *binv, const double *beta, int64_t lc, double *qrow, int *nparts,
                 const uint64_t *pairs, int64_t nnz, int64_t row_off, int win, int slab_off, const int16_t *col16)
{
    const int64_t tiles = ceil_div(n, kFusedRows);
    LZ_ARG_CHECK(tiles >= 1 && tiles < (1LL << 31), "tile count");
    LZ_ARG_CHECK(pairs != nullptr, "strip row orders (strip_pairs) missing");
    const bool buf = nx < (1 << 24);  // 128-B rows: X < 2 GiB
    if (buf || win) {
        const bool wide = (double)nnz > 10.2 * (double)n;  // rows too long for the 2376-entry stage
        const int nc = wide ? 10 : 14;
        static_assert(14 <= kPairPad, "row orders must cover the last tile's strips");
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)16 * nc), h->n_cu));
        static_assert(kMaxB * kMaxB >= 256, "h->partials2 holds one 16 x 16 slab per pass-1 block");
        const int ev = prof_begin(h, PROF_SPMM_PASS);
        auto go = [&](auto kern) {  // one folded slab per block, at h->partials2
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (nc + 2)), 0, h->stream, n, rp, col, col16, val, Wg, nx, Wown,
                               Qbuf, Wn, binv, beta, lc, qrow, h->partials2 + (int64_t)slab_off * 256, h->err_flag,
                               pairs, row_off);
        };
        if (!wide && buf && col16) go(k_fused_pp16<14, 2376, 3, 2, false, true>);
        else if (!wide && col16) go(k_fused_pp16<14, 2376, 3, 2, true, true>);
        else if (!wide && buf) go(k_fused_pp16<14, 2376, 3, 2, false>);
        else if (!wide) go(k_fused_pp16<14, 2376, 3, 2, true>);
        else if (buf) go(k_fused_pp16<10, 4400, 2, 2, false>);
        else go(k_fused_pp16<10, 4400, 2, 2, true>);
        prof_end(h, ev);
        LZ_LAUNCH_CHECK();
        *nparts = grid;
        return LZ_OK;
    }
    LZ_ARG_CHECK(slab_off == 0, "the 64-bit fused pass covers the whole row range (slab_off 0)");
    LZ_TRY(ensure_partials(h, tiles * 256));
    const int ev = prof_begin(h, PROF_SPMM_PASS);
    hipLaunchKernelGGL(k_fused_spmm16<false>, dim3((unsigned)tiles), dim3(512), 0, h->stream, n, rp, col, val, Wg, nx,
                       Wown, Qbuf, Wn, binv, beta, lc, qrow, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    // fold the per-tile slabs to <= 256 (fixed order) at h->partials2
    return fold_slabs(h, h->partials, tiles, 256, nparts);
}

int fused_update16(lz_handle *h, int64_t n, double *Wn, const double *Q, const double *alpha,
                   int *nparts)
{
    // persistent, one block of 8 waves per CU (256 slabs for the sqrtm to
    // reduce), rows walked last-first.  Measured (C3): 1 block of 8 waves
    // 0.723 ms, 2 blocks 0.740, 3 0.758, 4 0.738; forward order 0.761 ms
    const int64_t units = ceil_div(ceil_div(n, 16), 8);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, (int64_t)h->n_cu));
    LZ_TRY(ensure_partials(h, (size_t)grid * 256));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    hipLaunchKernelGGL((k_fused_update16<true, 8>), dim3(grid), dim3(512), 0, h->stream, n, Wn, Q, alpha,
                       h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

// the SWAP form (k_fused_update16 above): Xown = W'' (was W_j), Wn = W_j (was W')
int fused_update16_swap(lz_handle *h, int64_t n, double *Wn, double *Xown, const double *alpha, int *nparts)
{
    const int64_t units = ceil_div(ceil_div(n, 16), 8);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, (int64_t)h->n_cu));
    LZ_TRY(ensure_partials(h, (size_t)grid * 256));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    hipLaunchKernelGGL((k_fused_update16<true, 8, true>), dim3(grid), dim3(512), 0, h->stream, n, Wn, Xown, alpha,
                       h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

// ===================================================== single-vector Lanczos
// Two streaming passes per step; the scalar reductions are finished redundantly
// (same fixed order, so the same bits) by every workgroup of the next pass, so
// no separate reduction launch and no host round trip:
//   k_vl_spmv    beta_j = sqrt(sum slabs); q_j[r] = w[r]/beta_j (in place over
//                q_{j-1}[r] after reading it); w'[r] = (A w)[r]/beta_j -
//                beta_j q_{j-1}[r]; slabs of w'.q_j
//   k_vl_update  alpha_j = sum slabs; w' -= alpha_j q_j; slabs of w'.w'
constexpr int kVlThreads = 512;

__device__ __forceinline__ double block_sum_slabs(const double *__restrict__ part, int P,
                                                  double *red)
{
    double s = 0.0;
    for (int i = threadIdx.x; i < P; i += blockDim.x) s += part[i];
    // fixed-shape tree: deterministic for fixed P and blockDim
    red[threadIdx.x] = s;
    __syncthreads();
    for (int st = blockDim.x / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__device__ __forceinline__ void block_store_slab(double v, double *red, double *__restrict__ out)
{
    red[threadIdx.x] = v;
    __syncthreads();
    for (int st = blockDim.x / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// slabs of x.x (start of the recurrence, ||b||^2)
template <typename T>
__global__ __launch_bounds__(kVlThreads) void k_vl_sq(int64_t n, const T *__restrict__ x,
                                                      double *__restrict__ part)
{
    __shared__ double red[kVlThreads];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double xi = x[i];
        s = fma(xi, xi, s);
    }
    block_store_slab(s, red, part);
}

// beta_j = ||w|| rounded to T, and the scale 1./beta_j the reference multiplies
// by (`mult_scalar(1./beta[j])`, vector_lanczos.hpp:46-47: a double quotient
// rounded to T).  For T = double: sqrt and 1/sqrt, as before.
template <typename T>
__device__ __forceinline__ void vl_beta(double bsq, T &beta, T &rbeta)
{
    beta = (T)sqrt(bsq);
    rbeta = (T)(1.0 / (double)beta);
}

template <typename T, int LV>
__global__ __launch_bounds__(kVlThreads) void k_vl_spmv(
    int64_t n, const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
    const T *__restrict__ val, const T *__restrict__ w, T *__restrict__ qbuf,
    T *__restrict__ wn, const double *__restrict__ part_in, int P, int has_prev, int64_t lc,
    T *__restrict__ qrow, T *__restrict__ beta_out, double *__restrict__ part_out)
{
    __shared__ double red[kVlThreads];
    const double bsq = block_sum_slabs(part_in, P, red);
    T beta, rbeta;
    vl_beta(bsq, beta, rbeta);
    if (blockIdx.x == 0 && threadIdx.x == 0) *beta_out = beta;
    constexpr int RB = kVlThreads / LV;
    const int gi = threadIdx.x / LV, p = threadIdx.x % LV;
    double dot = 0.0;
    XcdSched sch(ceil_div(n, RB));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t row = u * RB + gi;
        const bool valid = row < n;
        const int64_t k0 = valid ? rp[row] : 0, k1 = valid ? rp[row + 1] : 0;
        T acc = 0;
        int64_t k = k0 + p;
        for (; k + LV < k1; k += 2 * LV) {
            const int c0 = col[k], c1 = col[k + LV];
            const T v0 = val[k], v1 = val[k + LV];
            acc = fma(v0, w[c0], acc);
            acc = fma(v1, w[c1], acc);
        }
        if (k < k1) acc = fma(val[k], w[col[k]], acc);
#pragma unroll
        for (int off = LV / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (valid && p == 0) {
            const T qj = w[row] * rbeta;
            T wv = acc * rbeta;
            if (has_prev) wv = fma(-beta, qbuf[row], wv);
            qbuf[row] = qj;
            wn[row] = wv;
            dot = fma((double)wv, (double)qj, dot);
            if (row == lc) *qrow = qj;
        }
    }
    block_store_slab(dot, red, part_out);
}

// CSR-stream form of k_vl_spmv (same outputs).  A tile of R rows is one
// contiguous run of the CSR arrays: each thread loads whole 4-entry quads of it
// (one 16-B col load, two 16-B val loads), gathers the four w values, and parks
// the products in LDS; then thread t sums row t's products in CSR order and
// runs the row epilogue.  Against the lanes-per-row kernel this issues ~4x fewer
// vector-memory instructions per row (col/val vectorised, the epilogue on every
// lane instead of one in LV), which is what a 10-nnz-per-row SpMV spends.
// A run longer than NQ quads per thread (a heavy tile) takes a wave per row.
// The row sum adds rounded products left to right, the oracle's arithmetic.
template <int NT, int NQ>
__global__ __launch_bounds__(NT) void k_vl_spmv_cs(
    int64_t n, int64_t nnz, const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ w, double *__restrict__ qbuf,
    double *__restrict__ wn, const double *__restrict__ part_in, int P, int has_prev, int64_t lc,
    double *__restrict__ qrow, double *__restrict__ beta_out, double *__restrict__ part_out)
{
    constexpr int R = NT, CAPQ = NQ * NT;
    __shared__ double red[NT];
    __shared__ double prod[4 * CAPQ];
    __shared__ double yrow[R];
    __shared__ int64_t srp[R + 1];
    const double bsq = block_sum_slabs(part_in, P, red);
    double beta, rbeta;
    vl_beta(bsq, beta, rbeta);
    if (blockIdx.x == 0 && threadIdx.x == 0) *beta_out = beta;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    double dot = 0.0;
    XcdSched sch(ceil_div(n, R));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * R;
        const int rows = (int)(n - r0 < R ? n - r0 : R);
        for (int i = t; i <= rows; i += NT) srp[i] = rp[r0 + i];
        __syncthreads();
        const int64_t k0 = srp[0], k1 = srp[rows];
        double acc = 0.0;
        if (((k1 + 3) >> 2) - (k0 >> 2) <= CAPQ) {  // block-uniform
            const int64_t qb = k0 >> 2, qe = (k1 + 3) >> 2;
            int c[NQ][4];
            double v[NQ][4], x[NQ][4];
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                const int64_t q = qb + t + (int64_t)NT * i;
#pragma unroll
                for (int j = 0; j < 4; ++j) { c[i][j] = 0; v[i][j] = 0.0; }
                if (q < qe) {
                    if (4 * q + 4 <= nnz) {
                        const int4 c4 = *reinterpret_cast<const int4 *>(col + 4 * q);
                        const double2 va = *reinterpret_cast<const double2 *>(val + 4 * q);
                        const double2 vb = *reinterpret_cast<const double2 *>(val + 4 * q + 2);
                        c[i][0] = c4.x; c[i][1] = c4.y; c[i][2] = c4.z; c[i][3] = c4.w;
                        v[i][0] = va.x; v[i][1] = va.y; v[i][2] = vb.x; v[i][3] = vb.y;
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (4 * q + j < nnz) { c[i][j] = col[4 * q + j]; v[i][j] = val[4 * q + j]; }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                const int64_t q = qb + t + (int64_t)NT * i;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t e = 4 * q + j;
                    x[i][j] = (q < qe && e >= k0 && e < k1) ? w[c[i][j]] : 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                const int64_t q = qb + t + (int64_t)NT * i;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t e = 4 * q + j;
                    if (q < qe && e >= k0 && e < k1) {
#pragma clang fp contract(off)
                        prod[e - k0] = v[i][j] * x[i][j];
                    }
                }
            }
            __syncthreads();
            if (t < rows)
                for (int64_t k = srp[t] - k0, e = srp[t + 1] - k0; k < e; ++k) acc += prod[k];
        } else {  // heavy tile: a wave per row, lanes strided, fixed-shape shuffle tree
            for (int r = wv; r < rows; r += NT / 64) {
                double a = 0.0;
                for (int64_t k = srp[r] + lane; k < srp[r + 1]; k += 64) a = fma(val[k], w[col[k]], a);
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
                if (lane == 0) yrow[r] = a;
            }
            __syncthreads();
            if (t < rows) acc = yrow[t];
        }
        if (t < rows) {
            const int64_t row = r0 + t;
            const double qj = w[row] * rbeta;
            double wvv = acc * rbeta;
            if (has_prev) wvv = fma(-beta, qbuf[row], wvv);
            qbuf[row] = qj;
            wn[row] = wvv;
            dot = fma(wvv, qj, dot);
            if (row == lc) *qrow = qj;
        }
        __syncthreads();  // srp / prod / yrow reused by the next tile
    }
    block_store_slab(dot, red, part_out);
}

// Half band width max_k |col[k] - row(k)| of the operator (once per solve);
// band[0] must be zero on entry.
__global__ __launch_bounds__(256) void k_vl_band(int64_t n, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ col,
                                                 unsigned long long *__restrict__ band)
{
    unsigned long long m = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x)
        for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k) {
            const int64_t d = (int64_t)col[k] - r;
            const unsigned long long a = (unsigned long long)(d < 0 ? -d : d);
            m = a > m ? a : m;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(band, m);
}

// Band-window form of k_vl_spmv (same outputs, same per-row arithmetic: LV
// lanes per row, strided, fixed xor tree).  Block g owns the contiguous rows
// [n g / G, n (g+1) / G) and walks them in tiles of R; the gathered vector
// lives in an LDS ring holding w[r0 - H, r0 + R + H) for the current tile
// (H = the operator's half band width) while the next tile's R-element slab
// arrives from registers.  A banded operator's 10 gathers per row then cost
// LDS reads instead of ~10 L2 requests each holding a texture-path miss slot
// (PMC on C2: ~1e7 L2 requests per SpMV, the whole bound of the gather kernels).
// Operators with 2H + 2R > the ring gather from global memory (same kernel).
// Shapes <threads = tile rows, ring doubles>: <1024, 16384>, one block per CU,
// for half bands up to 7168; <512, 9216>, two blocks per CU (one block's loads
// overlap the other's row phase), for half bands up to 4096.

// Tile loop of k_vl_spmv_win; WIN selects LDS-ring or global gathers at
// compile time (a runtime select would make every gather a flat load).
template <typename T, int LV, int NT, int RING, bool WIN>
__device__ __forceinline__ double vl_win_tiles(int64_t n, int64_t c0, int64_t c1, int64_t H,
                                               const int64_t *__restrict__ rp,
                                               const int32_t *__restrict__ col,
                                               const T *__restrict__ val,
                                               const T *__restrict__ w, T *__restrict__ qbuf,
                                               T *__restrict__ wn, int has_prev, int64_t lc,
                                               T *__restrict__ qrow, T beta, T rbeta,
                                               T *ring, T *yrow, int32_t *rps)
{
    constexpr int R = NT;
    constexpr int RPP = NT / LV, PASSES = R / RPP;  // rows per pass, passes per tile
    const int t = threadIdx.x, g = t / LV, p = t % LV;
    const int64_t base = c0 - H;  // ring slot of w[i]: (i - base) mod RING
    auto slot = [&](int64_t i) -> int { return (int)((uint32_t)(i - base) % (uint32_t)RING); };
    auto wat = [&](int64_t i) -> T { return WIN ? ring[slot(i)] : w[i]; };
    double dot = 0.0;
    // the first tile's row pointers; later tiles' are loaded one tile ahead
    auto rows_at = [&](int64_t r) { return (int)(c1 - r < R ? c1 - r : R); };
    int64_t nkb = 0, nke = 0, nrp = 0;
    if (c0 < c1) {
        const int rw = rows_at(c0);
        nkb = rp[c0];
        nke = rp[c0 + rw];
        nrp = t < rw ? rp[c0 + t] : 0;
    }
    for (int64_t r0 = c0; r0 < c1; r0 += R) {
        const int rows = rows_at(r0);
        // next tile's slab and this thread's epilogue row, issued first
        const int64_t si = r0 + R + H + t;
        const T slab = (WIN && si < n) ? w[si] : T(0);
        const int64_t erow = r0 + t;
        const T qprev = (t < rows && has_prev) ? qbuf[erow] : T(0);
        // CSR offsets relative to the tile's first entry (a tile's run < 2^31).
        // The tile's row pointers come in one coalesced load per thread and
        // go through LDS: read per row by each lane group they were PASSES x 2
        // dependent-address loads, which the compiler issued one at a time
        // (one VGPR, vmcnt(0) after each).
        const int64_t kb = nkb, kend = nke;
        if (t < rows) rps[t] = (int)(nrp - kb);
        __syncthreads();
        if (r0 + R < c1) {  // the next tile's row pointers, in flight behind this tile
            const int rw = rows_at(r0 + R);
            nkb = kend;
            nke = rp[r0 + R + rw];
            nrp = t < rw ? rp[r0 + R + t] : 0;
        }
        const int32_t *cb = col + kb;
        const T *vb = val + kb;
        int ks[PASSES], ke[PASSES];
#pragma unroll
        for (int s = 0; s < PASSES; ++s) {
            const int lr = s * RPP + g;
            ks[s] = lr < rows ? rps[lr] : 0;
            ke[s] = lr < rows ? (lr + 1 < rows ? rps[lr + 1] : (int)(kend - kb)) : 0;
        }
        int c[PASSES][2];
        T v[PASSES][2];
#pragma unroll
        for (int s = 0; s < PASSES; ++s)
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
                const int k = ks[s] + p + h2 * LV;
                c[s][h2] = k < ke[s] ? cb[k] : -1;
                v[s][h2] = k < ke[s] ? vb[k] : T(0);
            }
#pragma unroll
        for (int s = 0; s < PASSES; ++s) {
            T acc = 0;
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2)
                if (c[s][h2] >= 0) acc = fma(v[s][h2], wat(c[s][h2]), acc);
            for (int k = ks[s] + p + 2 * LV; k < ke[s]; k += LV) acc = fma(vb[k], wat(cb[k]), acc);
#pragma unroll
            for (int off = LV / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
            if (p == 0) yrow[s * RPP + g] = acc;
        }
        __syncthreads();
        if (t < rows) {
            const T qj = wat(erow) * rbeta;
            T wv = yrow[t] * rbeta;
            if (has_prev) wv = fma(-beta, qprev, wv);
            qbuf[erow] = qj;
            wn[erow] = wv;
            dot = fma((double)wv, (double)qj, dot);
            if (erow == lc) *qrow = qj;
        }
        if (WIN && si < n) ring[slot(si)] = slab;  // disjoint from this tile's window (2H + 2R <= ring)
        __syncthreads();
    }
    return dot;
}

template <typename T, int LV, int NT, int RING>
__global__ __launch_bounds__(NT) void k_vl_spmv_win(
    int64_t n, const int64_t *__restrict__ rp, const int32_t *__restrict__ col,
    const T *__restrict__ val, const T *__restrict__ w, T *__restrict__ qbuf,
    T *__restrict__ wn, const double *__restrict__ part_in, int P, int has_prev, int64_t lc,
    T *__restrict__ qrow, T *__restrict__ beta_out, double *__restrict__ part_out,
    const unsigned long long *__restrict__ band)
{
    constexpr int R = NT, NI = (RING + NT - 1) / NT;
    __shared__ T ring[RING];
    __shared__ double red[R];  // the slab reduction scratch
    __shared__ T yrow[R];
    const int t = threadIdx.x;
    const int64_t H = (int64_t)*band;
    const bool win = 2 * H + 2 * R <= RING;  // block-uniform
    const int64_t c0 = n * blockIdx.x / gridDim.x, c1 = n * (blockIdx.x + 1) / gridDim.x;
    // first window w[c0 - H, c0 + R + H): all loads in flight, then the slab sum
    T wi[NI];
    const int64_t lo = c0 - H < 0 ? 0 : c0 - H, hi = c0 + R + H < n ? c0 + R + H : n;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int64_t i = lo + t + (int64_t)k * NT;
        wi[k] = (win && i < hi) ? w[i] : T(0);
    }
    const double bsq = block_sum_slabs(part_in, P, red);
    T beta, rbeta;
    vl_beta(bsq, beta, rbeta);
    if (blockIdx.x == 0 && t == 0) *beta_out = beta;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int64_t i = lo + t + (int64_t)k * NT;
        if (win && i < hi) ring[(int)((uint32_t)(i - (c0 - H)) % (uint32_t)RING)] = wi[k];
    }
    __syncthreads();
    // red (the slab scratch) is free during the tiles: it holds each tile's row pointers
    int32_t *rps = reinterpret_cast<int32_t *>(red);
    static_assert(sizeof(red) >= NT * sizeof(int32_t), "row pointers of a tile fit the slab scratch");
    const double dot = win ? vl_win_tiles<T, LV, NT, RING, true>(n, c0, c1, H, rp, col, val, w, qbuf, wn, has_prev,
                                                                 lc, qrow, beta, rbeta, ring, yrow, rps)
                           : vl_win_tiles<T, LV, NT, RING, false>(n, c0, c1, H, rp, col, val, w, qbuf, wn,
                                                                  has_prev, lc, qrow, beta, rbeta, ring, yrow, rps);
    block_store_slab(dot, red, part_out);
}

template <typename T>
__global__ __launch_bounds__(kVlThreads) void k_vl_update(int64_t n, T *__restrict__ wn,
                                                          const T *__restrict__ q,
                                                          const double *__restrict__ part_in,
                                                          int P, T *__restrict__ alpha_out,
                                                          double *__restrict__ part_out)
{
    __shared__ double red[kVlThreads];
    const T alpha = (T)block_sum_slabs(part_in, P, red);
    if (blockIdx.x == 0 && threadIdx.x == 0) *alpha_out = alpha;
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const T v = fma(-alpha, q[i], wn[i]);
        wn[i] = v;
        const double vd = v;
        s = fma(vd, vd, s);
    }
    block_store_slab(s, red, part_out);
}

template <typename T>
int vector_lanczos_dev(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                       const T *val, int m, int64_t lc, const T *b, T *q, T *alpha, T *beta, T *q0,
                       T *q1, T *w)
{
    constexpr bool F64 = std::is_same<T, double>::value;
    const double mean = n > 0 ? (double)nnz / (double)n : 10.0;
    const int lv = mean <= 5 ? 4 : mean <= 12 ? 8 : mean <= 28 ? 16 : mean <= 60 ? 32 : 64;
    // LZ_VL_KERNEL=cs / cs2: the CSR-stream kernel, 512 / 256-row tiles (needs
    // 16-B aligned col/val); row: lanes-per-row; win512 / win1024: one band-window
    // shape.  Default: the band window whose ring holds the operator's half band
    // (measured once per solve: one host sync), else lanes-per-row.
    const char *vk = getenv("LZ_VL_KERNEL");
    const bool al16 = ((uintptr_t)col & 15) == 0 && ((uintptr_t)val & 15) == 0;
    const int cs = !(F64 && vk && al16) ? 0 : !strcmp(vk, "cs") ? 1 : !strcmp(vk, "cs2") ? 2 : 0;
    unsigned long long *band = reinterpret_cast<unsigned long long *>(h->partials + 8192);
    int win = 0;  // 1: <512, 9216>, 2: <1024, 16384>
    if (!cs && lv <= 8 && !(vk && !strcmp(vk, "row"))) {
        LZ_HIP_TRY(hipMemsetAsync(band, 0, sizeof(*band), h->stream));
        hipLaunchKernelGGL(k_vl_band, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), h->n_cu * 4))),
                           dim3(256), 0, h->stream, n, rp, col, band);
        LZ_LAUNCH_CHECK();
        unsigned long long H = 0;
        LZ_HIP_TRY(hipMemcpyAsync(&H, band, sizeof(H), hipMemcpyDeviceToHost, h->stream));
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        win = (vk && !strcmp(vk, "win512")) ? 1 : (vk && !strcmp(vk, "win1024")) ? 2
              : 2 * H + 2 * 512 <= 9216     ? 1
              : 2 * H + 2 * 1024 <= 16384   ? 2
                                            : 0;
    }
    const int grid = win == 1  ? (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 512), (int64_t)h->n_cu * 2))
                     : win == 2 ? (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 1024), (int64_t)h->n_cu))
                     : cs == 1 ? (int)std::max<int64_t>(8, std::min<int64_t>(ceil_div(n, 512), (int64_t)h->n_cu * 2))
                     : cs == 2 ? (int)std::max<int64_t>(8, std::min<int64_t>(ceil_div(n, 256), (int64_t)h->n_cu * 5))
                               : (int)std::max<int64_t>(
                              8, std::min<int64_t>(ceil_div(n, kVlThreads / lv), (int64_t)h->n_cu * 4));
    const int gridu = (int)std::max<int64_t>(
        8, std::min<int64_t>(ceil_div(n, kVlThreads), (int64_t)h->n_cu * 4));
    // slabs: two alternating regions of h->partials
    double *pa = h->partials, *pb = h->partials + 4096;
    const int gsq = gridu;
    hipLaunchKernelGGL(k_vl_sq<T>, dim3(gsq), dim3(kVlThreads), 0, h->stream, n, b, pa);
    LZ_LAUNCH_CHECK();
    int P = gsq;
    const T *wcur = b;
    T *wbuf[2] = {w, q1};
    int wi = 0;
    for (int j = 0; j < m; ++j) {
        T *wnext = wbuf[wi];
        const int ev_s = prof_begin(h, PROF_SPMM_PASS);  // the SpMV pass (bench: C2 roofline)
#define LZ_VL_CASE(LV)                                                                          \
    case LV:                                                                                    \
        hipLaunchKernelGGL((k_vl_spmv<T, LV>), dim3(grid), dim3(kVlThreads), 0, h->stream, n, rp, \
                           col, val, wcur, q0, wnext, pa, P, j > 0 ? 1 : 0, lc, q + j, beta + j, \
                           pb);                                                                 \
        break;
        if (win) {
#define LZ_VL_WIN(LV, NT, RING)                                                                            \
    hipLaunchKernelGGL((k_vl_spmv_win<T, LV, NT, RING>), dim3(grid), dim3(NT), 0, h->stream, n, rp, col, val, \
                       wcur, q0, wnext, pa, P, j > 0 ? 1 : 0, lc, q + j, beta + j, pb, band)
            if (win == 1) {
                if (lv == 4) LZ_VL_WIN(4, 512, 9216); else LZ_VL_WIN(8, 512, 9216);
            } else {
                if (lv == 4) LZ_VL_WIN(4, 1024, 16384); else LZ_VL_WIN(8, 1024, 16384);
            }
#undef LZ_VL_WIN
        } else if (cs) {  // fp64 only (cs is 0 otherwise); the casts are no-ops there
            auto vd = reinterpret_cast<const double *>(val);
            auto wc = reinterpret_cast<const double *>(wcur);
            auto qd = reinterpret_cast<double *>(q0), wd = reinterpret_cast<double *>(wnext);
            auto qr = reinterpret_cast<double *>(q + j), bj = reinterpret_cast<double *>(beta + j);
            if (cs == 1)
                hipLaunchKernelGGL((k_vl_spmv_cs<512, 3>), dim3(grid), dim3(512), 0, h->stream, n, nnz, rp,
                                   col, vd, wc, qd, wd, pa, P, j > 0 ? 1 : 0, lc, qr, bj, pb);
            else
                hipLaunchKernelGGL((k_vl_spmv_cs<256, 3>), dim3(grid), dim3(256), 0, h->stream, n, nnz, rp,
                                   col, vd, wc, qd, wd, pa, P, j > 0 ? 1 : 0, lc, qr, bj, pb);
        } else {
            switch (lv) {
                LZ_VL_CASE(4)
                LZ_VL_CASE(8)
                LZ_VL_CASE(16)
                LZ_VL_CASE(32)
                LZ_VL_CASE(64)
            }
        }
#undef LZ_VL_CASE
        prof_end(h, ev_s);
        LZ_LAUNCH_CHECK();
        const int ev_u = prof_begin(h, PROF_UPDATE_PASS);
        hipLaunchKernelGGL(k_vl_update<T>, dim3(gridu), dim3(kVlThreads), 0, h->stream, n, wnext, q0,
                           pb, grid, alpha + j, pa);
        prof_end(h, ev_u);
        LZ_LAUNCH_CHECK();
        P = gridu;
        wcur = wnext;
        wi ^= 1;
    }
    // the reference's post-call state (vector_lanczos.hpp:60,62): q0 = q1 =
    // q_{m-1} (q0 already holds it; q1 untouched at m = 1) and w = the last
    // residual, which alternated between w and q1
    if (wcur != w) LZ_HIP_TRY(hipMemcpyAsync(w, wcur, sizeof(T) * (size_t)n, hipMemcpyDeviceToDevice, h->stream));
    if (m >= 2) LZ_HIP_TRY(hipMemcpyAsync(q1, q0, sizeof(T) * (size_t)n, hipMemcpyDeviceToDevice, h->stream));
    return LZ_OK;
}

template int vector_lanczos_dev<double>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *,
                                        const double *, int, int64_t, const double *, double *, double *,
                                        double *, double *, double *, double *);
template int vector_lanczos_dev<float>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *,
                                       const float *, int, int64_t, const float *, float *, float *, float *,
                                       float *, float *, float *);

}  // namespace lz
