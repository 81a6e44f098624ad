// lz_spmm.hip -- CSR sparse x tall-skinny kernels for gfx950.
//
// Replaces the reference's ELL-4 kernels ell::SpMM / ell::SpMV
// (kernels/spmv_spmm.hpp:105-199).  Design (see DESIGN.md "SpMM"):
//   * CSR (int64 row_ptr, int32 col, T val); X / Y row-major n x b, so one
//     gathered X row is b*sizeof(T) contiguous bytes (128 B at b=16 fp64)
//     instead of b scattered 8-B loads of the reference's column-major block.
//   * one tile of consecutive rows per workgroup, XCD-remapped (xcd_remap) so
//     the tiles in flight on an XCD form a narrow row window and a banded
//     operator's X gather stays in that XCD's L2; the tile's (col, val) run is
//     staged through LDS in one batch of coalesced loads.
//   * one "group" of LPR = b*sizeof(T)/16 lanes per row, each lane owning a
//     16-byte slice of the row, 8 independent X gathers per lane per step.
//   * b == 1 (SpMV): CSR-vector, LV lanes per row with a wave64 xor-shuffle
//     reduction per row.
// Variants measured and dropped (DESIGN.md "SpMM variants"): grid-stride
// streaming, persistent queue with software pipelining, LDS-DMA gather.
#include "lz_common.hpp"
#include "lz_kernels.hpp"
#include "lz_internal.hpp"

namespace lz {

template <typename T, int B>
struct SpmmShape {
    static constexpr int VEC = (16 / (int)sizeof(T)) < B ? (16 / (int)sizeof(T)) : B;
    static constexpr int LPR = B / VEC;  // lanes per row
    static constexpr int RB = 256 / LPR; // rows per workgroup pass
};

// Store a finished nr x b Y tile (element (r, c) = get(r, c), in LDS) into a
// column-major Y (element (r, c) at r + c*ldy): nr contiguous elements per
// column, 16 B per lane where Y + r0 + c*ldy is 16-B aligned for every column
// (ldy and r0 multiples of 16 B / sizeof(T), Y aligned), else one element per lane.
template <typename T, typename Get>
__device__ __forceinline__ void store_tile_cm(T *__restrict__ Y, int64_t r0, int nr, int b, int64_t ldy, Get get)
{
    constexpr int EPV = 16 / (int)sizeof(T);
    const bool vec = ((reinterpret_cast<uintptr_t>(Y) & 15) == 0) && (ldy % EPV == 0) && (r0 % EPV == 0);
    if (vec) {
        const int nq = (nr + EPV - 1) / EPV;
        for (int idx = threadIdx.x; idx < b * nq; idx += blockDim.x) {
            const int c = idx / nq, r = (idx - c * nq) * EPV;
            T *dst = Y + r0 + r + (int64_t)c * ldy;
            if (r + EPV <= nr) {
                Vec<T, EPV> v;
#pragma unroll
                for (int e = 0; e < EPV; ++e) v.v[e] = get(r + e, c);
                stv<T, EPV>(dst, v);
            } else {
                for (int e = 0; r + e < nr; ++e) dst[e] = get(r + e, c);
            }
        }
    } else {
        for (int idx = threadIdx.x; idx < b * nr; idx += blockDim.x) {
            const int c = idx / nr, r = idx - c * nr;
            Y[(r0 + r) + (int64_t)c * ldy] = get(r, c);
        }
    }
}

// Tile-per-block SpMM (fallback for X >= 2 GiB or n >= 2^24).  A block owns a tile of
// RB*RPG consecutive rows; group gi (LPR lanes) owns rows gi + RB*j, j < RPG.
// The block stages the tile's (col, val) range into LDS with coalesced loads
// (one HBM round trip per tile, amortised over RPG gather rounds), then every
// group gathers its rows' X rows 8 nnz at a time (8 independent 16-byte loads
// per lane in flight), reading (col, val) from LDS.  One tile per block with
// the XCD remap keeps each XCD's in-flight tiles contiguous (L2-resident X
// window).  Tiles with more than CAP nnz are staged in CAP-sized chunks.
template <typename T, int B, int CAP, int RPG, bool YCM = false>
__global__ __launch_bounds__(256) void k_spmm_lds(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx, int64_t /*nx*/,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, UNR = 8, TR = RB * RPG;
    __shared__ __align__(16) int32_t cs[CAP];
    __shared__ T vs[CAP];
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int64_t r0 = xcd_remap(blockIdx.x, gridDim.x) * TR;
    const int64_t rend = (r0 + TR < n) ? r0 + TR : n;
    const int64_t kA = rp[r0], kB = rp[rend];
    int64_t k0[RPG], k1[RPG];
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        const int64_t row = r0 + gi + RB * j;
        k0[j] = row < n ? rp[row] : kB;
        k1[j] = row < n ? rp[row + 1] : kB;
    }
    const T *Xp = X + p * VEC;
    T acc[RPG][VEC];
#pragma unroll
    for (int j = 0; j < RPG; ++j)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[j][i] = T(0);
    for (int64_t c0 = kA; c0 < kB; c0 += CAP) {  // block-uniform
        const int64_t c1 = (c0 + CAP < kB) ? c0 + CAP : kB;
        if (c0 != kA) __syncthreads();
        for (int64_t k = c0 + tid; k < c1; k += 256) {
            cs[k - c0] = col[k];
            vs[k - c0] = val[k];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPG; ++j) {
            const int64_t a = k0[j] > c0 ? k0[j] : c0, e = k1[j] < c1 ? k1[j] : c1;
            for (int64_t kb = a; kb < e; kb += UNR) {  // group-uniform
                const int cnt = (int)((e - kb) < UNR ? (e - kb) : UNR);
                const int base = (int)(kb - c0);
                Vec<T, VEC> xs[UNR];
                T vv[UNR];
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    const int li = base + (t < cnt ? t : 0);
                    vv[t] = vs[li];
                    // exec-masked beyond the row's end
                    if (t < cnt) xs[t] = ldv<T, VEC>(Xp + (int64_t)cs[li] * ldx);
                }
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    if (t < cnt) {
#pragma unroll
                        for (int i = 0; i < VEC; ++i) acc[j][i] = fma(vv[t], xs[t].v[i], acc[j][i]);
                    }
                }
            }
        }
    }
    if constexpr (YCM) {  // column-major Y: the tile through LDS (over the staged run, so
                          // the kernel's LDS and occupancy stay as they are), TR
                          // contiguous elements per column
        constexpr bool ALIAS = sizeof(T) * B * (TR + 1) <= sizeof(int32_t) * CAP;
        T(*yt)[TR + 1];
        if constexpr (ALIAS) {
            __syncthreads();  // every wave is done with cs
            yt = reinterpret_cast<T(*)[TR + 1]>(cs);
        } else {
            __shared__ T ytb[B][TR + 1];
            yt = ytb;
        }
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int i = 0; i < VEC; ++i) yt[p * VEC + i][gi + RB * j] = acc[j][i];
        __syncthreads();
        store_tile_cm<T>(Y, r0, (int)(rend - r0), B, ldy, [&](int r, int c) { return yt[c][r]; });
        return;
    }
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        const int64_t row = r0 + gi + RB * j;
        if (row < n) {
            Vec<T, VEC> o;
#pragma unroll
            for (int i = 0; i < VEC; ++i) o.v[i] = acc[j][i];
            stv<T, VEC>(Y + row * ldy + p * VEC, o);
        }
    }
}

// VALU-lean variant of k_spmm_lds.  The gather of the tile kernel costs ~180
// VALU instructions per 8-load step (64-bit address arithmetic, an exec mask
// per load, index clamping); at ~60 % of the SIMDs' issue time (PMC:
// SQ_INSTS_VALU 468M for 22M VMEM reads) that, not memory, bounds it.  Here X
// is read through a buffer resource with 32-bit byte offsets (X must be
// < 2 GiB, n < 2^24), entries past the row's end get an out-of-range offset (the load
// returns 0 without touching memory, and fma(v, 0, acc) == acc), and the run
// is read from LDS at immediate offsets -- ~5 VALU per load.  The LDS run has
// UNR zeroed slack slots past the chunk so the tail reads are finite.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lz_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

template <typename T, int VEC, int AUX = 0>
__device__ __forceinline__ Vec<T, VEC> ldbuf(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    Vec<T, VEC> v;
    if constexpr (sizeof(T) * VEC == 16) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        __builtin_memcpy(&v, &u, 16);
    } else if constexpr (sizeof(T) * VEC == 8) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        __builtin_memcpy(&v, &u, 8);
    } else {
        const auto u = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
        __builtin_memcpy(&v, &u, 4);
    }
    return v;
}

template <typename T, int B, int CAP, int RPG, int UNR = 8, bool YCM = false>
__global__ __launch_bounds__(256) void k_spmm_buf(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx, int64_t nx,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, TR = RB * RPG;
    constexpr int EPV = 16 / (int)sizeof(T);                // values per 16-B load
    constexpr int SPTC = ((CAP + 4) / 4 + 255) / 256;         // 16-B col loads per thread
    constexpr int SPTV = ((CAP + EPV) / EPV + 255) / 256;     // 16-B val loads per thread
    __shared__ int32_t cs[CAP + UNR];
    __shared__ T vs[CAP + UNR];
    __shared__ int64_t rps[TR + 1];
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int64_t r0 = xcd_remap(blockIdx.x, gridDim.x) * TR;
    const int64_t rend = (r0 + TR < n) ? r0 + TR : n;
    const int64_t kA = rp[r0], kB = rp[rend];
    const int64_t nnz = rp[n];
    // the tile's row pointers: one load per thread, shared through LDS
    for (int t = tid; t <= TR; t += 256) rps[t] = rp[(r0 + t < rend) ? r0 + t : rend];
    const __amdgpu_buffer_rsrc_t xr = lz_rsrc(X, (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
    const uint32_t rowb = (uint32_t)(ldx * sizeof(T)), lane_off = p * VEC * sizeof(T);
    T acc[RPG][VEC];
#pragma unroll
    for (int j = 0; j < RPG; ++j)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[j][i] = T(0);
    int64_t k0[RPG], k1[RPG];
    for (int64_t c0 = kA; c0 < kB; c0 += CAP) {  // block-uniform
        const int64_t c1 = (c0 + CAP < kB) ? c0 + CAP : kB;
        if (c0 != kA) __syncthreads();
        {   // the chunk in one batch of 16-B loads (aligned down), scattered into LDS;
            // buffer bases at the chunk so offsets stay 32-bit for any nnz; a 16-B
            // piece reaching past nnz (last tile only) is read element-wise
            const int64_t bc = c0 & ~(int64_t)3, bv = c0 & ~(int64_t)(EPV - 1);
            const __amdgpu_buffer_rsrc_t cr = lz_rsrc(col + bc, 0x7fffffffu);
            const __amdgpu_buffer_rsrc_t vr = lz_rsrc(val + bv, 0x7fffffffu);
            int4 ct[SPTC];
            int4 vt[SPTV];
#pragma unroll
            for (int q = 0; q < SPTC; ++q) {
                const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
                ct[q] = int4{0, 0, 0, 0};
                if (k + 4 <= nnz && k < c1)
                    ct[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(cr, (uint32_t)((k - bc) * 4), 0, 0));
                else if (k < c1) {
                    ct[q].x = col[k];
                    if (k + 1 < nnz) ct[q].y = col[k + 1];
                    if (k + 2 < nnz) ct[q].z = col[k + 2];
                }
            }
#pragma unroll
            for (int q = 0; q < SPTV; ++q) {
                const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
                vt[q] = int4{0, 0, 0, 0};
                if (k + EPV <= nnz && k < c1) {
                    vt[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(vr, (uint32_t)((k - bv) * sizeof(T)), 0, 0));
                } else if (k < c1) {
                    T tv[EPV] = {};
                    for (int e = 0; e < EPV && k + e < nnz; ++e) tv[e] = val[k + e];
                    __builtin_memcpy(&vt[q], tv, 16);
                }
            }
#pragma unroll
            for (int q = 0; q < SPTC; ++q) {
                const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
                const int32_t cv[4] = {ct[q].x, ct[q].y, ct[q].z, ct[q].w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (k + e >= c0 && k + e < c1) cs[k + e - c0] = cv[e];
            }
#pragma unroll
            for (int q = 0; q < SPTV; ++q) {
                const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
                T tv[EPV];
                __builtin_memcpy(tv, &vt[q], 16);
#pragma unroll
                for (int e = 0; e < EPV; ++e)
                    if (k + e >= c0 && k + e < c1) vs[k + e - c0] = tv[e];
            }
        }
        if (tid < UNR) {  // finite slack past the chunk
            cs[c1 - c0 + tid] = 0;
            vs[c1 - c0 + tid] = T(0);
        }
        __syncthreads();
        if (c0 == kA) {
#pragma unroll
            for (int j = 0; j < RPG; ++j) {
                const int r = gi + RB * j;
                k0[j] = rps[r < TR ? r : TR];
                k1[j] = rps[r + 1 < TR ? r + 1 : TR];
            }
        }
#pragma unroll
        for (int j = 0; j < RPG; ++j) {
            const int a = (int)((k0[j] > c0 ? k0[j] : c0) - c0), e = (int)((k1[j] < c1 ? k1[j] : c1) - c0);
            for (int kb = a; kb < e; kb += UNR) {  // group-uniform
                const int cnt = e - kb;
                int32_t cc[UNR];
                T vv[UNR];
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    cc[t] = cs[kb + t];
                    vv[t] = vs[kb + t];
                }
                Vec<T, VEC> xs[UNR];
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    // n < 2^24 (checked at launch): 24-bit multiply is full rate
                    const uint32_t off =
                        t < cnt ? __umul24((unsigned)cc[t], rowb) + lane_off : 0x80000000u;
                    xs[t] = ldbuf<T, VEC>(xr, off);
                }
#pragma unroll
                for (int t = 0; t < UNR; ++t)
#pragma unroll
                    for (int i = 0; i < VEC; ++i) acc[j][i] = fma(vv[t], xs[t].v[i], acc[j][i]);
            }
        }
    }
    if constexpr (YCM) {  // column-major Y: the tile through LDS, TR contiguous elements per column
        __shared__ T yt[B][TR + 1];
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int i = 0; i < VEC; ++i) yt[p * VEC + i][gi + RB * j] = acc[j][i];
        __syncthreads();
        store_tile_cm<T>(Y, r0, (int)(rend - r0), B, ldy, [&](int r, int c) { return yt[c][r]; });
        return;
    }
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        const int64_t row = r0 + gi + RB * j;
        if (row < n) {
            Vec<T, VEC> o;
#pragma unroll
            for (int i = 0; i < VEC; ++i) o.v[i] = acc[j][i];
            stv<T, VEC>(Y + row * ldy + p * VEC, o);
        }
    }
}

// nnz-split SpMM with row results through LDS.  Every gather wave-instruction
// costs the texture path the same ~16 cycles whatever its live lanes (the TA
// is ~97 % busy in k_spmm_buf, PMC r01), so the lever is live lanes per
// instruction: each group of LPR lanes walks an equal, 8-aligned slice of the
// tile's nonzero run regardless of row boundaries (all 8 loads of a step live
// except in a group's last step).  A row that ends inside a group's slice is
// written to an LDS Y tile (ds_write, no texture-path cost -- the first
// nnz-split kernel stored it to global from inside the divergent loop, one
// partial-exec store instruction per row end, which ate the gain); a group's
// first and last rows go to head/tail slots and are summed in a fixed order,
// so results stay bitwise reproducible; the Y tile leaves with full-lane
// coalesced stores.
// WIN (X of 2^24+ rows or >= 2 GiB, 128-B rows): X is read through a buffer
// resource based at the tile's smallest column (found while the run is
// staged), so offsets stay 32-bit; a tile whose columns span more than the
// window goes to the long-tile queue, whose kernel then gathers with 64-bit
// addresses.  Banded operators of any size keep the buffer-addressed gather
// (BASELINE config C4: 40M rows on one GPU).
// YCM: Y is column-major (element (r, c) at r + c*ldy, the reference's
// Dense_matrix layout): the finished Y tile leaves column by column, nrows
// contiguous elements per column (the caller transposed X in).
// U row piece = Y piece - Wp[row] . M[:, piece] (k in order, one fma chain per
// element): the C5 beta^2 epilogue of k_spmm_seg (EPI).
// The B / VEC = 8 lanes of a row (consecutive lanes) each load one 16-B piece
// of the row and pass it round by lane shuffles: one load per piece, not B / 4.
template <typename T, int B, int VEC>
__device__ __forceinline__ Vec<T, VEC> epi_piece(Vec<T, VEC> y, const T *__restrict__ wrow, const T *Ms, int pc)
{
    static_assert(B / 4 == 8 && VEC == 4, "b = 32 fp32 rows: 8 lanes of 4 values");
    // W_{j-1} is streamed once: a non-temporal load, so it does not push the
    // gathered W_j rows out of the caches (C5 SpMM 2.937 -> 2.893 ms,
    // profiles/r05o_c5_epi_nt_ab.log)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v m4 = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(wrow + 4 * pc));
    const float4 mine = make_float4(m4.x, m4.y, m4.z, m4.w);
    const int base = (int)(threadIdx.x & 63) & ~7;
#pragma unroll
    for (int k4 = 0; k4 < B / 4; ++k4) {
        const T w[4] = {__shfl(mine.x, base + k4, 64), __shfl(mine.y, base + k4, 64), __shfl(mine.z, base + k4, 64),
                        __shfl(mine.w, base + k4, 64)};
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < VEC; ++i) y.v[i] = fma(-w[e], Ms[(4 * k4 + e) * B + pc * VEC + i], y.v[i]);
    }
    return y;
}

// ---- CU-partitioned SpMM (LZ_SPMM_PF, diagnostic build only: measured and
// dropped in round 6, DESIGN.md 4 SpMM "Round 6") ----
// The tile kernel runs on a stream masked to most of each XCD's CUs; a
// prefetch kernel on the rest pulls the CSR runs, row pointers and the X rows
// the XCD's next tiles touch first into that XCD's L2, paced by the number of
// tile blocks the XCD has started.  Control words: one 128-B line per XCC
// (only that XCD's CUs touch it, so workgroup-scope atomics -- performed in
// the XCD's own L2, not at memory like agent-scope ones on a multi-XCD chip
// -- are enough; round 6's first version used agent scope and its contended
// memory-side atomics took the launch from 1.2 to 6.5-17.6 ms):
//   [32 x + 0]  tile blocks started on XCC x        (tile kernel)
//   [32 x + 1]  XCC x's block group blockIdx % 8    (tile kernel; -1 until known)
//   [32 x + 2]  prefetch chunk ticket
//   [32 x + 3]  highest X row prefetched (-1 at the start)
[[maybe_unused]] constexpr int kPfCtl = 256;

__device__ __forceinline__ int xcc_id()
{
    return (int)(__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 7u);  // HW_REG_XCC_ID
}

template <typename T, int B, int TR, int CAP, bool WIN, int MODE, bool YCM = false, bool EPI = false, bool PF = false>
__global__ __launch_bounds__(256) void k_spmm_seg(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx, int64_t nx,
                                                  T *__restrict__ Y, int64_t ldy, int *__restrict__ longq,
                                                  int parity, const T *__restrict__ Wp, const T *__restrict__ Mm,
                                                  int diag, int *__restrict__ pfc)
{
    // MODE 0: tiles whose run exceeds the stage (or, WIN, whose columns exceed
    //         the window) are queued (longq[0] = count, longq[1..] = tile ids)
    //         for MODE 1, so their code path costs the main kernel no registers;
    // MODE 1: persistent blocks over the queued tiles: CAP-sized chunks, each
    //         split over the 32 groups; rows accumulate in the LDS Y tile
    //         across chunks (chunk order, then group order: bitwise
    //         reproducible).  A row-wise walk would leave one 8-lane group
    //         serialising a 10^5-entry row (power-law degrees, config 5).
    using S = SpmmShape<T, B>;
    // UNR: gathers in flight per lane per step.  16 measured slower at both C3
    // (118 VGPRs, 1.34 vs 1.15 ms) and C5 (124 VGPRs, 4 waves per SIMD: 3.25
    // vs 2.96 ms, profiles/r05b_c5_unr_ab.log)
    constexpr int VEC = S::VEC, LPR = S::LPR, G = 256 / LPR, UNR = 8;
    static_assert(TR <= 255, "row ids are bytes");
    __shared__ int32_t rel[TR + 1];
    __shared__ int32_t cs[CAP + UNR];
    __shared__ T vs[CAP + UNR];
    __shared__ uint8_t rid[CAP + UNR];
    __shared__ Vec<T, VEC> yt[TR][LPR];      // the tile's finished rows
    __shared__ Vec<T, VEC> head[G][LPR];     // a group's piece of a row begun in an earlier slice
    __shared__ int32_t cmin, cmax;           // WIN: the tile's column range
    // EPI (b = 32 fp32, the C5 Q-free step in its beta^2 form): the stored row
    // is U = Y - Wp M (Wp: W_{j-1}, M = beta_{j-1}^-1 G_j, 32 x 32 in LDS)
    __shared__ T Ms[EPI ? B * B : 1];
    const int tid = threadIdx.x;
    const bool epi = EPI && Wp != nullptr;
    if (epi)
        for (int e = tid; e < B * B; e += 256) Ms[e] = Mm[e];  // visible after the staging barriers
    const int gi = tid / LPR, p = tid % LPR;
    const uint32_t rowb = (uint32_t)(ldx * sizeof(T)), lane_off = p * VEC * sizeof(T);
    Vec<T, VEC> zero;
#pragma unroll
    for (int i = 0; i < VEC; ++i) zero.v[i] = T(0);
    if constexpr (MODE == 1) {
        const __amdgpu_buffer_rsrc_t xr = lz_rsrc(X, WIN ? 0u : (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
        // the gather of one step: buffer loads, or (WIN) 64-bit addressed loads
        auto gather = [&](const int32_t cc[UNR], int live, Vec<T, VEC> xs[UNR]) {
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                if constexpr (WIN) {
                    xs[t] = t < live ? ldv<T, VEC>(X + (int64_t)cc[t] * ldx + p * VEC) : zero;
                } else {
                    const uint32_t off = t < live ? __umul24((unsigned)cc[t], rowb) + lane_off : 0x80000000u;
                    xs[t] = ldbuf<T, VEC>(xr, off);
                }
            }
        };
        // this launch's count slot; the other slot is zeroed for the next launch
        // (no memset per call: the queue counts alternate between longq[0] / [1]).
        // parity 2 / 3: a planned launch -- the list an earlier call queued
        // (count at longq[parity - 2]), left as it is for the next planned call
        const bool planned = parity >= 2;
        const int cnt = longq[planned ? parity - 2 : parity];
        if (!planned && blockIdx.x == 0 && threadIdx.x == 0) longq[parity ^ 1] = 0;
        for (int qi = blockIdx.x; qi < cnt; qi += gridDim.x) {
            const int64_t r0 = (int64_t)longq[2 + qi] * TR;
            const int nrows = (int)((n - r0) < TR ? (n - r0) : TR);
            const int64_t kA = rp[r0];
            __syncthreads();  // the previous tile is done with rel / yt
            if (tid <= nrows) rel[tid] = (int)(rp[r0 + tid] - kA);
            const int64_t N64 = rp[r0 + nrows] - kA;
            for (int idx = tid; idx < TR * LPR; idx += 256) yt[idx / LPR][idx % LPR] = zero;
            for (int64_t c0 = kA; c0 < kA + N64; c0 += CAP) {
                const int64_t c1 = (c0 + CAP < kA + N64) ? c0 + CAP : kA + N64;
                const int Nc = (int)(c1 - c0), cb = (int)(c0 - kA);  // chunk length, offset in the run
                __syncthreads();  // rel visible; the previous chunk is done with cs / vs / rid / head
                for (int k = tid; k < Nc; k += 256) {
                    // (streamed once: non-temporal, as the tile pass's staging)
                    cs[k] = __builtin_nontemporal_load(&col[c0 + k]);
                    vs[k] = __builtin_nontemporal_load(&val[c0 + k]);
                    int lo = 0, hi = nrows - 1;  // the row holding entry cb + k: rel[r] <= cb + k < rel[r + 1]
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (rel[mid] <= cb + k) lo = mid;
                        else hi = mid - 1;
                    }
                    rid[k] = (uint8_t)lo;
                }
                if (tid < UNR) {
                    cs[Nc + tid] = 0;
                    vs[Nc + tid] = T(0);
                    rid[Nc + tid] = 255;
                }
                __syncthreads();
                const int E = ((Nc + G - 1) / G + UNR - 1) / UNR * UNR;
                const int start = gi * E, end = (start + E < Nc) ? start + E : Nc;
                if (start < end) {  // group-uniform
                    int cur = rid[start];
                    bool open = (rel[cur] - cb > 0 ? rel[cur] - cb : 0) < start;
                    Vec<T, VEC> acc = zero;
                    auto flush = [&]() {
                        if (open) {
                            head[gi][p] = acc;
                        } else {
#pragma unroll
                            for (int i2 = 0; i2 < VEC; ++i2) yt[cur][p].v[i2] += acc.v[i2];
                        }
                    };
                    for (int s0 = start; s0 < end; s0 += UNR) {
                        int32_t cc[UNR];
                        T vv[UNR];
                        int rr[UNR];
#pragma unroll
                        for (int t = 0; t < UNR; ++t) {
                            cc[t] = cs[s0 + t];
                            vv[t] = vs[s0 + t];
                            rr[t] = rid[s0 + t];
                        }
                        Vec<T, VEC> xs[UNR];
                        gather(cc, end - s0, xs);
#pragma unroll
                        for (int t = 0; t < UNR; ++t) {
                            const int r = s0 + t < end ? rr[t] : cur;
                            if (r != cur) {
                                flush();
                                acc = zero;
                                cur = r;
                                open = false;
                            }
#pragma unroll
                            for (int i2 = 0; i2 < VEC; ++i2) acc.v[i2] = fma(vv[t], xs[t].v[i2], acc.v[i2]);
                        }
                    }
                    flush();
                }
                __syncthreads();
                for (int r = gi; r < nrows; r += G) {  // rows over several slices of this chunk
                    const int a = (rel[r] > cb ? rel[r] : cb) - cb,
                              e = (rel[r + 1] < cb + Nc ? rel[r + 1] : cb + Nc) - cb;
                    if (a >= e) continue;
                    const int g1 = a / E, g2 = (e - 1) / E;
                    for (int g = g1 + 1; g <= g2; ++g) {
#pragma unroll
                        for (int i2 = 0; i2 < VEC; ++i2) yt[r][p].v[i2] += head[g][p].v[i2];
                    }
                }
            }
            __syncthreads();
            if constexpr (YCM) {
                store_tile_cm<T>(Y, r0, nrows, B, ldy, [&](int r, int c) { return yt[r][c / VEC].v[c % VEC]; });
            } else {
                for (int idx = tid; idx < nrows * LPR; idx += 256) {
                    Vec<T, VEC> y = yt[idx / LPR][idx % LPR];
                    if constexpr (EPI)
                        if (epi) y = epi_piece<T, B, VEC>(y, Wp + (r0 + idx / LPR) * B, Ms, idx % LPR);
                    stv<T, VEC>(Y + (r0 + idx / LPR) * ldy + (idx % LPR) * VEC, y);
                }
            }
        }
        return;
    } else {
    // diag > 0 (LZ_SPMM_DIAG, a measurement of the tile structure, results
    // wrong): block b runs tile mid + (its tile mod diag), so the row pointers,
    // CSR runs, X window and Y rows of all blocks are those of `diag` tiles --
    // L2-resident -- from the middle of the operator (rows with the full band,
    // so the same entries per row and per-tile instruction mix as the real run)
    // (diag bit 30: the Y rows stored stay the block's own, so only the reads
    // are L2-resident)
    const int64_t tdx = xcd_remap(blockIdx.x, gridDim.x);
    const int dmod = diag > 0 ? diag & 0x3fffffff : 0;  // (diag < 0: the LZ_SPMM_HOT probe below)
    const int64_t dmid = dmod > 0 ? ((int64_t)gridDim.x / 2 / dmod) * dmod : 0;
    const int64_t r0 = (dmod > 0 ? tdx % dmod + dmid : tdx) * TR;
    const int64_t ry = (diag > 0 && (diag & (1 << 30))) ? tdx * TR : r0;  // the Y tile's first row
    const int nrows = (int)((n - r0) < TR ? (n - r0) : TR);
    const int64_t kA = rp[r0];
    if (tid <= nrows) rel[tid] = (int)(rp[r0 + tid] - kA);
    if constexpr (WIN) {
        if (tid == 0) {
            cmin = 0x7fffffff;
            cmax = -1;
        }
    }
    const int64_t N64 = rp[r0 + nrows] - kA;
    if (N64 > CAP) {  // block-uniform (planned: the listed tile runs in the long-tile pass)
        if (tid == 0 && parity < 2) longq[2 + atomicAdd(&longq[parity], 1)] = (int)(r0 / TR);
        return;
    }
    const int N = (int)N64;
    if constexpr (PF) {  // publish this block's start to the XCD's prefetcher
        if (tid == 0) {
            const int x = xcc_id();
            __hip_atomic_fetch_add(&pfc[32 * x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((blockIdx.x >> 3) < 8)
                __hip_atomic_exchange(&pfc[32 * x + 1], (int)(blockIdx.x & 7), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    {  // stage the run with 16-B loads (aligned down; a piece reaching past nnz,
       // last tile only, element-wise), then the row id of every entry
        constexpr int EPV = 16 / (int)sizeof(T);
        constexpr int SPTC = ((CAP + 4) / 4 + 255) / 256, SPTV = ((CAP + EPV) / EPV + 255) / 256;
        const int64_t nnz = rp[n], kB = kA + N;
        const int64_t bc = kA & ~(int64_t)3, bv = kA & ~(int64_t)(EPV - 1);
        const __amdgpu_buffer_rsrc_t cr = lz_rsrc(col + bc, 0x7fffffffu);
        const __amdgpu_buffer_rsrc_t vr = lz_rsrc(val + bv, 0x7fffffffu);
        constexpr int AUX = 2;  // nt: streamed once, keep the X window in L2
        int4 ct[SPTC];
        int4 vt[SPTV];
#pragma unroll
        for (int q = 0; q < SPTC; ++q) {
            const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
            ct[q] = int4{0, 0, 0, 0};
            if (k + 4 <= nnz && k < kB)
                ct[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(cr, (uint32_t)((k - bc) * 4), 0, AUX));
            else if (k < kB) {
                ct[q].x = col[k];
                if (k + 1 < nnz) ct[q].y = col[k + 1];
                if (k + 2 < nnz) ct[q].z = col[k + 2];
            }
        }
#pragma unroll
        for (int q = 0; q < SPTV; ++q) {
            const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
            vt[q] = int4{0, 0, 0, 0};
            if (k + EPV <= nnz && k < kB) {
                vt[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(vr, (uint32_t)((k - bv) * sizeof(T)), 0, AUX));
            } else if (k < kB) {
                T tv[EPV] = {};
                for (int e = 0; e < EPV && k + e < nnz; ++e) tv[e] = val[k + e];
                __builtin_memcpy(&vt[q], tv, 16);
            }
        }
        __syncthreads();  // rel (and, WIN, the column range's initial values)
        if (tid < nrows)
            for (int k = rel[tid]; k < rel[tid + 1]; ++k) rid[k] = (uint8_t)tid;
        int lmin = 0x7fffffff, lmax = -1;
#pragma unroll
        for (int q = 0; q < SPTC; ++q) {
            const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
            const int32_t cv[4] = {ct[q].x, ct[q].y, ct[q].z, ct[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (k + e >= kA && k + e < kB) {
                    cs[k + e - kA] = cv[e];
                    if constexpr (WIN) {
                        lmin = cv[e] < lmin ? cv[e] : lmin;
                        lmax = cv[e] > lmax ? cv[e] : lmax;
                    }
                }
        }
        if constexpr (WIN) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const int a = __shfl_xor(lmin, o, 64), b2 = __shfl_xor(lmax, o, 64);
                lmin = a < lmin ? a : lmin;
                lmax = b2 > lmax ? b2 : lmax;
            }
            if ((tid & 63) == 0) {
                atomicMin(&cmin, lmin);
                atomicMax(&cmax, lmax);
            }
        }
#pragma unroll
        for (int q = 0; q < SPTV; ++q) {
            const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
            T tv[EPV];
            __builtin_memcpy(tv, &vt[q], 16);
#pragma unroll
            for (int e = 0; e < EPV; ++e)
                if (k + e >= kA && k + e < kB) vs[k + e - kA] = tv[e];
        }
        if (tid < UNR) {
            cs[N + tid] = 0;
            vs[N + tid] = T(0);
            rid[N + tid] = 255;
        }
        __syncthreads();
    }
    // the gather source: all of X, or (WIN) a window based at the tile's smallest column
    uint32_t wb = 0;
    __amdgpu_buffer_rsrc_t xr;
    if constexpr (WIN) {
        const int64_t lo = N > 0 ? cmin : 0, span = N > 0 ? (int64_t)cmax - cmin + 1 : 0;
        const int64_t wrows = (int64_t)(0x7fffffff / rowb) < kWinRows ? (int64_t)(0x7fffffff / rowb) : kWinRows;
        if (span > wrows) {  // block-uniform: columns too far apart for one window
            if (tid == 0 && parity < 2) longq[2 + atomicAdd(&longq[parity], 1)] = (int)(r0 / TR);
            return;
        }
        wb = (uint32_t)lo;
        xr = lz_rsrc(X + lo * ldx, (uint32_t)(span * rowb));
    } else {
        xr = lz_rsrc(X, (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
    }
    const int E = ((N + G - 1) / G + UNR - 1) / UNR * UNR;  // slice length, UNR-aligned
    const int start = gi * E, end = (start + E < N) ? start + E : N;
    if (start < end) {  // group-uniform
        int cur = rid[start];
        bool open = rel[cur] < start;  // cur began in an earlier group's slice
        Vec<T, VEC> acc = zero;
        for (int s0 = start; s0 < end; s0 += UNR) {
            int32_t cc[UNR];
            T vv[UNR];
            int rr[UNR];
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                cc[t] = cs[s0 + t];
                vv[t] = vs[s0 + t];
                rr[t] = rid[s0 + t];
            }
            Vec<T, VEC> xs[UNR];
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                const uint32_t off =
                    s0 + t < end ? __umul24((unsigned)cc[t] - wb, rowb) + lane_off : 0x80000000u;
#ifdef LZ_DIAG
                if (diag < 0) {  // (LZ_SPMM_HOT: columns < K gathered with the default policy, the rest with aux)
                    const int hk = (-diag) & 0xffffff, ha = ((-diag) >> 24) & 3;
                    if (cc[t] < hk) xs[t] = ldbuf<T, VEC>(xr, off);
                    else if (ha == 1) xs[t] = ldbuf<T, VEC, 2>(xr, off);
                    else if (ha == 2) xs[t] = ldbuf<T, VEC, 16>(xr, off);
                    else xs[t] = ldbuf<T, VEC, 18>(xr, off);
                    continue;
                }
#endif
                xs[t] = ldbuf<T, VEC>(xr, off);
            }
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                const int r = s0 + t < end ? rr[t] : cur;
                if (r != cur) {  // row cur ends inside the slice
                    if (open) head[gi][p] = acc;
                    else yt[cur][p] = acc;  // a whole row
                    acc = zero;
                    cur = r;
                    open = false;
                }
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc.v[i] = fma(vv[t], xs[t].v[i], acc.v[i]);
            }
        }
        // the slice's last row: whole, or the first piece of a row later slices continue
        if (open) head[gi][p] = acc;
        else yt[cur][p] = acc;
    }
    __syncthreads();
    // rows over several slices: first piece (in yt) + the later groups' heads,
    // in group order; empty rows
    for (int r = gi; r < nrows; r += G) {
        const int a = rel[r], e = rel[r + 1];
        if (a == e) {
            yt[r][p] = zero;
            continue;
        }
        const int g1 = a / E, g2 = (e - 1) / E;
        if (g1 == g2) continue;
        Vec<T, VEC> sum = yt[r][p];
        for (int g = g1 + 1; g <= g2; ++g) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) sum.v[i] += head[g][p].v[i];
        }
        yt[r][p] = sum;
    }
    __syncthreads();
    if constexpr (YCM) {
        store_tile_cm<T>(Y, r0, nrows, B, ldy, [&](int r, int c) { return yt[r][c / VEC].v[c % VEC]; });
        return;
    }
    for (int idx = tid; idx < nrows * LPR; idx += 256) {
        if (ry + idx / LPR >= n) break;  // (diag only: a Y tile shorter than the tile read)
        T *dst = Y + (ry + idx / LPR) * ldy + (idx % LPR) * VEC;
        Vec<T, VEC> y = yt[idx / LPR][idx % LPR];
        if constexpr (EPI)
            if (epi) y = epi_piece<T, B, VEC>(y, Wp + (r0 + idx / LPR) * B, Ms, idx % LPR);
        if constexpr (sizeof(T) * VEC == 16) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4 u;
            __builtin_memcpy(&u, &y, 16);
            __builtin_nontemporal_store(u, reinterpret_cast<u32x4 *>(dst));
        } else {
            stv<T, VEC>(dst, y);
        }
    }
    }  // MODE 0
}

#ifdef LZ_DIAG  // (measured and dropped in round 6: the diagnostic build only)
// The prefetch side of the CU-partitioned SpMM.  Persistent blocks, each on
// the XCD it reads from HW_REG_XCC_ID: the XCD's tiles (xcd_remap's range for
// its block group) are cut into chunks of C tiles, claimed in order by ticket;
// chunk c waits until the XCD has started c*C - D tile blocks (never more than
// D tiles ahead of the dispatch front) and skips itself when the front has
// passed it.  A chunk's rows [ra, rb) read four contiguous byte ranges: their
// row pointers, their CSR columns and values, and the X rows their band first
// reaches on this XCD, [ra + hw, rb + hw) (hw: the operator's largest
// |column - row|, once per operator; the XCD's first chunk also the band
// below, [ra - hw, ra + hw)).  The block streams them by LDS-DMA into a
// scratch slot it never reads (1 KB per wave-instruction, no register
// destinations, no waits but the last): the data only has to be in the XCD's
// L2 when the tile blocks read it.  Every wait is bounded, and nothing here
// affects results.
template <int TR>
__global__ __launch_bounds__(256) void k_spmm_pf(int64_t n, int64_t ntiles, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ col, const char *__restrict__ val,
                                                 int vsz, const char *__restrict__ X, int64_t nx, int rowb,
                                                 int *__restrict__ ctl, int C, int D, int64_t hw)
{
    __shared__ __attribute__((aligned(16))) char trash[4][1024];
    __shared__ int s_g;
    __shared__ int64_t s_c;
    const int tid = threadIdx.x, lane = tid & 63, x = xcc_id();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid == 0) {
        int g = -1;
        for (int it = 0; it < (1 << 14); ++it) {
            g = __hip_atomic_fetch_add(&ctl[32 * x + 1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (g >= 0) break;
            __builtin_amdgcn_s_sleep(8);
        }
        s_g = g;
    }
    __syncthreads();
    const int g = __builtin_amdgcn_readfirstlane(s_g);
    if (g < 0) return;  // the XCD ran no tile block in time (bounded wait)
    const int64_t q = ntiles >> 3, r8 = ntiles & 7;
    const int64_t t0 = g < r8 ? g * (q + 1) : r8 * (q + 1) + (g - r8) * q, len = q + (g < r8 ? 1 : 0);
    const int64_t nch = (len + C - 1) / C;
    // the block's pieces of one byte range [b0, b1), 1 KB per wave-instruction
    auto stream = [&](const char *base, int64_t b0, int64_t b1) {
        if (b1 <= b0) return;
        b0 &= ~(int64_t)15;
        const int64_t pieces = (b1 - b0 + 1023) >> 10;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<char *>(base + b0), (short)0, (int)(b1 - b0), 0x00020000);
        for (int64_t p = w; p < pieces; p += 4)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (ws_lds_t *)&trash[w][0], 16, (uint32_t)(p * 1024 + 16 * lane),
                                                     0, 0, 0);
    };
    for (;;) {
        if (tid == 0) {
            int64_t c = __hip_atomic_fetch_add(&ctl[32 * x + 2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int64_t need = c * C - D;
            bool ok = c >= nch;
            for (int it = 0; it < (1 << 14) && !ok; ++it) {
                ok = __hip_atomic_fetch_add(&ctl[32 * x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= need;
                if (!ok) __builtin_amdgcn_s_sleep(2);
            }
            if (!ok) c = nch;  // the tile blocks stopped advancing: give up (bounded)
            // the front has passed the whole chunk: nothing left to pull ahead
            if (c < nch &&
                __hip_atomic_fetch_add(&ctl[32 * x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (c + 1) * C)
                c = -1 - c;
            s_c = c;
        }
        __syncthreads();
        // (wave-uniform in the compiler's eyes too: scalar resources below, no
        // readfirstlane loops around the DMAs)
        const int64_t c = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)s_c >> 32)) << 32) |
                                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s_c));
        __syncthreads();  // (s_c is rewritten by the next claim)
        if (c >= nch) break;
        if (c < 0) continue;
        const int64_t ta = t0 + c * C, tb = (c + 1) * C < len ? ta + C : t0 + len;
        const int64_t ra = ta * TR, rb = tb * TR < n ? tb * TR : n;
        const int64_t ka = rp[ra], kb = rp[rb];
        stream(reinterpret_cast<const char *>(rp), ra * 8, (rb + 1) * 8);
        stream(reinterpret_cast<const char *>(col), ka * 4, kb * 4);
        stream(val, ka * vsz, kb * vsz);
        int64_t x0 = c == 0 ? ra - hw : ra + hw, x1 = rb + hw;
        x0 = x0 < 0 ? 0 : x0;
        x1 = x1 > nx ? nx : x1;
        stream(X, x0 * rowb, x1 * rowb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no DMA into LDS the block has released)
}

// the operator's band: max |column - row| (the prefetcher's X lead), atomics
// on one word
__global__ __launch_bounds__(256) void k_band(int64_t n, const int64_t *__restrict__ rp,
                                              const int32_t *__restrict__ col, int *__restrict__ out)
{
    int m = 0;
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256)
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
            const int64_t d = (int64_t)col[k] - r;
            const int a = (int)(d < 0 ? -d : d);
            m = a > m ? a : m;
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int v = __shfl_xor(m, o, 64);
        m = v > m ? v : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

__global__ void k_pf_init(int *ctl)
{
    const int i = threadIdx.x;
    if (i < kPfCtl) ctl[i] = (i % 32 == 1 || i % 32 == 3) ? -1 : 0;
}
#endif  // LZ_DIAG

// Row-major SpMM at a block width off the tuned set (b not a power of two):
// thread (r, c) sums row r in CSR order; the b threads of a row read the same
// (col, val) line and b contiguous elements of each gathered X row.
template <typename T>
__global__ __launch_bounds__(256) void k_spmm_any_b(int64_t n, int b, const int64_t *__restrict__ rp,
                                                    const int32_t *__restrict__ col, const T *__restrict__ val,
                                                    const T *__restrict__ X, int64_t ldx, T *__restrict__ Y,
                                                    int64_t ldy)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * b; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / b;
        const int c = (int)(i - r * b);
        T acc = T(0);
        for (int64_t k = rp[r], e = rp[r + 1]; k < e; ++k) acc = fma(val[k], X[(int64_t)col[k] * ldx + c], acc);
        Y[r * ldy + c] = acc;
    }
}

// Column-major compatibility path (the reference's Dense_matrix layout,
// element (r,c) at r + c*ld).  One thread per row; any b.
template <typename T>
__global__ __launch_bounds__(256) void k_spmm_cm(int64_t n, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ col,
                                                 const T *__restrict__ val, int b,
                                                 const T *__restrict__ X, int64_t ldx,
                                                 T *__restrict__ Y, int64_t ldy)
{
    for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n;
         row += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k0 = rp[row], k1 = rp[row + 1];
        for (int c = 0; c < b; ++c) {
            T acc = T(0);
            for (int64_t k = k0; k < k1; ++k) acc = fma(val[k], X[(int64_t)col[k] + c * ldx], acc);
            Y[row + c * ldy] = acc;
        }
    }
}

// CSR-vector SpMV: LV lanes per row, strided nnz, xor-shuffle reduction.
template <typename T, int LV>
__global__ __launch_bounds__(256) void k_spmv(int64_t n, const int64_t *__restrict__ rp,
                                              const int32_t *__restrict__ col,
                                              const T *__restrict__ val, const T *__restrict__ x,
                                              T *__restrict__ y)
{
    constexpr int RB = 256 / LV;
    const int gi = threadIdx.x / LV, p = threadIdx.x % LV;
    XcdSched sch(ceil_div(n, RB));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t row = u * RB + gi;
        const bool valid = row < n;
        const int64_t k0 = valid ? rp[row] : 0, k1 = valid ? rp[row + 1] : 0;
        T acc = T(0);
        int64_t k = k0 + p;
        for (; k + LV < k1; k += 2 * LV) {
            const int c0 = col[k], c1 = col[k + LV];
            const T v0 = val[k], v1 = val[k + LV];
            acc = fma(v0, x[c0], acc);
            acc = fma(v1, x[c1], acc);
        }
        if (k < k1) acc = fma(val[k], x[col[k]], acc);
#pragma unroll
        for (int off = LV / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (valid && p == 0) y[row] = acc;
    }
}

// ---------------------------------------------------------------------------
// Fixed-nnz tiles (experiment; LZ_SPMM_FNZ=1 selects it for 128-B rows).
// Tile t owns the rows whose FIRST entry lies in [tK, (t+1)K): the CSR window
// it stages, entries [tK - 1, tK + K + S), is known from t alone, so the run's
// loads issue at once, beside the one load of its first row trow[t] -- no
// row-pointer round trip ahead of them.  Row ends ride in bit 31 of a copy of
// the column index (colf, built once per operator), so row starts, row ids and
// row offsets come from one block scan over the staged flags.  Requires: no
// empty rows, every row <= S + 1 entries, at most RMAX rows per tile, columns
// < 2^31 (fnz_prepare checks, else the default kernel runs).
constexpr int kFnzK = 448, kFnzS = 64, kFnzRmax = 88;

__global__ __launch_bounds__(256) void k_fnz_flags(int64_t n, const int64_t *__restrict__ rp,
                                                   const int32_t *__restrict__ col, int32_t *__restrict__ colf,
                                                   int *__restrict__ stats)
{
    int maxlen = 0, bad = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = rp[r], e = rp[r + 1];
        const int64_t len = e - a;
        maxlen = len > maxlen ? (int)(len < (1 << 30) ? len : (1 << 30)) : maxlen;
        bad |= len == 0;
        for (int64_t k = a; k < e; ++k) {
            const int32_t c = col[k];
            bad |= c < 0;
            colf[k] = (int32_t)((uint32_t)c | (k == e - 1 ? 0x80000000u : 0u));
        }
    }
    atomicMax(&stats[0], maxlen);
    if (bad) atomicOr(&stats[1], 1);
}

// trow[t] = first row whose first entry is >= t*K (rows before it start earlier)
__global__ __launch_bounds__(256) void k_fnz_trow(int64_t ntiles, int64_t n, const int64_t *__restrict__ rp, int K,
                                                  int32_t *__restrict__ trow, int *__restrict__ stats)
{
    int maxrows = 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t key = t * K;
        int64_t lo = 0, hi = n;  // smallest r in [0, n] with rp[r] >= key
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (rp[mid] >= key) hi = mid;
            else lo = mid + 1;
        }
        trow[t] = (int32_t)lo;
        if (t > 0) {  // rows of tile t - 1
            int64_t lo2 = 0, hi2 = n;
            const int64_t key2 = (t - 1) * (int64_t)K;
            while (lo2 < hi2) {
                const int64_t mid = (lo2 + hi2) >> 1;
                if (rp[mid] >= key2) hi2 = mid;
                else lo2 = mid + 1;
            }
            const int64_t nr = lo - lo2;
            maxrows = nr > maxrows ? (int)(nr < (1 << 30) ? nr : (1 << 30)) : maxrows;
        }
    }
    atomicMax(&stats[2], maxrows);
}

template <typename T, int B, int K, int S, int RMAX>
__global__ __launch_bounds__(256) void k_spmm_fnz(int64_t nnz, const int32_t *__restrict__ colf,
                                                  const T *__restrict__ val, const int32_t *__restrict__ trow,
                                                  const T *__restrict__ X, int64_t ldx, int64_t nx,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using Sh = SpmmShape<T, B>;
    constexpr int VEC = Sh::VEC, LPR = Sh::LPR, G = 256 / LPR, UNR = 8;
    constexpr int WIN = K + S + 1;           // local i <-> entry tK - 1 + i
    constexpr int EPT = (WIN + 255) / 256;   // scan: entries per thread
    static_assert(RMAX <= 255 && K % 4 == 0, "row ids are bytes; 16-B column pieces");
    __shared__ int32_t cs[WIN + UNR];
    __shared__ T vs[WIN + UNR];
    __shared__ uint8_t rid[WIN + UNR];
    __shared__ int32_t rel[RMAX + 1];
    __shared__ Vec<T, VEC> yt[RMAX][LPR];
    __shared__ Vec<T, VEC> head[G][LPR];
    __shared__ int32_t wsum[4], bnd[2];
    const int tid = threadIdx.x;
    const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t e0 = t * K - 1;  // entry of local index 0
    const int32_t row0 = trow[t], row1 = trow[t + 1];
    const int nrows = row1 - row0;  // rows owned (their first entry in [tK, tK + K))
    {   // stage entries [e0, e0 + WIN) with 16-B loads; entries outside [0, nnz) read as row ends
        constexpr int EPV = 16 / (int)sizeof(T);
        const int64_t bc = e0 < 0 ? 0 : (e0 & ~(int64_t)3), bv = e0 < 0 ? 0 : (e0 & ~(int64_t)(EPV - 1));
        const int64_t ce = e0 + WIN;  // one past the last staged entry
        constexpr int SPTC = ((WIN + 4) / 4 + 255) / 256, SPTV = ((WIN + EPV) / EPV + 255) / 256;
        const __amdgpu_buffer_rsrc_t cr = lz_rsrc(colf + bc, 0x7fffffffu);
        const __amdgpu_buffer_rsrc_t vr = lz_rsrc(val + bv, 0x7fffffffu);
        constexpr int AUX = 2;  // nt: streamed once
        int4 ct[SPTC];
        int4 vt[SPTV];
#pragma unroll
        for (int q = 0; q < SPTC; ++q) {
            const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
            ct[q] = int4{0, 0, 0, 0};
            if (k + 4 <= nnz && k < ce)
                ct[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(cr, (uint32_t)((k - bc) * 4), 0, AUX));
            else if (k < ce && k < nnz) {
                ct[q].x = colf[k];
                if (k + 1 < nnz) ct[q].y = colf[k + 1];
                if (k + 2 < nnz) ct[q].z = colf[k + 2];
            }
        }
#pragma unroll
        for (int q = 0; q < SPTV; ++q) {
            const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
            vt[q] = int4{0, 0, 0, 0};
            if (k + EPV <= nnz && k < ce) {
                vt[q] = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(vr, (uint32_t)((k - bv) * sizeof(T)), 0, AUX));
            } else if (k < ce && k < nnz) {
                T tv[EPV] = {};
                for (int e = 0; e < EPV && k + e < nnz; ++e) tv[e] = val[k + e];
                __builtin_memcpy(&vt[q], tv, 16);
            }
        }
        // entries before 0 or past nnz: a row end (flag) with a zero value
        for (int i = tid; i < WIN + UNR; i += 256) {
            const int64_t e = e0 + i;
            if (e < 0 || e >= nnz || i >= WIN) {
                cs[i] = (int32_t)0x80000000u;
                vs[i] = T(0);
            }
        }
#pragma unroll
        for (int q = 0; q < SPTC; ++q) {
            const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
            const int32_t cv[4] = {ct[q].x, ct[q].y, ct[q].z, ct[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (k + e >= e0 && k + e < ce && k + e >= 0 && k + e < nnz) cs[k + e - e0] = cv[e];
        }
#pragma unroll
        for (int q = 0; q < SPTV; ++q) {
            const int64_t k = bv + EPV * (int64_t)(tid + 256 * q);
            T tv[EPV];
            __builtin_memcpy(tv, &vt[q], 16);
#pragma unroll
            for (int e = 0; e < EPV; ++e)
                if (k + e >= e0 && k + e < ce && k + e >= 0 && k + e < nnz) vs[k + e - e0] = tv[e];
        }
        __syncthreads();
    }
    // Block scan of the row-end flags.  E(i) = ends in local [0, i).  A row
    // starts at local i when local i - 1 ends one; the owned rows start in
    // [1, K], so an entry at local i lies in owned row E(i) - 1 when
    // 0 <= E(i) - 1 < nrows (entries of the row begun before tK count 0 ends,
    // entries past the last owned row count nrows + 1).
    int f[EPT], cnt = 0;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int i = tid * EPT + u;
        f[u] = i < WIN ? (int)((uint32_t)cs[i] >> 31) : 0;
        cnt += f[u];
    }
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if ((tid & 63) >= o) incl += y;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    if (tid == 0) {
        bnd[0] = WIN;
        bnd[1] = 0;
    }
    __syncthreads();
    int Ei = incl - cnt;
    for (int w = 0; w < (tid >> 6); ++w) Ei += wsum[w];
    int lo = WIN, hi = 0;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
        const int i = tid * EPT + u;
        const int r = Ei - 1;
        if (i < WIN && r >= 0 && r < nrows) {
            rid[i] = (uint8_t)r;
            if ((uint32_t)cs[i - 1] >> 31) rel[r] = i;  // i >= 1 here: local 0 is never owned
            if (f[u] && r == nrows - 1) rel[nrows] = i + 1;
            lo = i < lo ? i : lo;
            hi = i + 1 > hi ? i + 1 : hi;
        }
        Ei += f[u];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int a2 = __shfl_xor(lo, o, 64), b2 = __shfl_xor(hi, o, 64);
        lo = a2 < lo ? a2 : lo;
        hi = b2 > hi ? b2 : hi;
    }
    if ((tid & 63) == 0) {
        atomicMin(&bnd[0], lo);
        atomicMax(&bnd[1], hi);
    }
    __syncthreads();
    if (nrows <= 0) return;  // block-uniform: a long row from an earlier tile covers this one
    const int b0 = bnd[0], b1 = bnd[1], N = b1 - b0;
    const __amdgpu_buffer_rsrc_t xr = lz_rsrc(X, (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
    const int gi = tid / LPR, p = tid % LPR;
    const uint32_t rowb = (uint32_t)(ldx * sizeof(T)), lane_off = p * VEC * sizeof(T);
    Vec<T, VEC> zero;
#pragma unroll
    for (int i = 0; i < VEC; ++i) zero.v[i] = T(0);
    const int Es = ((N + G - 1) / G + UNR - 1) / UNR * UNR;  // slice length, UNR-aligned
    const int start = b0 + gi * Es, end = (start + Es < b1) ? start + Es : b1;
    if (start < end) {  // group-uniform
        int cur = rid[start];
        bool open = rel[cur] < start;  // cur began in an earlier group's slice
        Vec<T, VEC> acc = zero;
        for (int s0 = start; s0 < end; s0 += UNR) {
            int32_t cc[UNR];
            T vv[UNR];
            int rr[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                cc[u] = cs[s0 + u] & 0x7fffffff;
                vv[u] = vs[s0 + u];
                rr[u] = rid[s0 + u];
            }
            Vec<T, VEC> xs[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const uint32_t off = s0 + u < end ? __umul24((unsigned)cc[u], rowb) + lane_off : 0x80000000u;
                xs[u] = ldbuf<T, VEC>(xr, off);
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int r = s0 + u < end ? rr[u] : cur;
                if (r != cur) {  // row cur ends inside the slice
                    if (open) head[gi][p] = acc;
                    else yt[cur][p] = acc;
                    acc = zero;
                    cur = r;
                    open = false;
                }
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc.v[i] = fma(vv[u], xs[u].v[i], acc.v[i]);
            }
        }
        if (open) head[gi][p] = acc;
        else yt[cur][p] = acc;
    }
    __syncthreads();
    // rows over several slices: first piece (in yt) + the later groups' heads, in group order
    for (int r = gi; r < nrows; r += G) {
        const int a = rel[r] - b0, e = rel[r + 1] - b0;
        const int g1 = a / Es, g2 = (e - 1) / Es;
        if (g1 == g2) continue;
        Vec<T, VEC> sum = yt[r][p];
        for (int g = g1 + 1; g <= g2; ++g) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) sum.v[i] += head[g][p].v[i];
        }
        yt[r][p] = sum;
    }
    __syncthreads();
    for (int idx = tid; idx < nrows * LPR; idx += 256) {
        T *dst = Y + ((int64_t)row0 + idx / LPR) * ldy + (idx % LPR) * VEC;
        Vec<T, VEC> y = yt[idx / LPR][idx % LPR];
        if constexpr (sizeof(T) * VEC == 16) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4 uu;
            __builtin_memcpy(&uu, &y, 16);
            __builtin_nontemporal_store(uu, reinterpret_cast<u32x4 *>(dst));
        } else {
            stv<T, VEC>(dst, y);
        }
    }
}

// Build (or reuse) the fixed-nnz format of an operator (cached on the handle
// by its pointers and sizes; experiment: a caller changing the arrays in
// place behind the same pointers would see stale flags).  false: the operator
// has a shape the kernel does not cover (empty rows, rows past S + 1 entries,
// more than RMAX rows in a tile).
static int fnz_prepare(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, bool *ok)
{
    *ok = false;
    const int64_t ntiles = ceil_div(nnz, (int64_t)kFnzK);
    if (nnz <= 0 || n >= (1LL << 31) || ntiles + 1 >= (1LL << 31)) return LZ_OK;
    if (h->fnz_key[0] == (int64_t)(uintptr_t)rp && h->fnz_key[1] == (int64_t)(uintptr_t)col && h->fnz_key[2] == n &&
        h->fnz_key[3] == nnz) {
        *ok = h->fnz_ok;
        return LZ_OK;
    }
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    (void)hipFree(h->fnz_colf);
    (void)hipFree(h->fnz_trow);
    h->fnz_colf = nullptr;
    h->fnz_trow = nullptr;
    h->fnz_key[0] = 0;
    LZ_HIP_TRY(hipMalloc(&h->fnz_colf, sizeof(int32_t) * (size_t)nnz));
    LZ_HIP_TRY(hipMalloc(&h->fnz_trow, sizeof(int32_t) * (size_t)(ntiles + 1)));
    int *stats = h->err_flag + 12;  // [0] max row length, [1] empty / negative, [2] max rows per tile
    LZ_HIP_TRY(hipMemsetAsync(stats, 0, 3 * sizeof(int), h->stream));
    const int g1 = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)256), (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_fnz_flags, dim3(g1), dim3(256), 0, h->stream, n, rp, col, h->fnz_colf, stats);
    const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ntiles + 1, (int64_t)256), (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_fnz_trow, dim3(g2), dim3(256), 0, h->stream, ntiles, n, rp, kFnzK, h->fnz_trow, stats);
    LZ_LAUNCH_CHECK();
    int st[3] = {0, 0, 0};
    LZ_HIP_TRY(hipMemcpyAsync(st, stats, sizeof(st), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    h->fnz_ok = st[1] == 0 && st[0] <= kFnzS + 1 && st[2] <= kFnzRmax;
    h->fnz_key[0] = (int64_t)(uintptr_t)rp;
    h->fnz_key[1] = (int64_t)(uintptr_t)col;
    h->fnz_key[2] = n;
    h->fnz_key[3] = nnz;
    *ok = h->fnz_ok;
    return LZ_OK;
}

template <typename T, int B>
static int launch_fnz(lz_handle *h, int64_t nnz, const T *val, const T *X, int64_t ldx, int64_t nx, T *Y,
                      int64_t ldy)
{
    const int64_t ntiles = ceil_div(nnz, (int64_t)kFnzK);
    hipLaunchKernelGGL((k_spmm_fnz<T, B, kFnzK, kFnzS, kFnzRmax>), dim3((unsigned)ntiles), dim3(256), 0, h->stream, nnz,
                       h->fnz_colf, val, h->fnz_trow, X, ldx, nx, Y, ldy);
    return LZ_OK;
}

// the long-tile queue for st tiles: count slots longq[0..1], then the list
static int ensure_longq(lz_handle *h, int64_t st)
{
    if ((size_t)st + 2 > h->longq_cap) {
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        (void)hipFree(h->longq);
        h->longq = nullptr;
        LZ_HIP_TRY(hipMalloc(&h->longq, sizeof(int) * ((size_t)st + 2)));
        // both count slots, on the handle's stream: a plain hipMemset runs on the
        // null stream, which does not order against a non-blocking stream (a
        // torch pool stream, a virtual rank's), so the kernels below could read
        // the fresh allocation's garbage as a queue count (round 5: wrong tiles
        // recomputed by the long-tile pass, or an illegal address)
        LZ_HIP_TRY(hipMemsetAsync(h->longq, 0, 2 * sizeof(int), h->stream));
        h->longq_cap = (size_t)st + 2;
        h->longq_parity = 0;
    }
    return LZ_OK;
}

#ifdef LZ_DIAG  // (measured and dropped in round 6: the diagnostic build only)
// LZ_SPMM_PF = "k[,C[,D[,span]]]" (read per call): the CU-partitioned SpMM with k
// of every 8 CUs of each XCD prefetching (0: off), chunks of C tiles (0: no
// prefetch kernel, the tile kernel alone on its CUs), at most D tiles ahead of
// the XCD's dispatch front, X rows only for a band under `span` rows.  LZ_SPMM_PF_MAP selects which mask bits are an XCD's
// CUs (0: bit i is CU i / 8 of XCC i % 8).
static bool pf_config(int *k, int *C, int *D, int *span)
{
    const char *e = getenv("LZ_SPMM_PF");
    if (!e || !*e) return false;
    int v[4] = {0, *C, *D, *span};
    const int got = sscanf(e, "%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3]);
    if (got < 1 || v[0] < 0 || v[0] > 7 || v[1] < 0 || v[2] < 0 || v[3] < 1) return false;
    *k = v[0];
    *C = v[1];
    *D = v[2];
    *span = v[3];
    return true;
}

static int pf_setup(lz_handle *h, int k)
{
    const char *mp = getenv("LZ_SPMM_PF_MAP");
    const int map = mp ? atoi(mp) : 0;
    const int key = k * 16 + map;
    if (h->pf_key == key) return LZ_OK;
    for (hipStream_t *s : {&h->pf_sg, &h->pf_sp})
        if (*s) {
            LZ_HIP_TRY(hipStreamSynchronize(*s));
            LZ_HIP_TRY(hipStreamDestroy(*s));
            *s = nullptr;
        }
    uint32_t mg[8] = {}, mpf[8] = {};
    for (int i = 0; i < 256; ++i) {
        // bit i -> XCC i % 8, local CU j = i / 8, which sits in shader engine
        // j % 4 (scripts/gprobe/cumask_probe.hip, profiles/r06a_cumask_probe.log).
        // The dispatcher deals workgroups evenly over the shader engines, so
        // the prefetch CUs are taken evenly from each engine (map 0: slot
        // j / 4 < k, k of each engine's 8); map 1 takes them from the low
        // engines (j % 8 < k: an engine left with 4 of its 8 CUs at k = 2 --
        // the tile kernel alone took 2.16 ms instead of 1.30 there,
        // profiles/r06j_spmm_masked_stream_ab.log)
        const int j = i / 8;
        const bool pf = map == 0 ? (j / 4) < k : (j % 8) < k;
        (pf ? mpf : mg)[i / 32] |= 1u << (i % 32);
    }
    LZ_HIP_TRY(hipExtStreamCreateWithCUMask(&h->pf_sg, 8, mg));
    if (k > 0) LZ_HIP_TRY(hipExtStreamCreateWithCUMask(&h->pf_sp, 8, mpf));  // (k = 0: every CU on the tile stream)
    for (hipEvent_t *e : {&h->ev_pff, &h->ev_pfg, &h->ev_pfp})
        if (!*e) LZ_HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    if (!h->pf_ctl) LZ_HIP_TRY(hipMalloc(&h->pf_ctl, sizeof(int) * (kPfCtl + 256)));
    h->pf_key = key;
    return LZ_OK;
}

template <typename T, int B, int TR, int CAP>
static int launch_seg_pf(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, const T *X,
                         int64_t ldx, int64_t nx, T *Y, int64_t ldy, int k, int C, int D, int span)
{
    const int64_t st = ceil_div(n, (int64_t)TR);
    LZ_TRY(pf_setup(h, k));
    // the operator's band, once per operator (keyed by its arrays and sizes)
    if (C > 0 && k > 0 && !(h->pf_band_key[0] == (int64_t)(uintptr_t)rp && h->pf_band_key[1] == (int64_t)(uintptr_t)col &&
                   h->pf_band_key[2] == n)) {
        int *band = h->pf_ctl + kPfCtl;
        LZ_HIP_TRY(hipMemsetAsync(band, 0, sizeof(int), h->stream));
        hipLaunchKernelGGL(k_band, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), 2048))),
                           dim3(256), 0, h->stream, n, rp, col, band);
        LZ_HIP_TRY(hipMemcpyAsync(&h->pf_band, band, sizeof(int), hipMemcpyDeviceToHost, h->stream));
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        h->pf_band_key[0] = (int64_t)(uintptr_t)rp;
        h->pf_band_key[1] = (int64_t)(uintptr_t)col;
        h->pf_band_key[2] = n;
    }
    const int parity = h->longq_parity;
    h->longq_parity ^= 1;
    hipLaunchKernelGGL(k_pf_init, dim3(1), dim3(kPfCtl), 0, h->stream, h->pf_ctl);
    LZ_HIP_TRY(hipEventRecord(h->ev_pff, h->stream));
    LZ_HIP_TRY(hipStreamWaitEvent(h->pf_sg, h->ev_pff, 0));
    if (k > 0) LZ_HIP_TRY(hipStreamWaitEvent(h->pf_sp, h->ev_pff, 0));
    // the tile kernel first (the two masked streams have queues of their own:
    // profiles/r06h_pf_trace.csv shows both kernels running at once)
    hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, false, 0, false, false, true>), dim3((unsigned)st), dim3(256), 0,
                       h->pf_sg, n, rp, col, val, X, ldx, nx, Y, ldy, h->longq, parity, nullptr, nullptr, 0, h->pf_ctl);
    // C = 0: the tile kernel alone on its CUs (the masked launch's own cost);
    // 8 blocks per prefetching CU (4 k CUs per XCD); a band wider than `span`
    // rows gets no X prefetch
    if (C > 0 && k > 0)
        hipLaunchKernelGGL((k_spmm_pf<TR>), dim3(8 * 4 * k * 8), dim3(256), 0, h->pf_sp, n, st, rp, col,
                           reinterpret_cast<const char *>(val), (int)sizeof(T), reinterpret_cast<const char *>(X),
                           h->pf_band < span ? nx : (int64_t)0, (int)(ldx * sizeof(T)), h->pf_ctl, C, D,
                           (int64_t)h->pf_band);
    const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>(st, (int64_t)h->n_cu * 4));
    hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, false, 1>), dim3(g2), dim3(256), 0, h->pf_sg, n, rp, col, val, X, ldx,
                       nx, Y, ldy, h->longq, parity, nullptr, nullptr, 0, nullptr);
    LZ_HIP_TRY(hipEventRecord(h->ev_pfg, h->pf_sg));
    LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_pfg, 0));
    if (k > 0) {
        LZ_HIP_TRY(hipEventRecord(h->ev_pfp, h->pf_sp));
        LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_pfp, 0));
    }
    return LZ_OK;
}

#endif  // LZ_DIAG

// nnz-split SpMM with the long-tile queue: the main kernel, then a persistent
// kernel over the queued tiles (an empty queue costs one short launch).
// plan_slot >= 0: the long tiles an earlier call on the same operator queued
// (count slot plan_slot, *slot_out of that call, or a list spmm_b2_plan made
// up front) -- the long-tile pass runs
// first, on its own stream, beside the main kernel, which then only skips them.
template <typename T, int B, int TR, int CAP, bool WIN, bool YCM = false, bool EPI = false>
static int launch_seg(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, const T *X,
                      int64_t ldx, int64_t nx, T *Y, int64_t ldy, const T *Wp = nullptr, const T *Mm = nullptr,
                      int plan_slot = -1, int *slot_out = nullptr)
{
    const int64_t st = ceil_div(n, (int64_t)TR);
    LZ_ARG_CHECK(st < (1LL << 31), "too many row tiles");
    LZ_TRY(ensure_longq(h, st));
    if (plan_slot >= 0) {
        LZ_ARG_CHECK(plan_slot <= 1 && (size_t)st + 2 <= h->longq_cap, "planned SpMM: no earlier queue");
        if (!h->lstream) {
            LZ_HIP_TRY(hipStreamCreateWithFlags(&h->lstream, hipStreamNonBlocking));
            LZ_HIP_TRY(hipEventCreateWithFlags(&h->ev_lfork, hipEventDisableTiming));
            LZ_HIP_TRY(hipEventCreateWithFlags(&h->ev_ljoin, hipEventDisableTiming));
        }
        const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>(st, (int64_t)h->n_cu * 4));
        LZ_HIP_TRY(hipEventRecord(h->ev_lfork, h->stream));
        LZ_HIP_TRY(hipStreamWaitEvent(h->lstream, h->ev_lfork, 0));
        hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, WIN, 1, YCM, EPI>), dim3(g2), dim3(256), 0, h->lstream, n, rp,
                           col, val, X, ldx, nx, Y, ldy, h->longq, 2 + plan_slot, Wp, Mm, 0, nullptr);
        LZ_HIP_TRY(hipEventRecord(h->ev_ljoin, h->lstream));
        hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, WIN, 0, YCM, EPI>), dim3((unsigned)st), dim3(256), 0, h->stream,
                           n, rp, col, val, X, ldx, nx, Y, ldy, h->longq, 2 + plan_slot, Wp, Mm, 0, nullptr);
        LZ_HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_ljoin, 0));
        return LZ_OK;
    }
#ifdef LZ_DIAG
    if constexpr (!WIN && !YCM && !EPI) {
        int k = 0, C = 8, D = 96, span = 65536;
        if (pf_config(&k, &C, &D, &span) && (k > 0 || C == 0))
            return launch_seg_pf<T, B, TR, CAP>(h, n, rp, col, val, X, ldx, nx, Y, ldy, k, C, D, span);
    }
#endif
    const int parity = h->longq_parity;
    h->longq_parity ^= 1;
    if (slot_out) *slot_out = parity;
    // diag: measurement only (results wrong), in a -DLZ_DIAG build alone:
    // LZ_SPMM_DIAG = tiles mod this (every input L2-resident, DESIGN.md 4
    // SpMM); LZ_SPMM_DIAG_Y=1: the Y tiles stay the blocks' own.  The shipped
    // library always passes 0.
#ifdef LZ_DIAG
    const char *dg = getenv("LZ_SPMM_DIAG");
    const char *dy = getenv("LZ_SPMM_DIAG_Y");
    int diag = (dg ? atoi(dg) : 0) | (dy && dy[0] == '1' ? 1 << 30 : 0);
    // LZ_SPMM_HOT = "K,a": gathers of columns < K with the default cache policy,
    // the others with a = 1: nt, 2: sc1, 3: sc1 nt (the Infinity-Cache residency
    // probe, scripts/hot_probe.py; K < 2^24)
    if (const char *hs = getenv("LZ_SPMM_HOT")) {
        int hk = 0, ha = 1;
        if (sscanf(hs, "%d,%d", &hk, &ha) >= 1 && hk >= 0 && hk < (1 << 24) && ha >= 1 && ha <= 3)
            diag = -(hk | (ha << 24));
    }
#else
    constexpr int diag = 0;
#endif
    hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, WIN, 0, YCM, EPI>), dim3((unsigned)st), dim3(256), 0, h->stream, n, rp,
                       col, val, X, ldx, nx, Y, ldy, h->longq, parity, Wp, Mm, diag, nullptr);
    const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>(st, (int64_t)h->n_cu * 4));
    hipLaunchKernelGGL((k_spmm_seg<T, B, TR, CAP, WIN, 1, YCM, EPI>), dim3(g2), dim3(256), 0, h->stream, n, rp, col, val,
                       X, ldx, nx, Y, ldy, h->longq, parity, Wp, Mm, 0, nullptr);
    return LZ_OK;
}

// Kernel choice.  128-B rows (b = 16 fp64, b = 32 fp32): the nnz-split
// k_spmm_seg, 48-row tiles with a 768-entry stage (<= 13 nnz/row on average:
// C3) or 1536 entries (C4: 25 nnz/row), windowed past 2^24 rows / 2 GiB of X.
// Other shapes: the row-per-group k_spmm_buf, or the 64-bit k_spmm_lds past
// 2 GiB / 2^24 rows.
// ycm (128-B rows only): Y column-major with leading dimension ldy.
template <typename T, int B>
static int launch_spmm_rm(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col,
                          const T *val, const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy, bool ycm = false)
{
    using S = SpmmShape<T, B>;
    if (n <= 0) return LZ_OK;
    // X has nx rows (the operator's columns), not n
    const bool buf_ok = nx * ldx * (int64_t)sizeof(T) < (1LL << 31) && nx < (1 << 24);
    const int ev = prof_begin(h, PROF_SPMM);
    int rc = LZ_OK;
    if constexpr (S::LPR == 8) {
        const bool wide = (double)nnz > 13.0 * (double)n;
        const char *fz = getenv("LZ_SPMM_FNZ");  // experiment: fixed-nnz tiles (read per call)
        bool fnz = false;
        if (fz && fz[0] == '1' && !ycm && buf_ok && ldx == B && ldy == B)
            LZ_TRY(fnz_prepare(h, n, nnz, rp, col, &fnz));
        if (fnz) {
            rc = launch_fnz<T, B>(h, nnz, val, X, ldx, nx, Y, ldy);
        } else if (ycm) {
            if (buf_ok && !wide) rc = launch_seg<T, B, 48, 768, false, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
            else if (buf_ok) rc = launch_seg<T, B, 48, 1536, false, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
            else if (!wide) rc = launch_seg<T, B, 48, 768, true, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
            else rc = launch_seg<T, B, 48, 1536, true, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
        } else if (buf_ok && !wide) rc = launch_seg<T, B, 48, 768, false>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (buf_ok) rc = launch_seg<T, B, 48, 1536, false>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (!wide) rc = launch_seg<T, B, 48, 768, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
        else rc = launch_seg<T, B, 48, 1536, true>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    } else {
        const int64_t tiles = ceil_div(n, (int64_t)S::RB * 2);
        LZ_ARG_CHECK(tiles < (1LL << 31), "too many row tiles");
        constexpr int CAP = S::RB * 32 < 1024 ? 1024 : (S::RB * 32 > 4096 ? 4096 : S::RB * 32);
        constexpr int CAP2 = CAP * 2 < 4096 ? CAP * 2 : 4096;
        if (ycm && buf_ok)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 8, true>), dim3((unsigned)tiles), dim3(256), 0, h->stream, n,
                               rp, col, val, X, ldx, nx, Y, ldy);
        else if (ycm)
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP2, 2, true>), dim3((unsigned)tiles), dim3(256), 0, h->stream, n,
                               rp, col, val, X, ldx, nx, Y, ldy);
        else if (buf_ok)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2>), dim3((unsigned)tiles), dim3(256), 0, h->stream, n, rp,
                               col, val, X, ldx, nx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP2, 2>), dim3((unsigned)tiles), dim3(256), 0, h->stream, n, rp,
                               col, val, X, ldx, nx, Y, ldy);
    }
    prof_end(h, ev);
    LZ_TRY(rc);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// C5 beta^2 step: U = A X - Wp M at b = 32 fp32, row-major, X < 2 GiB, <= 13
// nnz per row (the shapes k_spmm_seg<..., 768, false> covers); returns
// LZ_E_ARG otherwise so the caller keeps the separate pass E.
bool spmm_b2_ok(int64_t n, int64_t nnz, int64_t nx)
{
    return nx * 32 * (int64_t)sizeof(float) < (1LL << 31) && nx < (1 << 24) && (double)nnz <= 13.0 * (double)n;
}

// 48-row tiles whose CSR run exceeds `cap` entries (one thread a tile)
__global__ __launch_bounds__(256) void k_tile_overflow(int64_t n, const int64_t *__restrict__ rp, int cap,
                                                       int *__restrict__ count)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, r0 = t * 48;
    const bool over = r0 < n && rp[r0 + 48 < n ? r0 + 48 : n] - rp[r0] > cap;
    const uint64_t b = __ballot(over);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, __popcll(b));
}

int spmm_b2_stage(lz_handle *h, int64_t n, const int64_t *rp, int *cap)
{
    // The stage of the beta^2 SpMM, once per solve: 1024 entries where more
    // than 1 % of the 48-row tiles hold over 1024 (a heavy tail of long rows,
    // C5's power-law operator: 3.0 %; fewer tiles then go to the long-tile
    // pass, at 6 blocks per CU instead of 7: SpMM 2.888-2.893 -> 2.821-2.824
    // ms), 768 otherwise (1024 costs 7-8 % on banded and uniform-random
    // operators, whose tiles stay under 1024: 0 %, even where 3 % exceed
    // 768).  profiles/r05zz6_c5_tile_shape_ab.log, r05zzf_b2_stage_ab.log
    *cap = 768;
    if (n <= 0) return LZ_OK;
    const int64_t tiles = ceil_div(n, (int64_t)48);
    // a named slot of the handle's flag block ([0] the device error word, [8], [9]
    // and [12..15] the plans' words), not a word of the scratch the solve's b x b
    // matrices use
    int *dcount = h->err_flag + 4;
    LZ_HIP_TRY(hipMemsetAsync(dcount, 0, sizeof(int), h->stream));
    hipLaunchKernelGGL(k_tile_overflow, dim3((unsigned)ceil_div(tiles, (int64_t)256)), dim3(256), 0, h->stream, n, rp,
                       1024, dcount);
    LZ_LAUNCH_CHECK();
    int over = 0;
    LZ_HIP_TRY(hipMemcpyAsync(&over, dcount, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    if ((double)over > 0.01 * (double)tiles) *cap = 1024;
    return LZ_OK;
}

// the long-tile list of the solve, before its first SpMM: every 48-row tile
// whose run exceeds cap, so that the first step's long-tile pass can also run
// beside its tile pass (the tile pass in planned mode only skips them; the
// list order does not matter: each listed tile is computed by one block, in
// chunk order)
__global__ __launch_bounds__(256) void k_tile_list(int64_t n, const int64_t *__restrict__ rp, int cap,
                                                   int *__restrict__ count, int *__restrict__ list)
{
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, r0 = t * 48;
    if (r0 < n && rp[r0 + 48 < n ? r0 + 48 : n] - rp[r0] > cap) list[atomicAdd(count, 1)] = (int)t;
}

int spmm_b2_plan(lz_handle *h, int64_t n, const int64_t *rp, int cap, int *slot)
{
    const int64_t st = ceil_div(n, (int64_t)48);
    LZ_ARG_CHECK(st < (1LL << 31), "too many row tiles");
    LZ_TRY(ensure_longq(h, st));
    *slot = h->longq_parity;
    h->longq_parity ^= 1;
    // both counts zeroed: this list's, and the next unplanned call's (which
    // expects its slot at zero, as an unplanned call leaves the other one)
    LZ_HIP_TRY(hipMemsetAsync(h->longq, 0, 2 * sizeof(int), h->stream));
    if (n <= 0) return LZ_OK;
    hipLaunchKernelGGL(k_tile_list, dim3((unsigned)ceil_div(st, (int64_t)256)), dim3(256), 0, h->stream, n, rp, cap,
                       h->longq + *slot, h->longq + 2);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

int spmm_rm_b2(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const float *val,
               const float *X, int64_t nx, float *Y, const float *Wp, const float *Mm, int plan_slot, int *slot_out,
               int cap)
{
    LZ_ARG_CHECK(spmm_b2_ok(n, nnz, nx), "beta^2 SpMM epilogue: shape not covered");
    LZ_ARG_CHECK(cap == 768 || cap == 1024, "beta^2 SpMM stage: 768 or 1024 (spmm_b2_stage)");
    if (n <= 0) return LZ_OK;
    const int ev = prof_begin(h, PROF_SPMM);
    const int rc = cap == 1024 ? launch_seg<float, 32, 48, 1024, false, false, true>(h, n, rp, col, val, X, 32, nx, Y,
                                                                                   32, Wp, Mm, plan_slot, slot_out)
                               : launch_seg<float, 32, 48, 768, false, false, true>(h, n, rp, col, val, X, 32, nx, Y, 32,
                                                                                  Wp, Mm, plan_slot, slot_out);
    prof_end(h, ev);
    LZ_TRY(rc);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

template <typename T>
int spmm_rm(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy, bool ycm)
{
    LZ_ARG_CHECK(!(ycm && b == 1), "column-major Y store: b >= 2");
    switch (b) {
    case 1:
        LZ_ARG_CHECK(ldx == 1 && ldy == 1, "b = 1 row-major needs ldx = ldy = 1");
        return spmv<T>(h, n, rp, col, val, X, Y, nnz);
    case 2: return launch_spmm_rm<T, 2>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    case 4: return launch_spmm_rm<T, 4>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    case 8: return launch_spmm_rm<T, 8>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    case 16: return launch_spmm_rm<T, 16>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    case 32: return launch_spmm_rm<T, 32>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    case 64: return launch_spmm_rm<T, 64>(h, n, nnz, rp, col, val, X, ldx, nx, Y, ldy, ycm);
    default: {  // any other b <= 64: one thread per (row, column), CSR order (block widths off the tuned set)
        LZ_ARG_CHECK(b >= 1 && b <= 64, "row-major SpMM: 1 <= b <= 64");
        LZ_ARG_CHECK(!ycm, "column-major Y store: b a power of two");
        const int64_t nb = n * b;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nb, (int64_t)256), (int64_t)h->n_cu * 16));
        const int ev = prof_begin(h, PROF_SPMM);
        hipLaunchKernelGGL((k_spmm_any_b<T>), dim3(grid), dim3(256), 0, h->stream, n, b, rp, col, val, X, ldx, Y, ldy);
        prof_end(h, ev);
        LZ_LAUNCH_CHECK();
        return LZ_OK;
    }
    }
}

// Column-major block (b columns, leading dimension ld) -> row-major (ld = b),
// kCmRows rows per workgroup through LDS: the column reads and the row writes
// are both coalesced.
constexpr int kCmRows = 128;

template <typename T>
__global__ __launch_bounds__(256) void k_cm_transpose(int64_t rows, int b, const T *__restrict__ src,
                                                      int64_t ld, T *__restrict__ dst)
{
    constexpr int EPV = 16 / (int)sizeof(T);
    extern __shared__ __align__(16) unsigned char cm_lds[];  // b * (kCmRows + 1) elements
    T *tile = reinterpret_cast<T *>(cm_lds);
    const int64_t r0 = (int64_t)blockIdx.x * kCmRows;
    const int nr = (int)(rows - r0 < kCmRows ? rows - r0 : kCmRows);
    // column pieces of EPV rows (16 B) where every column start is 16-B aligned
    if (((reinterpret_cast<uintptr_t>(src) & 15) == 0) && ld % EPV == 0 && nr == kCmRows) {
        constexpr int NQ = kCmRows / EPV;
        for (int i = threadIdx.x; i < NQ * b; i += blockDim.x) {
            const int c = i / NQ, r = (i - c * NQ) * EPV;
            const Vec<T, EPV> v = ldv<T, EPV>(src + (int64_t)c * ld + r0 + r);
#pragma unroll
            for (int e = 0; e < EPV; ++e) tile[c * (kCmRows + 1) + r + e] = v.v[e];
        }
    } else {
        for (int i = threadIdx.x; i < kCmRows * b; i += blockDim.x) {
            const int c = i / kCmRows, r = i % kCmRows;
            if (r < nr) tile[c * (kCmRows + 1) + r] = src[(int64_t)c * ld + r0 + r];
        }
    }
    __syncthreads();
    // row pieces of EPV columns (b is a power of two >= 2; dst rows are b * sizeof(T) bytes)
    if (b % EPV == 0) {
        const int nb = b / EPV;
        for (int i = threadIdx.x; i < nr * nb; i += blockDim.x) {
            const int r = i / nb, c = (i - r * nb) * EPV;
            Vec<T, EPV> v;
#pragma unroll
            for (int e = 0; e < EPV; ++e) v.v[e] = tile[(c + e) * (kCmRows + 1) + r];
            stv<T, EPV>(dst + (r0 + r) * b + c, v);
        }
    } else {
        for (int i = threadIdx.x; i < nr * b; i += blockDim.x) {
            const int r = i / b, c = i % b;
            dst[r0 * b + i] = tile[c * (kCmRows + 1) + r];
        }
    }
}

// column-major rows x b block (leading dimension ld >= rows) -> row-major (ld = b)
template <typename T>
int to_row_major(lz_handle *h, int64_t rows, int b, const T *src, int64_t ld, T *dst)
{
    LZ_ARG_CHECK(b >= 1 && b <= kMaxB && ld >= rows && rows >= 0, "to_row_major: 1 <= b <= 64, ld >= rows");
    if (rows == 0) return LZ_OK;
    const size_t lds = sizeof(T) * (size_t)b * (kCmRows + 1);
    hipLaunchKernelGGL((k_cm_transpose<T>), dim3((unsigned)ceil_div(rows, (int64_t)kCmRows)), dim3(256), lds,
                       h->stream, rows, b, src, ld, dst);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}
template int to_row_major<double>(lz_handle *, int64_t, int, const double *, int64_t, double *);
template int to_row_major<float>(lz_handle *, int64_t, int, const float *, int64_t, float *);

template <typename T>
int spmm_cm(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy)
{
    if (n <= 0) return LZ_OK;
    // b = 2..64 (powers of two): a column-major gather touches b lines per
    // nonzero, the row-major kernel one, so X is transposed in once (read +
    // write) and the row-major SpMM kernels store their finished Y tiles column
    // by column themselves (TR contiguous elements per column).  Yee N=160, b=16
    // fp32: 3.69 ms direct, 2.61 ms with a separate Y transpose pass.
    // LZ_SPMM_CM=direct: the one-pass kernel.
    const char *cm_env = getenv("LZ_SPMM_CM");  // read per call (tests switch it)
    if (b >= 2 && (b & (b - 1)) == 0 && !(cm_env && cm_env[0] == 'd')) {  // the row-major kernel's b
        const size_t need = sizeof(T) * (size_t)b * (size_t)nx;
        if (need > h->cm_cap) {
            LZ_HIP_TRY(hipStreamSynchronize(h->stream));
            (void)hipFree(h->cm_buf);
            h->cm_buf = nullptr;
            h->cm_cap = 0;
            LZ_HIP_TRY(hipMalloc(&h->cm_buf, need));
            h->cm_cap = need;
        }
        T *Xr = static_cast<T *>(h->cm_buf);
        const size_t lds = sizeof(T) * (size_t)b * (kCmRows + 1);
        hipLaunchKernelGGL((k_cm_transpose<T>), dim3((unsigned)ceil_div(nx, (int64_t)kCmRows)), dim3(256), lds,
                           h->stream, nx, b, X, ldx, Xr);
        LZ_LAUNCH_CHECK();
        return spmm_rm<T>(h, n, nnz, rp, col, val, b, Xr, b, nx, Y, ldy, true);
    }
    const int grid = (int)std::min<int64_t>(ceil_div(n, 256), (int64_t)h->n_cu * 8);
    if (grid <= 0) return LZ_OK;
    hipLaunchKernelGGL((k_spmm_cm<T>), dim3(grid), dim3(256), 0, h->stream, n, rp, col, val, b,
                       X, ldx, Y, ldy);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

template <typename T>
int spmv(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, const T *x,
         T *y, int64_t nnz_hint)
{
    // lanes per row from the mean row length (nnz_hint <= 0: read it back is
    // not allowed here -- use 8, right for ~6-16 nnz/row)
    const double mean = (nnz_hint > 0 && n > 0) ? (double)nnz_hint / (double)n : 10.0;
    int lv = mean <= 5 ? 4 : mean <= 12 ? 8 : mean <= 28 ? 16 : mean <= 60 ? 32 : 64;
    const int64_t units = ceil_div(n, 256 / lv);
    const int grid = (int)std::min<int64_t>(units, (int64_t)h->n_cu * 8);
    if (grid <= 0) return LZ_OK;
#define LZ_SPMV_CASE(LV)                                                                       \
    case LV:                                                                                   \
        hipLaunchKernelGGL((k_spmv<T, LV>), dim3(grid), dim3(256), 0, h->stream, n, rp, col,  \
                           val, x, y);                                                         \
        break;
    switch (lv) {
        LZ_SPMV_CASE(4)
        LZ_SPMV_CASE(8)
        LZ_SPMV_CASE(16)
        LZ_SPMV_CASE(32)
        LZ_SPMV_CASE(64)
    }
#undef LZ_SPMV_CASE
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

template int spmm_rm<double>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *,
                             const double *, int, const double *, int64_t, int64_t, double *, int64_t, bool);
template int spmm_rm<float>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, int64_t, float *, int64_t, bool);
template int spmm_cm<double>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *,
                             const double *, int, const double *, int64_t, int64_t, double *, int64_t);
template int spmm_cm<float>(lz_handle *, int64_t, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, int64_t, float *, int64_t);
template int spmv<double>(lz_handle *, int64_t, const int64_t *, const int32_t *, const double *,
                          const double *, double *, int64_t);
template int spmv<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                         const float *, float *, int64_t);

}  // namespace lz
