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

// Tile-per-block SpMM (fallback for X >= 2 GiB or n >= 2^24).  A block owns a tile of
// RB*RPG consecutive rows; group gi (LPR lanes) owns rows gi + RB*j, j < RPG.
// The block stages the tile's (col, val) range into LDS with coalesced loads
// (one HBM round trip per tile, amortised over RPG gather rounds), then every
// group gathers its rows' X rows 8 nnz at a time (8 independent 16-byte loads
// per lane in flight), reading (col, val) from LDS.  One tile per block with
// the XCD remap keeps each XCD's in-flight tiles contiguous (L2-resident X
// window).  Tiles with more than CAP nnz are staged in CAP-sized chunks.
template <typename T, int B, int CAP, int RPG>
__global__ __launch_bounds__(256) void k_spmm_lds(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx, int64_t /*nx*/,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, UNR = 8, TR = RB * RPG;
    __shared__ int32_t cs[CAP];
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

template <typename T, int B, int CAP, int RPG, int UNR = 8, int MINW = 1, int PF = 0>
__global__ __launch_bounds__(256, MINW) void k_spmm_buf(int64_t n, const int64_t *__restrict__ rp,
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
    uint32_t pfx = 0;
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
        // PF > 0: touch every X row of the chunk once (one dword, one lane per
        // nonzero) before the gather steps, so the rows' first-touch L2 misses
        // overlap in one round instead of stalling successive 8-load steps
        uint32_t pfv[PF > 0 ? PF : 1];
        if constexpr (PF > 0) {
#pragma unroll
            for (int q = 0; q < PF; ++q) {
                const int k = tid + 256 * q;
                const uint32_t off = (k < (int)(c1 - c0)) ? __umul24((unsigned)cs[k], rowb) : 0x80000000u;
                pfv[q] = __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0);
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
        if constexpr (PF > 0) {
#pragma unroll
            for (int q = 0; q < PF; ++q) pfx ^= pfv[q];
        }
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
    if constexpr (PF > 0) {  // keeps the touches alive; ldy < 0 never happens
        if (ldy < 0 && pfx == 0x9e3779b9u) Y[0] = T(0);
    }
}

// Wave-specialised persistent SpMM (b = 16 fp64).  A wave that mixes HBM
// streaming loads with L2-resident gathers waits HBM latency at every gather
// step (vmcnt is in order: a load's data waits for every older load).  Measured
// (scripts/probe/gather_probe.hip): 8 gathers + 2 stream loads per step in the
// same waves took 2.5x longer than the same work split over gather-only and
// stream-only waves.  So each block has one LOADER wave that streams the CSR
// runs of the block's tiles into a ring of WS_K LDS stages with LDS-DMA
// (buffer_load_dwordx4 ... lds: no VGPRs, bounds-checked per chunk), and
// WS_NC CONSUMER waves that only gather X (L2) and store Y.  Hand-off through
// LDS words: ready[s] = tile sequence number once its DMA has landed (the
// loader waits vmcnt with a fixed number of DMA instructions per tile, so the
// count is a compile-time immediate); done[s] counts consumer waves finished
// with the stage.  Every spin is bounded (kWsSpin) so a logic error cannot
// hang the GPU.  Persistent grid, XCD-aware strided tile order (as
// k_fused_pw16 had) so an XCD's tiles in flight stay adjacent.
// WS_NC consumer waves (16 rows each), WS_K LDS stages, loader pipeline depth
// WS_D (tiles whose DMA is in flight), WS_CAP staged nonzeros per tile.
template <int WS_NC, int WS_K, int WS_D, int WS_CAP>
struct WsCfg {
    static constexpr int TR = 16 * WS_NC;
    static constexpr int RP_PIECES = (TR + 2) * 8 / 16;  // 16-B pieces of row_ptr
    static constexpr int COL_PIECES = (WS_CAP + 8) * 4 / 16;
    static constexpr int VAL_PIECES = (WS_CAP + 4) * 8 / 16;
    static constexpr int DMA_INSTR = ws_instr(RP_PIECES) + ws_instr(COL_PIECES) + ws_instr(VAL_PIECES);
    static_assert(DMA_INSTR * (WS_D - 1) <= 63, "vmcnt immediate");
    static_assert(WS_D <= WS_K, "pipeline depth");
    // one DMA wave-instruction lands 1 KiB (64 lanes x 16 B, out-of-range
    // lanes included), so every region is a whole number of KiB
    struct Stage {
        int64_t rp[ws_instr(RP_PIECES) * 128];
        int32_t col[ws_instr(COL_PIECES) * 256];
        double val[ws_instr(VAL_PIECES) * 128];
    };
};

template <int WS_NC, int WS_K, int WS_D, int WS_CAP>
__global__ __launch_bounds__(64 * (WS_NC + 1)) void k_spmm_ws(int64_t n, const int64_t *__restrict__ rp,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ X, int64_t nx,
                                                           double *__restrict__ Y, int *__restrict__ err)
{
    using C = WsCfg<WS_NC, WS_K, WS_D, WS_CAP>;
    constexpr int WS_TR = C::TR;
    __shared__ typename C::Stage st[WS_K];
    __shared__ int ready[WS_K], done[WS_K];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < WS_K) {
        ready[threadIdx.x] = -1;
        done[threadIdx.x] = 0;
    }
    __syncthreads();  // the only block barrier
    // this block's tile sequence (XCD-aware, strided)
    const int64_t T = ceil_div(n, (int64_t)WS_TR);
    int64_t begin, end, k, K;
    {
        const int64_t G = gridDim.x, b = blockIdx.x;
        if (G < 8) {
            begin = 0; end = T; k = b; K = G;
        } else {
            const int64_t x = b & 7;
            begin = T * x / 8;
            end = T * (x + 1) / 8;
            k = b >> 3;
            K = (G - x + 7) >> 3;
        }
    }
    const int64_t nt = (end - begin - k + K - 1) / K > 0 ? (end - begin - k + K - 1) / K : 0;
    const int64_t nnz = rp[n];
    // LDS hand-off words: workgroup-scope relaxed atomics (ds_read / ds_write,
    // never flat: flat ops would break the loader's counted vmcnt wait)
    auto ld = [](int *a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    if (w == 0) {
        // ------------------------------------------------------------ loader
        auto tile_r0 = [&](int64_t i) { return (begin + k + i * K) * WS_TR; };
#ifdef LZ_WS_PROBE
        long long c_done = 0, c_vm = 0;
        const long long c_start = clock64();
#endif
        int64_t kA_next = nt > 0 ? rp[tile_r0(0)] : 0;  // row_ptr of the next tile, one ahead
        for (int64_t i = 0; i < nt; ++i) {
            const int s = (int)(i % WS_K);
            const int64_t r0 = tile_r0(i), r1 = (r0 + WS_TR < n) ? r0 + WS_TR : n;
            const int64_t kA = kA_next;
            if (i + 1 < nt) kA_next = rp[tile_r0(i + 1)];
            if (i >= WS_K) {  // wait until every consumer is done with tile i - K
                long spin = 0;
                WS_T(t0);
                const uint32_t da = ws_lds_addr(&done[s]);
                while (ws_lds_read(da) < WS_NC * (int)(i / WS_K) && ++spin < kWsSpin) __builtin_amdgcn_s_sleep(1);
                if (spin >= kWsSpin) { *err = 1; break; }
#ifdef LZ_WS_PROBE
                c_done += clock64() - t0;
#endif
            }
            const int64_t ca = kA & ~(int64_t)3, va = kA & ~(int64_t)1;
            const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int64_t *>(rp + r0), (short)0,
                                                              (int)((r1 - r0 + 1) * 8), 0x00020000);
            const int64_t cb = (nnz - ca) * 4, vb = (nnz - va) * 8;
            const auto cr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t *>(col + ca), (short)0,
                                                              (int)(cb < 0x7fffffff ? cb : 0x7fffffff), 0x00020000);
            const auto vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(val + va), (short)0,
                                                              (int)(vb < 0x7fffffff ? vb : 0x7fffffff), 0x00020000);
            ws_dma(rr, st[s].rp, C::RP_PIECES, lane);
            ws_dma(cr, st[s].col, C::COL_PIECES, lane);
            ws_dma(vr, st[s].val, C::VAL_PIECES, lane);
            if (i >= WS_D - 1) {  // tile i-D+1 has landed once only D-1 tiles' DMA are younger
                WS_T(t1);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::DMA_INSTR * (WS_D - 1)) : "memory");
#ifdef LZ_WS_PROBE
                c_vm += clock64() - t1;
#endif
                const int64_t pub = i - (WS_D - 1);
                if (lane == 0) ws_lds_write(ws_lds_addr(&ready[(int)(pub % WS_K)]), (int)pub);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int64_t pub = nt - (WS_D - 1) > 0 ? nt - (WS_D - 1) : 0; pub < nt; ++pub)
            if (lane == 0) ws_lds_write(ws_lds_addr(&ready[(int)(pub % WS_K)]), (int)pub);
#ifdef LZ_WS_PROBE
        if (lane == 0) {
            (void)c_done;
            (void)c_vm;
            lz_ws_probe[8 * blockIdx.x + 4] = clock64() - c_start;
            lz_ws_probe[8 * blockIdx.x + 5] = nt;
        }
#endif
        return;
    }
    // -------------------------------------------------------------- consumers
    const int cw = w - 1, g = lane >> 3, p = lane & 7;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)(nx * 128), 0x00020000);
    const uint32_t lane_off = 16u * p;
#ifdef LZ_WS_PROBE
    long long c_ready = 0, c_gather = 0, c_steps = 0;
    const long long c_cstart = clock64();
    const long long w_cstart = wall_clock64();
#endif
    for (int64_t i = 0; i < nt; ++i) {
        const int s = (int)(i % WS_K);
        const int64_t t = begin + k + i * K;
        const int64_t r0 = t * WS_TR;
        long spin = 0;
        WS_T(t2);
        while (ld(&ready[s]) != (int)i && ++spin < kWsSpin) __builtin_amdgcn_s_sleep(1);
#ifdef LZ_WS_PROBE
        c_ready += clock64() - t2;
#endif
        if (spin >= kWsSpin) { *err = 2; break; }
        asm volatile("" ::: "memory");
        const typename C::Stage &S = st[s];
        const int64_t kA = S.rp[0];
        const int co = (int)(kA & 3), vo = (int)(kA & 1);  // stage offsets of entry kA
        const int runlen = (int)(S.rp[(r0 + WS_TR < n ? WS_TR : n - r0)] - kA);
        const int lr = 16 * cw + g;  // local rows lr, lr + 8
        const int nrow = (int)(n - r0 < WS_TR ? n - r0 : WS_TR);
        const int o0 = lr < nrow ? (int)(S.rp[lr] - kA) : 0;
        const int len0 = lr < nrow ? (int)(S.rp[lr + 1] - kA) - o0 : 0;
        const int o1 = lr + 8 < nrow ? (int)(S.rp[lr + 8] - kA) : 0;
        const int len1 = lr + 8 < nrow ? (int)(S.rp[lr + 9] - kA) - o1 : 0;
        const int cnt = len0 + len1;
        double y[4] = {0.0, 0.0, 0.0, 0.0};
        // the tile-uniform choice of (col, val) source is made outside the loop:
        // a merged loop makes the compiler wait vmcnt(0) before every LDS read
        // (the global-path load could target the same register), which
        // serialises every gather behind the previous ones
        WS_T(t3);
        if (runlen <= WS_CAP)
            ws_gather(S.col + co, S.val + vo, o0, len0, o1, cnt, xr, lane_off, y);
        else
            ws_gather(col + kA, val + kA, o0, len0, o1, cnt, xr, lane_off, y);
#ifdef LZ_WS_PROBE
        c_gather += clock64() - t3;
        c_steps += (cnt + 7) / 8;
#endif
        // this wave no longer reads the stage (its LDS reads have returned)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&done[s], 1);
#ifdef LZ_WS_NOSTORE
        if (y[0] == 1.2345e300) {  // diagnostic build: keep the math, drop the stores
#endif
        if (lr < nrow) *reinterpret_cast<double2 *>(Y + (r0 + lr) * 16 + 2 * p) = double2{y[0], y[1]};
        if (lr + 8 < nrow) *reinterpret_cast<double2 *>(Y + (r0 + lr + 8) * 16 + 2 * p) = double2{y[2], y[3]};
#ifdef LZ_WS_NOSTORE
        }
#endif
    }
#ifdef LZ_WS_PROBE
    if (cw == 0 && lane == 0) {
        lz_ws_probe[8 * blockIdx.x + 2] = c_ready;
        lz_ws_probe[8 * blockIdx.x + 3] = clock64() - c_cstart;
        lz_ws_probe[8 * blockIdx.x + 6] = w_cstart;
        lz_ws_probe[8 * blockIdx.x + 1] = c_gather;
        lz_ws_probe[8 * blockIdx.x + 0] = c_steps;
        lz_ws_probe[8 * blockIdx.x + 7] = wall_clock64();
    }
#endif
}

// Merge-based (nnz-split) tile SpMM.  Row-wise gathering wastes the load slots
// past each row's end: with 8 loads per step and ~10 nnz per row only 61 % of
// the issued 16-B gathers carry an entry on the C3 operator, and the gather
// pipe (TA: ~34 TB/s of 128-B L2-resident rows chip-wide, measured) is what
// the kernel waits on.  Here the tile's run of N entries is split evenly over
// the G groups (E = N/G rounded up to 8 per group, 91 % slot use at 128 rows),
// each group walks its range 8 entries per step and emits a row's partial sum
// whenever the row id changes: rows wholly inside a group are stored
// directly, a group's first and last rows go to LDS slots (HEAD, TAIL) and are
// finished after a barrier by summing the slots of the groups that cover
// them, in group order -- deterministic for a given tile size.  Tiles whose
// run exceeds CAP are processed row-wise from global memory.
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
template <typename T, int B, int TR, int CAP, int UNR = 8, bool NT = false, int GAUX = 0, int MODE = 2>
__global__ __launch_bounds__(256) void k_spmm_seg(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx, int64_t nx,
                                                  T *__restrict__ Y, int64_t ldy, int *__restrict__ longq)
{
    // MODE 0: tiles whose run exceeds the stage are queued (longq[0] = count,
    //         longq[1..] = tile ids) for MODE 1, so their code path costs the
    //         main kernel no registers;
    // MODE 1: persistent blocks over the queued tiles: CAP-sized chunks, each
    //         split over the 32 groups; rows accumulate in the LDS Y tile
    //         across chunks (chunk order, then group order: bitwise
    //         reproducible).  A row-wise walk would leave one 8-lane group
    //         serialising a 10^5-entry row (power-law degrees, config 5);
    // MODE 2: long tiles walked row-wise in place (A/B, other tile heights).
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, G = 256 / LPR;
    static_assert(TR <= 255, "row ids are bytes");
    __shared__ int32_t rel[TR + 1];
    __shared__ int32_t cs[CAP + UNR];
    __shared__ T vs[CAP + UNR];
    __shared__ uint8_t rid[CAP + UNR];
    __shared__ Vec<T, VEC> yt[TR][LPR];      // the tile's finished rows
    __shared__ Vec<T, VEC> head[G][LPR];     // a group's piece of a row begun in an earlier slice
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const __amdgpu_buffer_rsrc_t xr = lz_rsrc(X, (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
    const uint32_t rowb = (uint32_t)(ldx * sizeof(T)), lane_off = p * VEC * sizeof(T);
    Vec<T, VEC> zero;
#pragma unroll
    for (int i = 0; i < VEC; ++i) zero.v[i] = T(0);
    if constexpr (MODE == 1) {
        const int cnt = longq[0];
        for (int qi = blockIdx.x; qi < cnt; qi += gridDim.x) {
            const int64_t r0 = (int64_t)longq[1 + qi] * TR;
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
                cs[k] = col[c0 + k];
                vs[k] = val[c0 + k];
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
#pragma unroll
                    for (int t = 0; t < UNR; ++t) {
                        const uint32_t off =
                            s0 + t < end ? __umul24((unsigned)cc[t], rowb) + lane_off : 0x80000000u;
                        xs[t] = ldbuf<T, VEC, GAUX>(xr, off);
                    }
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
                const int a = (rel[r] > cb ? rel[r] : cb) - cb, e = (rel[r + 1] < cb + Nc ? rel[r + 1] : cb + Nc) - cb;
                if (a >= e) continue;
                const int g1 = a / E, g2 = (e - 1) / E;
                for (int g = g1 + 1; g <= g2; ++g) {
#pragma unroll
                    for (int i2 = 0; i2 < VEC; ++i2) yt[r][p].v[i2] += head[g][p].v[i2];
                }
            }
        }
        __syncthreads();
        for (int idx = tid; idx < nrows * LPR; idx += 256)
            stv<T, VEC>(Y + (r0 + idx / LPR) * ldy + (idx % LPR) * VEC, yt[idx / LPR][idx % LPR]);
        }
        return;
    } else {
    const int64_t r0 = xcd_remap(blockIdx.x, gridDim.x) * TR;
    const int nrows = (int)((n - r0) < TR ? (n - r0) : TR);
    const int64_t kA = rp[r0];
    if (tid <= nrows) rel[tid] = (int)(rp[r0 + tid] - kA);
    const int64_t N64 = rp[r0 + nrows] - kA;
    if (N64 > CAP) {  // block-uniform
        if constexpr (MODE == 0) {
            if (tid == 0) longq[1 + atomicAdd(&longq[0], 1)] = (int)(r0 / TR);
            return;
        } else {
        for (int r = gi; r < nrows; r += G) {
                const int64_t a = rp[r0 + r], e = rp[r0 + r + 1];
                Vec<T, VEC> acc = zero;
                for (int64_t k = a; k < e; k += UNR) {
                    Vec<T, VEC> xs[UNR];
                    T vv[UNR];
#pragma unroll
                    for (int t = 0; t < UNR; ++t) {
                        const bool ok = k + t < e;
                        vv[t] = ok ? val[k + t] : T(0);
                        const uint32_t off = ok ? __umul24((unsigned)col[k + t], rowb) + lane_off : 0x80000000u;
                        xs[t] = ldbuf<T, VEC>(xr, off);
                    }
#pragma unroll
                    for (int t = 0; t < UNR; ++t)
#pragma unroll
                        for (int i = 0; i < VEC; ++i) acc.v[i] = fma(vv[t], xs[t].v[i], acc.v[i]);
                }
                stv<T, VEC>(Y + (r0 + r) * ldy + p * VEC, acc);
            }
            return;
        }
    }
    const int N = (int)N64;
    {  // stage the run with 16-B loads (aligned down; a piece reaching past nnz,
       // last tile only, element-wise), then the row id of every entry
        constexpr int EPV = 16 / (int)sizeof(T);
        constexpr int SPTC = ((CAP + 4) / 4 + 255) / 256, SPTV = ((CAP + EPV) / EPV + 255) / 256;
        const int64_t nnz = rp[n], kB = kA + N;
        const int64_t bc = kA & ~(int64_t)3, bv = kA & ~(int64_t)(EPV - 1);
        const __amdgpu_buffer_rsrc_t cr = lz_rsrc(col + bc, 0x7fffffffu);
        const __amdgpu_buffer_rsrc_t vr = lz_rsrc(val + bv, 0x7fffffffu);
        constexpr int AUX = NT ? 2 : 0;  // nt: streamed once, keep the X window in L2
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
        __syncthreads();  // rel
        if (tid < nrows)
            for (int k = rel[tid]; k < rel[tid + 1]; ++k) rid[k] = (uint8_t)tid;
#pragma unroll
        for (int q = 0; q < SPTC; ++q) {
            const int64_t k = bc + 4 * (int64_t)(tid + 256 * q);
            const int32_t cv[4] = {ct[q].x, ct[q].y, ct[q].z, ct[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (k + e >= kA && k + e < kB) cs[k + e - kA] = cv[e];
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
                    s0 + t < end ? __umul24((unsigned)cc[t], rowb) + lane_off : 0x80000000u;
                xs[t] = ldbuf<T, VEC, GAUX>(xr, off);
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
    for (int idx = tid; idx < nrows * LPR; idx += 256) {
        T *dst = Y + (r0 + idx / LPR) * ldy + (idx % LPR) * VEC;
        if constexpr (NT && sizeof(T) * VEC == 16) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            u32x4 u;
            __builtin_memcpy(&u, &yt[idx / LPR][idx % LPR], 16);
            __builtin_nontemporal_store(u, reinterpret_cast<u32x4 *>(dst));
        } else {
            stv<T, VEC>(dst, yt[idx / LPR][idx % LPR]);
        }
    }
    }  // MODE 0 / 2
}

template <typename T, int B, int TR, int CAP>
__global__ __launch_bounds__(256) void k_spmm_merge(int64_t n, const int64_t *__restrict__ rp,
                                                    const int32_t *__restrict__ col,
                                                    const T *__restrict__ val,
                                                    const T *__restrict__ X, int64_t ldx, int64_t nx,
                                                    T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, G = 256 / LPR, UNR = 8, SPT = CAP / 256;
    static_assert(TR <= 255, "row ids are bytes");
    __shared__ int32_t rel[TR + 1];
    __shared__ int32_t cs[CAP + UNR];
    __shared__ T vs[CAP + UNR];
    __shared__ uint8_t rid[CAP + UNR];
    __shared__ Vec<T, VEC> part[G][2][LPR];  // HEAD / TAIL partial rows per group
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int64_t r0 = xcd_remap(blockIdx.x, gridDim.x) * TR;
    const int nrows = (int)((n - r0) < TR ? (n - r0) : TR);
    const int64_t kA = rp[r0];
    if (tid <= nrows) rel[tid] = (int)(rp[r0 + tid] - kA);
    const int64_t N64 = rp[r0 + nrows] - kA;
    const __amdgpu_buffer_rsrc_t xr = lz_rsrc(X, (uint32_t)(nx * ldx * (int64_t)sizeof(T)));
    const uint32_t rowb = (uint32_t)(ldx * sizeof(T)), lane_off = p * VEC * sizeof(T);
    auto store_row = [&](int r, const Vec<T, VEC> &o) { stv<T, VEC>(Y + (r0 + r) * ldy + p * VEC, o); };
    if (N64 > CAP) {  // block-uniform: long rows -- row-wise straight from global
        for (int r = gi; r < nrows; r += G) {
            const int64_t a = rp[r0 + r], e = rp[r0 + r + 1];
            Vec<T, VEC> acc;
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc.v[i] = T(0);
            for (int64_t k = a; k < e; k += UNR) {
                Vec<T, VEC> xs[UNR];
                T vv[UNR];
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    const bool ok = k + t < e;
                    vv[t] = ok ? val[k + t] : T(0);
                    const uint32_t off = ok ? __umul24((unsigned)col[k + t], rowb) + lane_off : 0x80000000u;
                    xs[t] = ldbuf<T, VEC>(xr, off);
                }
#pragma unroll
                for (int t = 0; t < UNR; ++t)
#pragma unroll
                    for (int i = 0; i < VEC; ++i) acc.v[i] = fma(vv[t], xs[t].v[i], acc.v[i]);
            }
            store_row(r, acc);
        }
        return;
    }
    const int N = (int)N64;
    {  // stage the run (one batch of loads) and the row id of every entry
        int32_t ct[SPT];
        T vt[SPT];
#pragma unroll
        for (int q = 0; q < SPT; ++q) {
            const int k = tid + 256 * q;
            ct[q] = k < N ? col[kA + k] : 0;
            vt[q] = k < N ? val[kA + k] : T(0);
        }
        __syncthreads();  // rel
        if (tid < nrows)
            for (int k = rel[tid]; k < rel[tid + 1]; ++k) rid[k] = (uint8_t)tid;
#pragma unroll
        for (int q = 0; q < SPT; ++q) {
            if (tid + 256 * q < N) {
                cs[tid + 256 * q] = ct[q];
                vs[tid + 256 * q] = vt[q];
            }
        }
        if (tid < UNR) {
            cs[N + tid] = 0;
            vs[N + tid] = T(0);
            rid[N + tid] = 255;
        }
        __syncthreads();
    }
    const int E = ((N + G - 1) / G + UNR - 1) / UNR * UNR;
    const int start = gi * E, end = (start + E < N) ? start + E : N;
    if (start < end) {  // group-uniform
        const int first = rid[start];
        int cur = first;
        Vec<T, VEC> acc;
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc.v[i] = T(0);
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
                    s0 + t < end ? __umul24((unsigned)cc[t], rowb) + lane_off : 0x80000000u;
                xs[t] = ldbuf<T, VEC>(xr, off);
            }
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                const int r = s0 + t < end ? rr[t] : cur;
                if (r != cur) {  // the segment of row cur ends: emit it
                    if (cur == first) part[gi][0][p] = acc;
                    else store_row(cur, acc);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) acc.v[i] = T(0);
                    cur = r;
                }
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc.v[i] = fma(vv[t], xs[t].v[i], acc.v[i]);
            }
        }
        part[gi][cur == first ? 0 : 1][p] = acc;
    }
    __syncthreads();
    // finish the rows that are some group's first or last row, and empty rows
    for (int r = gi; r < nrows; r += G) {
        const int a = rel[r], e = rel[r + 1];
        Vec<T, VEC> sum;
#pragma unroll
        for (int i = 0; i < VEC; ++i) sum.v[i] = T(0);
        if (a == e) {
            store_row(r, sum);
            continue;
        }
        const int g1 = a / E, g2 = (e - 1) / E;
        const bool head1 = a <= g1 * E;                            // first row of g1
        const int end2 = (g2 + 1) * E < N ? (g2 + 1) * E : N;
        const bool tail2 = e >= end2;                              // last row of g2
        if (g1 == g2 && !head1 && !tail2) continue;                // stored by its group
        for (int g = g1; g <= g2; ++g) {
            const Vec<T, VEC> &q = part[g][(g == g1 && !head1) ? 1 : 0][p];
#pragma unroll
            for (int i = 0; i < VEC; ++i) sum.v[i] += q.v[i];
        }
        store_row(r, sum);
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

template <typename T, int B>
static int launch_spmm_rm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col,
                          const T *val, const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int CAP = S::RB * 32 < 1024 ? 1024 : (S::RB * 32 > 4096 ? 4096 : S::RB * 32);
    if (n <= 0) return LZ_OK;
    // LZ_SPMM_KERNEL=tile forces the original tile kernel (A/B only); the
    // buffer-load kernel needs 32-bit X byte offsets and 24-bit columns
    static const char *variant = getenv("LZ_SPMM_KERNEL");
    static const char *rpg_env = getenv("LZ_SPMM_RPG");
    const int rpg = rpg_env ? atoi(rpg_env) : 2;
    const int64_t tiles = ceil_div(n, (int64_t)S::RB * rpg);
    LZ_ARG_CHECK(tiles < (1LL << 31), "too many row tiles");
    // X has nx rows (the operator's columns), not n
    const bool buf_ok = nx * ldx * (int64_t)sizeof(T) < (1LL << 31) && nx < (1 << 24);
    constexpr int CAP2 = CAP * 2 < 4096 ? CAP * 2 : 4096;
    const int ev = prof_begin(h, PROF_SPMM);
    if constexpr (B == 16 && std::is_same<T, double>::value) {
        if (buf_ok && ldx == 16 && ldy == 16 && variant && variant[0] == 'w') {
            // LZ_SPMM_KERNEL=w<cfg>: 0: 8 consumers, 3 stages, depth 2 (2 blocks/CU)
            //   1: 4 consumers, 4 stages, depth 3 (3 blocks/CU)  2: 8 consumers, 4 stages, depth 3 (1/CU)
            const int cfg = variant[1] ? variant[1] - '0' : 0;
            auto go = [&](auto kern, int tr, int bpc, int threads) {
                const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)tr),
                                                                             (int64_t)h->n_cu * bpc));
                hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, h->stream, n, rp, col, val, X, nx, Y,
                                   h->err_flag);
            };
            if (cfg == 1)
                go(k_spmm_ws<4, 4, 3, 888>, 64, 3, 320);
            else if (cfg == 2)
                go(k_spmm_ws<8, 4, 3, 1784>, 128, 1, 576);
            else
                go(k_spmm_ws<8, 3, 2, 1784>, 128, 2, 576);
            prof_end(h, ev);
            LZ_LAUNCH_CHECK();
            return LZ_OK;
        }
    }
    // default for 128-B rows (b = 16 fp64, b = 32 fp32): the nnz-split kernel
    // (48-row tiles, nt CSR stream); LZ_SPMM_KERNEL=b forces k_spmm_buf, s3/s6/s9
    // other tile heights (A/B)
    const bool seg = buf_ok && S::LPR == 8 && !(variant && variant[0] != 's');
    if (seg) {
        const char c = variant ? variant[1] : '4';
        const int tr = c == '9' ? 96 : c == '6' ? 64 : c == '3' ? 32 : 48;
        const int64_t st = ceil_div(n, (int64_t)tr);
        LZ_ARG_CHECK(st < (1LL << 31), "too many row tiles");
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)st), dim3(256), 0, h->stream, n, rp, col, val, X, ldx, nx, Y,
                               ldy, nullptr);
        };
        if (tr == 96)
            go(k_spmm_seg<T, B, 96, 1536, 8, true>);
        else if (tr == 64)
            go(k_spmm_seg<T, B, 64, 1024, 8, true>);
        else if (tr == 32)
            go(k_spmm_seg<T, B, 32, 512, 8, true>);
        else if (c == '5')  // A/B: long runs walked row-wise in place
            go(k_spmm_seg<T, B, 48, 768, 8, true, 0, 2>);
        else {
            // long tiles (run > stage) queued by the main kernel, then chunked by a
            // persistent second kernel (an empty queue costs one short launch)
            if ((size_t)st + 1 > h->longq_cap) {
                LZ_HIP_TRY(hipStreamSynchronize(h->stream));
                (void)hipFree(h->longq);
                h->longq = nullptr;
                LZ_HIP_TRY(hipMalloc(&h->longq, sizeof(int) * ((size_t)st + 1)));
                h->longq_cap = (size_t)st + 1;
            }
            LZ_HIP_TRY(hipMemsetAsync(h->longq, 0, sizeof(int), h->stream));
            hipLaunchKernelGGL((k_spmm_seg<T, B, 48, 768, 8, true, 0, 0>), dim3((unsigned)st), dim3(256), 0, h->stream,
                               n, rp, col, val, X, ldx, nx, Y, ldy, h->longq);
            const int g2 = (int)std::max<int64_t>(1, std::min<int64_t>(st, (int64_t)h->n_cu * 4));
            hipLaunchKernelGGL((k_spmm_seg<T, B, 48, 768, 8, true, 0, 1>), dim3(g2), dim3(256), 0, h->stream, n, rp,
                               col, val, X, ldx, nx, Y, ldy, h->longq);
        }
    } else if (buf_ok && variant && variant[0] == 'p') {  // first-touch prefetch round (A/B)
        hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 8, 1, 4>), dim3((unsigned)tiles), dim3(256), 0,
                           h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
    } else if (buf_ok && variant && variant[0] == 'm') {
        const int64_t mt = ceil_div(n, (int64_t)128);
        LZ_ARG_CHECK(mt < (1LL << 31), "too many row tiles");
        hipLaunchKernelGGL((k_spmm_merge<T, B, 128, 2048>), dim3((unsigned)mt), dim3(256), 0,
                           h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
    } else if (buf_ok && variant && variant[0] == 'x') {  // occupancy experiments: x<unr><waves/SIMD>
        const int unr = variant[1] - '0', occ = variant[2] - '0';
        if (unr == 4 && occ == 8)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 4, 8>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (unr == 4 && occ == 6)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 4, 6>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (unr == 8 && occ == 6)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 8, 6>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2, 8, 8>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
    } else if (buf_ok && !(variant && variant[0] == 't')) {  // k_spmm_buf
        if (rpg == 1)
            hipLaunchKernelGGL((k_spmm_buf<T, B, CAP, 1>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (rpg == 2)
            hipLaunchKernelGGL((k_spmm_buf<T, B, 1024, 2>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_buf<T, B, 4096, 4>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
    } else {
        if (rpg == 1)
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP, 1>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else if (rpg == 2)
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP2, 2>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_lds<T, B, 4096, 4>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, nx, Y, ldy);
    }
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

template <typename T>
int spmm_rm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy)
{
    switch (b) {
    case 1:
        LZ_ARG_CHECK(ldx == 1 && ldy == 1, "b = 1 row-major needs ldx = ldy = 1");
        return spmv<T>(h, n, rp, col, val, X, Y, 0);
    case 2: return launch_spmm_rm<T, 2>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    case 4: return launch_spmm_rm<T, 4>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    case 8: return launch_spmm_rm<T, 8>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    case 16: return launch_spmm_rm<T, 16>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    case 32: return launch_spmm_rm<T, 32>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    case 64: return launch_spmm_rm<T, 64>(h, n, rp, col, val, X, ldx, nx, Y, ldy);
    default:
        set_error("row-major SpMM supports b in {1,2,4,8,16,32,64}, got %d", b);
        return LZ_E_ARG;
    }
}

// Layout change between a column-major block (b columns, leading dimension
// ld) and a row-major one (ld = b), kCmRows rows per workgroup through LDS:
// both the column reads and the row writes are coalesced.  IN: col -> row
// (src = column-major, ld = its leading dimension); !IN: row -> col.
constexpr int kCmRows = 128;

template <typename T, bool IN>
__global__ __launch_bounds__(256) void k_cm_transpose(int64_t rows, int b, const T *__restrict__ src,
                                                      int64_t ld, T *__restrict__ dst)
{
    extern __shared__ __align__(16) unsigned char cm_lds[];  // b * (kCmRows + 1) elements
    T *tile = reinterpret_cast<T *>(cm_lds);
    const int64_t r0 = (int64_t)blockIdx.x * kCmRows;
    const int nr = (int)(rows - r0 < kCmRows ? rows - r0 : kCmRows);
    const int tot = nr * b;
    if constexpr (IN) {
        for (int i = threadIdx.x; i < kCmRows * b; i += blockDim.x) {
            const int c = i / kCmRows, r = i % kCmRows;
            if (r < nr) tile[c * (kCmRows + 1) + r] = src[(int64_t)c * ld + r0 + r];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < tot; i += blockDim.x) {
            const int r = i / b, c = i % b;
            dst[r0 * b + i] = tile[c * (kCmRows + 1) + r];
        }
    } else {
        for (int i = threadIdx.x; i < tot; i += blockDim.x) {
            const int r = i / b, c = i % b;
            tile[c * (kCmRows + 1) + r] = src[r0 * b + i];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kCmRows * b; i += blockDim.x) {
            const int c = i / kCmRows, r = i % kCmRows;
            if (r < nr) dst[(int64_t)c * ld + r0 + r] = tile[c * (kCmRows + 1) + r];
        }
    }
}

template <typename T>
int spmm_cm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, int64_t nx, T *Y, int64_t ldy)
{
    if (n <= 0) return LZ_OK;
    // b = 2..64 (powers of two): a column-major gather touches b lines per nonzero, the row-major
    // kernel one; transposing X in and Y out (read + write of each block once)
    // costs less (Yee N=160, b=16 fp32: 3.69 ms direct).  LZ_SPMM_CM=direct: the
    // one-pass kernel.
    static const char *cm_env = getenv("LZ_SPMM_CM");
    if (b >= 2 && (b & (b - 1)) == 0 && !(cm_env && cm_env[0] == 'd')) {  // the row-major kernel's b
        const size_t need = sizeof(T) * (size_t)b * (size_t)(nx + n);
        if (need > h->cm_cap) {
            LZ_HIP_TRY(hipStreamSynchronize(h->stream));
            (void)hipFree(h->cm_buf);
            h->cm_buf = nullptr;
            h->cm_cap = 0;
            LZ_HIP_TRY(hipMalloc(&h->cm_buf, need));
            h->cm_cap = need;
        }
        T *Xr = static_cast<T *>(h->cm_buf), *Yr = Xr + (size_t)b * nx;
        const size_t lds = sizeof(T) * (size_t)b * (kCmRows + 1);
        hipLaunchKernelGGL((k_cm_transpose<T, true>), dim3((unsigned)ceil_div(nx, (int64_t)kCmRows)), dim3(256), lds,
                           h->stream, nx, b, X, ldx, Xr);
        LZ_LAUNCH_CHECK();
        LZ_TRY(spmm_rm<T>(h, n, rp, col, val, b, Xr, b, nx, Yr, b));
        hipLaunchKernelGGL((k_cm_transpose<T, false>), dim3((unsigned)ceil_div(n, (int64_t)kCmRows)), dim3(256), lds,
                           h->stream, n, b, Yr, ldy, Y);
        LZ_LAUNCH_CHECK();
        return LZ_OK;
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

template int spmm_rm<double>(lz_handle *, int64_t, const int64_t *, const int32_t *,
                             const double *, int, const double *, int64_t, int64_t, double *, int64_t);
template int spmm_rm<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, int64_t, float *, int64_t);
template int spmm_cm<double>(lz_handle *, int64_t, const int64_t *, const int32_t *,
                             const double *, int, const double *, int64_t, int64_t, double *, int64_t);
template int spmm_cm<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, int64_t, float *, int64_t);
template int spmv<double>(lz_handle *, int64_t, const int64_t *, const int32_t *, const double *,
                          const double *, double *, int64_t);
template int spmv<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                         const float *, float *, int64_t);

}  // namespace lz
