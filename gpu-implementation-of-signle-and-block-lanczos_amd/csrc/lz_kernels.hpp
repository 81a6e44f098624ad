// lz_kernels.hpp -- device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lz {

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));

// XCD-contiguous work schedule.  Observed (speed only, never correctness):
// workgroups are dealt round-robin over the 8 XCDs, so block b runs on XCD
// b % 8.  Giving XCD x the contiguous unit range [U*x/8, U*(x+1)/8) keeps each
// XCD's private L2 on a sliding window of rows, which is what a banded sparse
// gather needs.  Every unit is visited exactly once for any grid size.
struct XcdSched {
    int64_t begin, end, step;
    __device__ XcdSched(int64_t units)
    {
        const int64_t G = gridDim.x, b = blockIdx.x;
        if (G < 8) {
            begin = b; end = units; step = G;
            return;
        }
        const int64_t x = b & 7, k = b >> 3;
        const int64_t K = (G - x + 7) >> 3;  // blocks on this XCD
        begin = units * x / 8 + k;
        end = units * (x + 1) / 8;
        step = K;
    }
};

// Bijective XCD-aware block -> tile remap (cdna_hip_programming.md T1): blocks
// are dealt round-robin over the 8 XCDs (speed only), so XCD x runs blocks
// x, x+8, ...; map them to the contiguous tile range of XCD x.  With one tile
// per block and in-order dispatch, the tiles in flight on one XCD form a
// narrow sliding window, which keeps a banded operator's X gather in its L2.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb)
{
    if (nb < 8) return b;
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return (x < r) ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// wave-private LDS hand-off: make this wave's LDS writes visible to its own
// later LDS reads (DS ops of one wave complete in order once lgkmcnt drains).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 16-byte (or smaller) vector of VEC elements of T
template <typename T, int VEC>
struct Vec {
    T v[VEC];
};

template <typename T, int VEC>
__device__ __forceinline__ Vec<T, VEC> ldv(const T *p)
{
    Vec<T, VEC> r;
    if constexpr (sizeof(T) * VEC == 16) {
        const uint4 u = *reinterpret_cast<const uint4 *>(p);
        __builtin_memcpy(&r, &u, 16);
    } else if constexpr (sizeof(T) * VEC == 8) {
        const uint2 u = *reinterpret_cast<const uint2 *>(p);
        __builtin_memcpy(&r, &u, 8);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) r.v[i] = p[i];
    }
    return r;
}

template <typename T, int VEC>
__device__ __forceinline__ void stv(T *p, const Vec<T, VEC> &r)
{
    if constexpr (sizeof(T) * VEC == 16) {
        uint4 u;
        __builtin_memcpy(&u, &r, 16);
        *reinterpret_cast<uint4 *>(p) = u;
    } else if constexpr (sizeof(T) * VEC == 8) {
        uint2 u;
        __builtin_memcpy(&u, &r, 8);
        *reinterpret_cast<uint2 *>(p) = u;
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) p[i] = r.v[i];
    }
}

// v_mfma_f64_16x16x4_f64: D(16x16) += A(16x4) * B(4x16).
// Lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; D lane l holds
// D[(l>>4) + 4*r][l&15], r = 0..3 -- i.e. for each r, element l of a
// contiguous row-major 4x16 chunk.
__device__ __forceinline__ d4_t mfma16(double a, double b, d4_t c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---- wave-specialised persistent kernels (loader wave + consumer waves) ----
// k_spmm_ws (lz_spmm.hip) and k_fused_ws16 (lz_fused.hip).
constexpr int ws_instr(int pieces) { return (pieces + 63) / 64; }
#ifdef LZ_WS_PROBE
// diagnostic builds (scripts/probe/ws_probe*.hip): per-block wait/cycle records
__device__ long long *lz_ws_probe;
__device__ int lz_ws_dbg;  // diagnostic timing masks (probe builds only)
#define WS_T(v) const long long v = clock64()
#else
#define WS_T(v)
#endif
#ifdef LZ_WS_PROBE_TL
// per-tile event timeline of blocks 0-3 (tiles < 256): 32 stamps per tile
__device__ long long *lz_ws_tl;
#define WS_TL(tile, slot)                                                                        \
    do {                                                                                         \
        if (blockIdx.x < 4 && (tile) < 256 && (threadIdx.x & 63) == 0)                         \
            lz_ws_tl[((int64_t)blockIdx.x * 256 + (tile)) * 32 + (slot)] = clock64();           \
    } while (0)
#else
#define WS_TL(tile, slot)
#endif
constexpr long kWsSpin = 1L << 24;

// Gather window of the 32-bit buffer-addressed kernels when the gather source
// has 2^24 rows of 128 B or more (X past 2 GiB): a strip / tile reads X
// through a buffer resource based kWinRows / 2 rows before its own row, and a
// once-per-operator check (gather_window_ok) proved its columns fall inside.
constexpr int64_t kWinRows = (1 << 24) - 1;

typedef __attribute__((address_space(3))) void ws_lds_t;

// LDS word access from the loader wave in inline asm: after an LDS-DMA the
// compiler inserts vmcnt(0) before any LDS instruction it emits (the DMA could
// alias it), which would wait for the tile in flight.  These words are never
// DMA targets.
__device__ __forceinline__ uint32_t ws_lds_addr(int *p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int *)p;
}
__device__ __forceinline__ int ws_lds_read(uint32_t a)
{
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}
__device__ __forceinline__ void ws_lds_write(uint32_t a, int v)
{
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

template <int AUX = 0>
__device__ __forceinline__ void ws_dma(__amdgpu_buffer_rsrc_t r, void *lds_base, int pieces, int lane)
{
#pragma unroll
    for (int q = 0; q < (pieces + 63) / 64; ++q) {
        const int piece = 64 * q + lane;
        // pieces past the end get an out-of-range offset (no memory access)
        const uint32_t off = piece < pieces ? 16u * piece : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (ws_lds_t *)((char *)lds_base + 1024 * q), 16, off, 0, 0, AUX);
    }
}

// Y rows (g, g+8) of one group: the two rows' entries walked as one list, 8 per
// step; masked slots read entry o0 and load nothing (out-of-range offset).
// AUX: the gather loads' cache-policy bits (16 = sc1: L2-served, bypassing L1,
// for a source written inside the same launch).
template <typename CP, typename VP, int AUX = 0>
__device__ __forceinline__ void ws_gather(CP cp, VP vp, int o0, int len0, int o1, int cnt,
                                          __amdgpu_buffer_rsrc_t xr, uint32_t lane_off, double y[4],
                                          uint32_t wb = 0)
{
    for (int f = 0; f < cnt; f += 8) {
        int32_t c[8];
        double v[8];
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
            const int ff = f + tt;
            int o = ff < len0 ? o0 + ff : o1 + (ff - len0);
            o = ff < cnt ? o : o0;
            c[tt] = cp[o];
            v[tt] = vp[o];
        }
        double2 xs[8];
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
            const uint32_t off = f + tt < cnt ? __umul24((unsigned)c[tt] - wb, 128u) + lane_off : 0x80000000u;
            const auto u4 = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, AUX);
            __builtin_memcpy(&xs[tt], &u4, 16);
        }
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
            if (f + tt < len0) {
                y[0] = fma(v[tt], xs[tt].x, y[0]);
                y[1] = fma(v[tt], xs[tt].y, y[1]);
            } else {  // masked entries: x == 0
                y[2] = fma(v[tt], xs[tt].x, y[2]);
                y[3] = fma(v[tt], xs[tt].y, y[3]);
            }
        }
    }
}

// ---- pass-1 stage layout (k_fused_pp16 in lz_fused.hip, k_wf16 in lz_wf.hip) ----
// Rows past n are out of range for the DMA and land as zeros.
template <int NC, int CAP, bool QREG = false, bool PR = false, typename CT = int32_t>
struct FwCfg {
    static constexpr int TR = 16 * NC;
    static constexpr int RP_PIECES = (TR + 2) * 8 / 16;
    static constexpr int CPP = 16 / (int)sizeof(CT);  // columns per 16-B piece
    static constexpr int COL_PIECES = (CAP + 2 * CPP) * (int)sizeof(CT) / 16;
    static constexpr int VAL_PIECES = (CAP + 4) * 8 / 16;
    static constexpr int DMA_INSTR =
        ws_instr(RP_PIECES) + ws_instr(COL_PIECES) + ws_instr(VAL_PIECES) + (QREG ? 0 : 2 * NC);
    static_assert(DMA_INSTR <= 63, "vmcnt immediate");
    struct Stage {
        int64_t rp[ws_instr(RP_PIECES) * 128];
        CT col[ws_instr(COL_PIECES) * 64 * CPP];
        double val[ws_instr(VAL_PIECES) * 128];
        double qt[QREG ? 2 : TR * 16];  // Q_{j-1} rows, per strip in slot order; then scratch
        uint64_t pr[PR ? 128 : 1];        // PR: the tile's strips' row orders (k_strip_pairs)
    };
    static constexpr int PR_PIECES = NC * 8 / 16 > 0 ? (NC * 8 + 15) / 16 : 1;
};


constexpr int64_t kPairPad = 16;  // >= strips per pass-1 tile (14)

// 16x16 scratch with XOR swizzle: element (r, c) at r*16 + (c ^ r); the MFMA
// operand read (16 rows, one column per lane group) hits 16 distinct banks.
__device__ __forceinline__ int fw_sw(int r, int c) { return r * 16 + (c ^ r); }

}  // namespace lz
