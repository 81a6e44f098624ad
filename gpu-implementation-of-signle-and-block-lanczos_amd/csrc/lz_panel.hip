// lz_panel.hip -- the column-panel SpMM candidate (round 5; b = 16 fp64):
// X staged through LDS in panels, row accumulators in registers.
//
// Why (DESIGN.md 4 SpMM): k_spmm_seg gathers one 128-B X line per nonzero
// through the texture path (1e8 lines = 12.8 GB of L2->L1 traffic at C3 for
// 1.28 GB of X), and that path -- ~20 cycles per 64-lane gather instruction,
// with the CSR stream's HBM latencies sharing the per-CU miss queue -- is what
// bounds it (0.77 ms with every input L2-resident, 1.18 ms as is).  Here a
// workgroup owns kPR consecutive rows and sweeps the X rows its columns reach
// in panels of kPW rows: each panel is loaded ONCE with coalesced 16-B loads
// (1 KB per wave-instruction) into LDS, and the block's entries in that panel
// read their X rows from LDS (ds_read_b128, no texture-path cost).  At C3
// (+-4096 band) a 2048-row block reaches (2048 + 8192) X rows for its 20480
// entries: half the lines of the gather kernel through the texture path.
//
// The entries come from a once-per-operator plan (scripts/panel_ab.py builds
// it with numpy for the measurement): for every row block and panel, the
// block's entries with columns in that panel in CSR order ("passes"; a panel
// with more than kPE entries is split over several passes), each stored as its
// value (8 B) and a 16-bit word (row slot << 9 | panel-local X row), the pass
// padded to 8 entries; per pass its panel's first X row, its first entry, and
// the 129 offsets of the block's 128 groups' lists in it.  That is 10 B per
// entry against CSR's 12 (the column becomes a 9-bit panel offset).
//
// Mapping: 16 waves; group G = 8 * wave + (lane >> 3) of 8 lanes owns rows
// r0 + 16 G + k, k = 0..15 (slot k), lane l8 = lane & 7 its 16-B piece (two
// doubles) of each row: 64 VGPRs of accumulators, indexed statically.  A pass
// runs, for k = 0..15, the group's entries of slot k while any group of the
// wave has one (a wave-uniform loop, ballot), so a wave pays the maximum over
// its 8 groups per slot.  Per row the entries are summed in column order, one
// fma chain: the same order as a row-sequential CSR product.
//
// Pipeline: one block per CU (LDS: two X panels of 64 KB + two entry buffers);
// the next pass's X panel and entries are loaded into registers before the
// current pass computes and written to the other LDS buffers after it, then
// ONE barrier per pass.
#include "lz_common.hpp"
#include "lz_diag.h"
#include "lz_internal.hpp"
#include "lz_kernels.hpp"

namespace lz {

constexpr int kPR = 2048;        // rows per block
constexpr int kPW = 512;         // X rows per panel
constexpr int kPE = 1536;        // entries per pass (at most)
constexpr int kPGO = 136;        // group-offset words per pass (kPR / 16 + 1 = 129 used, 16-B multiple)

__global__ __launch_bounds__(1024) void k_spmm_panel(int64_t n, int64_t nx, const double *__restrict__ X,
                                                     double *__restrict__ Y, const int32_t *__restrict__ bp0,
                                                     const int32_t *__restrict__ px0,
                                                     const int32_t *__restrict__ pe0,
                                                     const uint16_t *__restrict__ goff,
                                                     const double *__restrict__ ev, const uint16_t *__restrict__ ex)
{
    __shared__ double Xs[2][kPW * 16];
    __shared__ double Es[2][kPE];
    __shared__ uint16_t Ks[2][kPE];
    __shared__ uint16_t Go[2][kPGO];
    const int t = threadIdx.x, lane = t & 63, G = (t >> 6) * 8 + (lane >> 3), l8 = lane & 7;
    const int64_t r0 = (int64_t)blockIdx.x * kPR;
    const int i0 = bp0[blockIdx.x], i1 = bp0[blockIdx.x + 1];
    double2 acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = make_double2(0.0, 0.0);
    // pass i's data into registers: 4 x 16 B of the X panel, 16 B of values,
    // 16 B of entry words, 16 B of group offsets (by the threads that have them)
    uint4 xr[4], er, kr, gr;
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    auto fetch = [&](int i) {
        const int64_t xb = px0[i];
        const int e0 = pe0[i], ne = pe0[i + 1] - e0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t row = xb + (t + 1024 * q) / 8;  // 8 pieces of 16 B per X row
            xr[q] = row < nx ? reinterpret_cast<const uint4 *>(X + row * 16)[(t + 1024 * q) & 7] : z4;
        }
        er = 2 * t < ne ? reinterpret_cast<const uint4 *>(ev + e0)[t] : z4;
        kr = 8 * t < ne ? reinterpret_cast<const uint4 *>(ex + e0)[t] : z4;
        gr = t < kPGO / 8 ? reinterpret_cast<const uint4 *>(goff + (int64_t)i * kPGO)[t] : z4;
    };
    auto stash = [&](int b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) reinterpret_cast<uint4 *>(Xs[b])[t + 1024 * q] = xr[q];
        if (2 * t < kPE) reinterpret_cast<uint4 *>(Es[b])[t] = er;
        if (8 * t < kPE) reinterpret_cast<uint4 *>(Ks[b])[t] = kr;
        if (t < kPGO / 8) reinterpret_cast<uint4 *>(Go[b])[t] = gr;
    };
    if (i0 < i1) {
        fetch(i0);
        stash(0);
    }
    __syncthreads();
    for (int i = i0; i < i1; ++i) {
        const int b = (i - i0) & 1;
        if (i + 1 < i1) fetch(i + 1);  // in flight while this pass computes
        int cur = Go[b][G];
        const int end = Go[b][G + 1];
        const double *xs = Xs[b];
        const double *es = Es[b];
        const uint16_t *ks = Ks[b];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            while (true) {
                const uint32_t w = cur < end ? ks[cur] : 0xFFFFu;
                const bool on = (w >> 9) == (uint32_t)k;
                if (__ballot(on) == 0) break;  // wave-uniform
                if (on) {
                    const double v = es[cur];
                    const double2 x = *reinterpret_cast<const double2 *>(xs + (w & 511u) * 16 + 2 * l8);
                    acc[k].x = fma(v, x.x, acc[k].x);
                    acc[k].y = fma(v, x.y, acc[k].y);
                    ++cur;
                }
            }
        }
        if (i + 1 < i1) stash(b ^ 1);  // (buffer b ^ 1 was last read before the previous barrier)
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int64_t row = r0 + 16 * G + k;
        if (row < n) reinterpret_cast<double2 *>(Y + row * 16)[l8] = acc[k];
    }
}

int spmm_panel(lz_handle *h, int64_t n, int64_t nx, const double *X, double *Y, int nblocks, const int32_t *bp0,
               const int32_t *px0, const int32_t *pe0, const uint16_t *goff, const double *ev, const uint16_t *ex)
{
    LZ_ARG_CHECK(nblocks == ceil_div(n, (int64_t)kPR), "panel SpMM: one block per 2048 rows");
    if (n <= 0) return LZ_OK;
    const int ev_ = prof_begin(h, PROF_SPMM);
    hipLaunchKernelGGL(k_spmm_panel, dim3(nblocks), dim3(1024), 0, h->stream, n, nx, X, Y, bp0, px0, pe0, goff, ev,
                       ex);
    prof_end(h, ev_);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

}  // namespace lz

using namespace lz;

extern "C" int lz_debug_spmm_panel(lz_handle *h, int64_t n, int64_t nx, const void *X, void *Y, int nblocks,
                                   const int32_t *bp0, const int32_t *px0, const int32_t *pe0, const uint16_t *goff,
                                   const void *ev, const uint16_t *ex)
{
    LZ_ARG_CHECK(h && X && Y && bp0 && px0 && pe0 && goff && ev && ex, "panel SpMM: NULL argument");
    LZ_HIP_TRY(hipSetDevice(h->device));
    return spmm_panel(h, n, nx, static_cast<const double *>(X), static_cast<double *>(Y), nblocks, bp0, px0, pe0,
                      goff, static_cast<const double *>(ev), ex);
}
