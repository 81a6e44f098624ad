// lz_fused32.hip -- the Q-free block-Lanczos dense passes that run around a
// separate SpMM launch: b = 32 fp32 (BASELINE config C5) on
// v_mfma_f32_32x32x2_f32, and every other block width b <= 32 (fp64 or fp32,
// e.g. the reference driver's default N_COL = 4) on the VALU; gfx950.
//
// The iteration is the b = 16 fp64 one of lz_fused.hip / lz_api.hip
// (methods/block_lanczos.hpp:131-166 reassociated so Q_j = W_j beta_j^-1 is
// never stored), with the SpMM kept as its own launch: C5's power-law rows need
// the nnz-split tile kernel and its long-tile queue (lz_spmm.hip), and its
// random columns make the gather, not the dense work, the bound.  Per step:
//   SpMM     Y = A W_j                                         (A + 2 n b s)
//   pass E   Q_j = W_j beta_j^-1 (registers), W' = Y beta_j^-1 - W_{j-1} P1,
//            slabs of Q_j^T W', row probe of Q_j               (4 n b s)
//   finish   alpha_j = 0.5 (M + M^T), P2 = beta_j^-1 alpha_j
//   pass U   W'' = W' - W_j P2, slabs of W''^T W''              (3 n b s)
//   sqrtm    beta_{j+1}, beta_{j+1}^-1, P1 = beta_j^-1 beta_{j+1}
// against the reference order's 7 calls (A + 13 n b s).
//
// MFMA layout (32x32x2, f32): lane l supplies A[i = l&31][k] and B[k][j = l&31]
// at its k (k = 16(l>>5) + s at step s: a lane's A operands are 64 contiguous
// bytes of one row, four 16-B loads); register v of the result holds row
// (v&3) + 8(v>>2) + 4(l>>5), column l&31 of the 32 x 32 tile.  That result
// layout is also both operand layouts of a product contracted over the tile's
// rows (step v: k = (v&3) + 8(v>>2) + 4(l>>5)), so the Gram slabs take the
// result registers as they are, with no transpose.
#include <type_traits>
#include "lz_common.hpp"
#include "lz_internal.hpp"
#include "lz_kernels.hpp"

namespace lz {

typedef float f16v_t __attribute__((ext_vector_type(16)));
typedef unsigned u4v_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16v_t mfma32(float a, float b, f16v_t c)
{
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// a[s] = M[row][16 hh + s] for s = 0..15 (zeros past n): four 16-B loads
// (plain: the two halves of a 128-B row come from two lanes' loads, and with
// non-temporal loads C5's pass UB took 0.28 ms longer -- presumably each line
// fetched twice; profiles/r05u_c5_el_ub_nt_ab.log)
__device__ __forceinline__ void aop32(const float *__restrict__ M, int64_t row, bool ok, int hh, float a[16])
{
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) x = *reinterpret_cast<const float4 *>(M + row * 32 + 16 * hh + 4 * c);
        a[4 * c] = x.x; a[4 * c + 1] = x.y; a[4 * c + 2] = x.z; a[4 * c + 3] = x.w;
    }
}

// B operand table of a 32 x 32 row-major matrix S in the permuted contraction
// order: b[s] = sc * S[16 hh + s][jr]
__device__ __forceinline__ void bop32(const float *__restrict__ S, float sc, int hh, int jr, float b[16])
{
#pragma unroll
    for (int s = 0; s < 16; ++s) b[s] = sc * S[(16 * hh + s) * 32 + jr];
}

// the block's waves' 32 x 32 Gram accumulators summed in wave order (double)
// into its slab part[blockIdx.x]
template <int NW>
__device__ __forceinline__ void block_slab32(double (*red)[1024], const f16v_t &g, int lane, int w,
                                             double *__restrict__ part)
{
#pragma unroll
    for (int v = 0; v < 16; ++v) red[w][((v & 3) + 8 * (v >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = (double)g[v];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 64 * NW) {
        double s = 0.0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) s += red[ww][e];
        part[(int64_t)blockIdx.x * 1024 + e] = s;
    }
}

constexpr int kF32Waves = 4;  // 4 waves x 32 rows per unit

// Pass E.  Wprev may alias Wn (row r is read into registers before the same
// wave stores it); P1 == nullptr at j = 0.
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_e32(int64_t n, const float *__restrict__ Y,
                                                              const float *__restrict__ Wj, const float *Wprev,
                                                              float *Wn, const float *__restrict__ binv,
                                                              const float *__restrict__ P1, int64_t lc,
                                                              float *__restrict__ qrow, double *__restrict__ part)
{
    __shared__ double red[kF32Waves][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, jr = lane & 31;
    const bool has_prev = P1 != nullptr;
    float bo[16], po[16];
    bop32(binv, 1.0f, hh, jr, bo);
    if (has_prev) bop32(P1, -1.0f, hh, jr, po);
    f16v_t slab;
#pragma unroll
    for (int v = 0; v < 16; ++v) slab[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * (32 * kF32Waves) + 32 * w;
        const int64_t row = r0 + jr;
        const bool ok = row < n;
        float wa[16], ya[16], pa[16];
        aop32(Wj, row, ok, hh, wa);
        aop32(Y, row, ok, hh, ya);
        if (has_prev) aop32(Wprev, row, ok, hh, pa);
        f16v_t q, wn;
#pragma unroll
        for (int v = 0; v < 16; ++v) q[v] = wn[v] = 0.0f;
#pragma unroll
        for (int s = 0; s < 16; ++s) q = mfma32(wa[s], bo[s], q);     // Q_j = W_j beta^-1
#pragma unroll
        for (int s = 0; s < 16; ++s) wn = mfma32(ya[s], bo[s], wn);   // Y beta^-1
        if (has_prev) {
#pragma unroll
            for (int s = 0; s < 16; ++s) wn = mfma32(pa[s], po[s], wn);  // - W_{j-1} P1
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
            if (rr < n) {
                Wn[rr * 32 + jr] = wn[v];
                if (rr == lc) qrow[jr] = q[v];
            }
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) slab = mfma32(q[v], wn[v], slab);  // Q_j^T W' (rows past n: 0)
    }
    block_slab32<kF32Waves>(red, slab, lane, w, part);
}

// Pass U: Wn <- Wn - Wj P2, slabs of Wn^T Wn.
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_u32(int64_t n, float *__restrict__ Wn,
                                                              const float *__restrict__ Wj,
                                                              const float *__restrict__ P2,
                                                              double *__restrict__ part)
{
    __shared__ double red[kF32Waves][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, jr = lane & 31;
    float bo[16];
    bop32(P2, -1.0f, hh, jr, bo);
    f16v_t g;
#pragma unroll
    for (int v = 0; v < 16; ++v) g[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * (32 * kF32Waves) + 32 * w;
        float wa[16];
        aop32(Wj, r0 + jr, r0 + jr < n, hh, wa);
        f16v_t acc;  // W' in result layout: two 128-B rows per load instruction
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
            acc[v] = rr < n ? Wn[rr * 32 + jr] : 0.0f;
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma32(wa[s], bo[s], acc);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
            if (rr < n) Wn[rr * 32 + jr] = acc[v];
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) g = mfma32(acc[v], acc[v], g);
    }
    block_slab32<kF32Waves>(red, g, lane, w, part);
}

// The beta^2 form of the step (C5; the SpMM's epilogue stores U = W' beta_j =
// A W_j - W_{j-1} beta_{j-1}^-1 G_j, so pass E shrinks to the slabs W_j^T U):
//   pass EL  slabs of W_j^T U                                   (2 n b s, reads only)
//   pass UB  W'' = U beta_j^-1 - W_j P2 (P2 = beta_j^-1 alpha_j), slabs of W''^T W''
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_el32(int64_t n, const float *__restrict__ Wj,
                                                               const float *__restrict__ U,
                                                               double *__restrict__ part)
{
    __shared__ double red[kF32Waves][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, jr = lane & 31;
    f16v_t g;
#pragma unroll
    for (int v = 0; v < 16; ++v) g[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * (32 * kF32Waves) + 32 * w;
        float wv[16], uv[16];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
            // non-temporal (each instruction reads whole 128-B rows): the
            // stream leaves the caches to pass UB's rows (C5 step -1 %,
            // profiles/r05u_c5_el_ub_nt_ab.log)
            wv[v] = rr < n ? __builtin_nontemporal_load(&Wj[rr * 32 + jr]) : 0.0f;
            uv[v] = rr < n ? __builtin_nontemporal_load(&U[rr * 32 + jr]) : 0.0f;
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) g = mfma32(wv[v], uv[v], g);
    }
    block_slab32<kF32Waves>(red, g, lane, w, part);
}

// QO (the solve's last step): also Q = W_j beta^-1 into Qa and (when not
// null) Qb -- the reference's post-call Q0 = Q1 = Q_{m-1} -- from the W_j rows
// the wave already holds; Qa / Qb may alias U / W_j (a unit's rows are loaded
// by the wave that stores them, before it stores them).
template <bool QO>
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_ub32(int64_t n, const float *U, const float *Wj,
                                                               const float *__restrict__ binv,
                                                               const float *__restrict__ P2, float *__restrict__ Wn,
                                                               double *__restrict__ part, float *Qa, float *Qb)
{
    __shared__ double red[kF32Waves][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, jr = lane & 31;
    float bo[16], po[16];
    bop32(binv, 1.0f, hh, jr, bo);
    bop32(P2, -1.0f, hh, jr, po);
    f16v_t g;
#pragma unroll
    for (int v = 0; v < 16; ++v) g[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * (32 * kF32Waves) + 32 * w;
        const int64_t row = r0 + jr;
        const bool ok = row < n;
        float ua[16], wa[16];
        aop32(U, row, ok, hh, ua);
        aop32(Wj, row, ok, hh, wa);
        f16v_t acc, acc2;  // two independent chains (each MFMA waits on its predecessor)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = acc2[v] = 0.0f;
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
            acc = mfma32(ua[s2], bo[s2], acc);    // U beta^-1
            acc2 = mfma32(wa[s2], po[s2], acc2);  // - W_j P2
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] += acc2[v];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
            if (rr < n) Wn[rr * 32 + jr] = acc[v];
        }
        if constexpr (QO) {
            f16v_t q;
#pragma unroll
            for (int v = 0; v < 16; ++v) q[v] = 0.0f;
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) q = mfma32(wa[s2], bo[s2], q);  // W_j beta^-1
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
                if (rr < n) {
                    Qa[rr * 32 + jr] = q[v];
                    if (Qb) Qb[rr * 32 + jr] = q[v];
                }
            }
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) g = mfma32(acc[v], acc[v], g);  // rows past n: 0
    }
    block_slab32<kF32Waves>(red, g, lane, w, part);
}

// Pass UB with coalesced operand loads (round 6; LZ_UB_DMA=0 selects
// k_fused_ub32 above).  aop32 has each lane read its own row's half, so one
// load instruction touches 32 different 128-B lines (32 B of each) and the
// next three touch them again: pass UB moved its 3 n b s at 4.1 TB/s where
// pass EL, whose instructions read whole rows, reached 5.7.  Here each wave
// pulls its 32-row strip of U and of W_j into LDS by LDS-DMA, 16 B per lane,
// 1 KB (8 whole rows) per instruction, one strip ahead of the one it
// computes; each lane's global piece is chosen so the strip lands XOR-swizzled
// (row r's 16-B chunk c at position 8 r + (c ^ (r & 7))), and the MFMA
// A-operands -- a lane's 64 contiguous bytes of its row -- come back as four
// conflict-free ds_read_b128.  The products, their order and the stores are
// k_fused_ub32's, so the results are the same bits.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ub_rsrc(const float *p, int64_t rows)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), (short)0, (int)(rows * 128), 0x00020000);
}

// Store a 32 x 32 fp32 strip held in the MFMA result layout (lane (hh, jr):
// row (v & 3) + 8 (v >> 2) + 4 hh, column jr) as whole rows: through a 4-KB
// LDS slot of the wave's that it no longer reads (sixteen ds_write_b32, row
// rr's chunk c at position 8 rr + (c ^ (rr & 7)) as the DMA layout), back as
// four ds_read_b128 of 8 whole rows each, out as four 16-B stores (1 KB per
// instruction) instead of sixteen 4-B ones.  Rows past the resource's end are
// dropped.  The wave's reads of `slot` must be done before the call (they
// are: their values feed the MFMAs that made `acc`).
template <int AUX>
__device__ __forceinline__ void rstore_slot(float *slot, const f16v_t &acc, int jr, int hh, int lane,
                                            __amdgpu_buffer_rsrc_t nr)
{
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int rr = (v & 3) + 8 * (v >> 2) + 4 * hh;
        slot[rr * 32 + 4 * ((jr >> 2) ^ (rr & 7)) + (jr & 3)] = acc[v];
    }
    const int r8 = lane >> 3, c = lane & 7;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u4v_t x = *reinterpret_cast<const u4v_t *>(&slot[4 * (64 * k + 8 * r8 + (c ^ (r8 & 7)))]);
        __builtin_amdgcn_raw_buffer_store_b128(x, nr, (uint32_t)(1024 * k + 128 * r8 + 16 * c), 0, AUX);
    }
}

template <bool QO>
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_ub32d(int64_t n, const float *U, const float *Wj,
                                                                const float *__restrict__ binv,
                                                                const float *__restrict__ P2, float *__restrict__ Wn,
                                                                double *__restrict__ part, float *Qa, float *Qb,
                                                                int dbg)
{
    // per wave: two slots x (U strip, W_j strip) of 4 KB; the block slab's
    // reduction reuses the same memory after the loop
    __shared__ __attribute__((aligned(16))) float ust[kF32Waves][2][2][1024];
    // w wave-uniform in the compiler's eyes too, so every buffer resource below is
    // scalar (with w = threadIdx.x >> 6 it built them per lane and wrapped each
    // buffer access in a readfirstlane loop)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), hh = lane >> 5,
              jr = lane & 31;
    float bo[16], po[16];
    bop32(binv, 1.0f, hh, jr, bo);
    bop32(P2, -1.0f, hh, jr, po);
    f16v_t g;
#pragma unroll
    for (int v = 0; v < 16; ++v) g[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    const int64_t nst = sch.end > sch.begin ? (sch.end - sch.begin + sch.step - 1) / sch.step : 0;
    // DMA piece of this lane: LDS position 64 k + lane holds row 8 k + lane / 8,
    // chunk (lane & 7) ^ ((lane >> 3) & 7) of the strip
    const uint32_t goff = (uint32_t)((lane >> 3) * 128 + 16 * ((lane & 7) ^ ((lane >> 3) & 7)));
    // this lane's A-operand chunks 4 hh + cc of row jr
    const uint32_t rbase = (uint32_t)(jr * 128);
    auto dma = [&](int64_t s) {
        const int slot = (int)(s & 1);
        const int64_t r0 = (sch.begin + s * sch.step) * (32 * kF32Waves) + 32 * w;
        const int64_t rows = s < nst && r0 < n ? (n - r0 < 32 ? n - r0 : 32) : 0;
        const __amdgpu_buffer_rsrc_t ur = ub_rsrc(U + (rows ? r0 * 32 : 0), rows);
        const __amdgpu_buffer_rsrc_t wr = ub_rsrc(Wj + (rows ? r0 * 32 : 0), rows);
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // rows past the strip's end: out of range, land as zeros
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (ws_lds_t *)&ust[w][slot][0][256 * k], 16, goff + 1024 * k, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (ws_lds_t *)&ust[w][slot][1][256 * k], 16, goff + 1024 * k, 0, 0, 0);
        }
    };
#ifdef LZ_DIAG
    // timing diagnostics (results wrong; diagnostic build only): dbg 16 skips the
    // MFMAs, 32 the DMAs, their waits and the W'' stores
    const bool no_mfma = dbg & 16, no_mem = dbg & 32;
#else
    constexpr bool no_mfma = false, no_mem = false;
#endif
    if (!no_mem) dma(0);
    for (int64_t s = 0; s < nst; ++s) {
        if (!no_mem) dma(s + 1);
        // strip s landed: only strip s + 1's 8 DMAs may still be in flight.  (Not
        // vmcnt(8 + ST) for strip s - 1's ST younger stores: a store can be
        // acknowledged before an older load returns, so that count could be
        // reached with strip s's data still on its way -- the first version
        // read such operands, and round 6 re-checked it: vmcnt(12) with the
        // four row stores of strip s - 1 in flight gave NaN alphas at once,
        // profiles/r06w_ub_wait_ab.log.  Loads return in order, so at most 8
        // left means strip s is in.)
        if (dbg & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (!no_mem) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        const uint32_t sb = ws_lds_addr(reinterpret_cast<int *>(&ust[w][(int)(s & 1)][0][0]));
        float4 u4[4], w4[4];
        const uint32_t o0 = sb + rbase + 16u * (uint32_t)((4 * hh + 0) ^ (jr & 7)),
                       o1 = sb + rbase + 16u * (uint32_t)((4 * hh + 1) ^ (jr & 7)),
                       o2 = sb + rbase + 16u * (uint32_t)((4 * hh + 2) ^ (jr & 7)),
                       o3 = sb + rbase + 16u * (uint32_t)((4 * hh + 3) ^ (jr & 7));
        asm volatile(
            "ds_read_b128 %0, %8\n\t"
            "ds_read_b128 %1, %9\n\t"
            "ds_read_b128 %2, %10\n\t"
            "ds_read_b128 %3, %11\n\t"
            "ds_read_b128 %4, %8 offset:4096\n\t"
            "ds_read_b128 %5, %9 offset:4096\n\t"
            "ds_read_b128 %6, %10 offset:4096\n\t"
            "ds_read_b128 %7, %11 offset:4096\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(u4[0]), "=&v"(u4[1]), "=&v"(u4[2]), "=&v"(u4[3]), "=&v"(w4[0]), "=&v"(w4[1]), "=&v"(w4[2]),
              "=&v"(w4[3])
            : "v"(o0), "v"(o1), "v"(o2), "v"(o3)
            : "memory");
        float ua[16], wa[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            ua[4 * c] = u4[c].x; ua[4 * c + 1] = u4[c].y; ua[4 * c + 2] = u4[c].z; ua[4 * c + 3] = u4[c].w;
            wa[4 * c] = w4[c].x; wa[4 * c + 1] = w4[c].y; wa[4 * c + 2] = w4[c].z; wa[4 * c + 3] = w4[c].w;
        }
        const int64_t r0 = (sch.begin + s * sch.step) * (32 * kF32Waves) + 32 * w;
        f16v_t acc, acc2;  // two independent chains (each MFMA waits on its predecessor)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = acc2[v] = 0.0f;
        if (no_mfma) {
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] = ua[v] - wa[v];
        } else {
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) {
                acc = mfma32(ua[s2], bo[s2], acc);    // U beta^-1
                acc2 = mfma32(wa[s2], po[s2], acc2);  // - W_j P2
            }
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] += acc2[v];
        // (rows past n: out-of-range offsets, no write.  __float_as_uint, not
        // __builtin_bit_cast(uint32_t, acc[v]): hipcc of ROCm 7.2 stored acc[0]
        // sixteen times for the latter in this unrolled loop)
        const __amdgpu_buffer_rsrc_t nr = ub_rsrc(Wn + (r0 < n ? r0 * 32 : 0), r0 < n ? (n - r0 < 32 ? n - r0 : 32) : 0);
        // non-temporal: the next step's SpMM gathers these rows at random (C5:
        // SpMM 2.800 -> 2.787 ms, step 4.133 -> 4.112 ms, profiles/r06i_c5_ub_nt_ab.log)
        if (dbg & 4) {  // (A/B: 4-B stores straight from the result layout)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const uint32_t rr = (uint32_t)((v & 3) + 8 * (v >> 2) + 4 * hh);
                if (dbg & 2) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[v]), nr, rr * 128 + 4 * jr, 0, 0);
                else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[v]), nr, rr * 128 + 4 * jr, 0, 2);
            }
        } else if (no_mem) {
        } else if (dbg & 2) {
            rstore_slot<0>(&ust[w][(int)(s & 1)][0][0], acc, jr, hh, lane, nr);
        } else {
            rstore_slot<2>(&ust[w][(int)(s & 1)][0][0], acc, jr, hh, lane, nr);  // (U strip s: read above)
        }
        if constexpr (QO) {
            f16v_t q;
#pragma unroll
            for (int v = 0; v < 16; ++v) q[v] = 0.0f;
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) q = mfma32(wa[s2], bo[s2], q);  // W_j beta^-1
            const int64_t nrow = r0 < n ? (n - r0 < 32 ? n - r0 : 32) : 0;
            const __amdgpu_buffer_rsrc_t qa = ub_rsrc(Qa + (nrow ? r0 * 32 : 0), nrow);
            const __amdgpu_buffer_rsrc_t qb = ub_rsrc((Qb ? Qb : Qa) + (nrow ? r0 * 32 : 0), Qb ? nrow : 0);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const uint32_t rr = (uint32_t)((v & 3) + 8 * (v >> 2) + 4 * hh);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(q[v]), qa, rr * 128 + 4 * jr, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(q[v]), qb, rr * 128 + 4 * jr, 0, 0);
            }
        }
        if (!no_mfma) {
#pragma unroll
            for (int v = 0; v < 16; ++v) g = mfma32(acc[v], acc[v], g);  // rows past n: 0
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done with its slots: the reduction reuses them
    block_slab32<kF32Waves>(reinterpret_cast<double (*)[1024]>(&ust[0][0][0][0]), g, lane, w, part);
}

// The same staging for the pass-E form's two passes (round 6; LZ_UB_DMA=0
// selects k_fused_e32 / k_fused_u32): every 32 x 32 fp32 operand strip a wave
// reads comes in by LDS-DMA one strip ahead, swizzled as above; A-operands by
// ds_read_b128, result-layout operands (row (v & 3) + 8 (v >> 2) + 4 hh,
// column jr) by ds_read_b32.  The same products in the same order as the
// register forms: the same bits.
__device__ __forceinline__ void dma_strip32(const float *M, int64_t r0, int64_t rows, float *slot, uint32_t goff)
{
    const __amdgpu_buffer_rsrc_t r = ub_rsrc(M + (rows ? r0 * 32 : 0), rows);
#pragma unroll
    for (int k = 0; k < 4; ++k)  // rows past the strip's end: out of range, land as zeros
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (ws_lds_t *)&slot[256 * k], 16, goff + 1024 * k, 0, 0, 0);
}

// a[s] = strip row jr, float 16 hh + s (the MFMA A-operand), from a swizzled slot
__device__ __forceinline__ void aop_slot(uint32_t sb, int jr, int hh, float a[16])
{
    const uint32_t rb = sb + (uint32_t)(jr * 128);
    float4 x[4];
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %5\n\t"
        "ds_read_b128 %2, %6\n\t"
        "ds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
        : "v"(rb + 16u * (uint32_t)((4 * hh + 0) ^ (jr & 7))), "v"(rb + 16u * (uint32_t)((4 * hh + 1) ^ (jr & 7))),
          "v"(rb + 16u * (uint32_t)((4 * hh + 2) ^ (jr & 7))), "v"(rb + 16u * (uint32_t)((4 * hh + 3) ^ (jr & 7)))
        : "memory");
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        a[4 * c] = x[c].x; a[4 * c + 1] = x[c].y; a[4 * c + 2] = x[c].z; a[4 * c + 3] = x[c].w;
    }
}

// r[v] = strip row (v & 3) + 8 (v >> 2) + 4 hh, column jr (the MFMA result
// layout; row rr's chunk jr / 4 sits at position 8 rr + ((jr / 4) ^ (rr & 7))).
// Two asm statements of eight reads and their wait each: the values may be
// used only after the wait, which the compiler cannot see across statements.
__device__ __forceinline__ void rop_slot(uint32_t sb, int jr, int hh, f16v_t &r)
{
    uint32_t a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int rr = (i & 3) + 8 * (i >> 2) + 4 * hh;
        a[i] = sb + (uint32_t)(rr * 128) + 16u * (uint32_t)((jr >> 2) ^ (rr & 7)) + 4u * (uint32_t)(jr & 3);
    }
    float v[16];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
        asm volatile(
            "ds_read_b32 %0, %8\n\t"
            "ds_read_b32 %1, %9\n\t"
            "ds_read_b32 %2, %10\n\t"
            "ds_read_b32 %3, %11\n\t"
            "ds_read_b32 %4, %12\n\t"
            "ds_read_b32 %5, %13\n\t"
            "ds_read_b32 %6, %14\n\t"
            "ds_read_b32 %7, %15\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(v[8 * hf]), "=&v"(v[8 * hf + 1]), "=&v"(v[8 * hf + 2]), "=&v"(v[8 * hf + 3]),
              "=&v"(v[8 * hf + 4]), "=&v"(v[8 * hf + 5]), "=&v"(v[8 * hf + 6]), "=&v"(v[8 * hf + 7])
            : "v"(a[8 * hf]), "v"(a[8 * hf + 1]), "v"(a[8 * hf + 2]), "v"(a[8 * hf + 3]), "v"(a[8 * hf + 4]),
              "v"(a[8 * hf + 5]), "v"(a[8 * hf + 6]), "v"(a[8 * hf + 7])
            : "memory");
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = v[i];
}

// Pass U (DMA form): Wn <- Wn - Wj P2, slabs of Wn^T Wn
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_u32d(int64_t n, float *__restrict__ Wn,
                                                               const float *__restrict__ Wj,
                                                               const float *__restrict__ P2,
                                                               double *__restrict__ part, int dbg)
{
    __shared__ __attribute__((aligned(16))) float ust[kF32Waves][2][2][1024];  // slots x (W_j, Wn) strips
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), hh = lane >> 5,
              jr = lane & 31;
    float bo[16];
    bop32(P2, -1.0f, hh, jr, bo);
    f16v_t g;
#pragma unroll
    for (int v = 0; v < 16; ++v) g[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    const int64_t nst = sch.end > sch.begin ? (sch.end - sch.begin + sch.step - 1) / sch.step : 0;
    const uint32_t goff = (uint32_t)((lane >> 3) * 128 + 16 * ((lane & 7) ^ ((lane >> 3) & 7)));
    auto rows_of = [&](int64_t s, int64_t *r0) {
        *r0 = (sch.begin + s * sch.step) * (32 * kF32Waves) + 32 * w;
        return s < nst && *r0 < n ? (n - *r0 < 32 ? n - *r0 : (int64_t)32) : (int64_t)0;
    };
    auto dma = [&](int64_t s) {
        int64_t r0;
        const int64_t rows = rows_of(s, &r0);
        dma_strip32(Wj, r0, rows, &ust[w][s & 1][0][0], goff);
        dma_strip32(Wn, r0, rows, &ust[w][s & 1][1][0], goff);
    };
    dma(0);
    for (int64_t s = 0; s < nst; ++s) {
        dma(s + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // strip s in (loads return in order)
        const uint32_t sb = ws_lds_addr(reinterpret_cast<int *>(&ust[w][(int)(s & 1)][0][0]));
        float wa[16];
        aop_slot(sb, jr, hh, wa);
        f16v_t acc;  // W' in result layout
        rop_slot(sb + 4096, jr, hh, acc);
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) acc = mfma32(wa[s2], bo[s2], acc);
        int64_t r0;
        const int64_t rows = rows_of(s, &r0);
        const __amdgpu_buffer_rsrc_t nr = ub_rsrc(Wn + (rows ? r0 * 32 : 0), rows);
        if (dbg & 4) {  // (A/B: 4-B stores straight from the result layout)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const uint32_t rr = (uint32_t)((v & 3) + 8 * (v >> 2) + 4 * hh);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[v]), nr, rr * 128 + 4 * jr, 0, 0);
            }
        } else {
            rstore_slot<0>(&ust[w][(int)(s & 1)][1][0], acc, jr, hh, lane, nr);  // (Wn strip s: read above)
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) g = mfma32(acc[v], acc[v], g);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    block_slab32<kF32Waves>(reinterpret_cast<double (*)[1024]>(&ust[0][0][0][0]), g, lane, w, part);
}

// Pass E (DMA form).  Wprev may alias Wn: strip s's rows are in LDS before the
// wave stores them, and the other strips' rows are not its.  One strip slot
// per wave (three operand strips, 12 KB; 2 blocks per CU at 190 registers).
__global__ __launch_bounds__(64 * kF32Waves) void k_fused_e32d(int64_t n, const float *__restrict__ Y,
                                                               const float *__restrict__ Wj, const float *Wprev,
                                                               float *Wn, const float *__restrict__ binv,
                                                               const float *__restrict__ P1, int64_t lc,
                                                               float *__restrict__ qrow, double *__restrict__ part,
                                                               int dbg)
{
    __shared__ __attribute__((aligned(16))) float ust[kF32Waves][3][1024];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), hh = lane >> 5,
              jr = lane & 31;
    const bool has_prev = P1 != nullptr;
    float bo[16], po[16];
    bop32(binv, 1.0f, hh, jr, bo);
    if (has_prev) bop32(P1, -1.0f, hh, jr, po);
    f16v_t slab;
#pragma unroll
    for (int v = 0; v < 16; ++v) slab[v] = 0.0f;
    XcdSched sch(ceil_div(n, (int64_t)(32 * kF32Waves)));
    const uint32_t goff = (uint32_t)((lane >> 3) * 128 + 16 * ((lane & 7) ^ ((lane >> 3) & 7)));
    const uint32_t sb = ws_lds_addr(reinterpret_cast<int *>(&ust[w][0][0]));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * (32 * kF32Waves) + 32 * w;
        const int64_t rows = r0 < n ? (n - r0 < 32 ? n - r0 : (int64_t)32) : (int64_t)0;
        dma_strip32(Wj, r0, rows, &ust[w][0][0], goff);
        dma_strip32(Y, r0, rows, &ust[w][1][0], goff);
        dma_strip32(has_prev ? Wprev : Wj, r0, has_prev ? rows : 0, &ust[w][2][0], goff);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float wa[16], ya[16], pa[16];
        aop_slot(sb, jr, hh, wa);
        aop_slot(sb + 4096, jr, hh, ya);
        if (has_prev) aop_slot(sb + 8192, jr, hh, pa);
        f16v_t q, wn;
#pragma unroll
        for (int v = 0; v < 16; ++v) q[v] = wn[v] = 0.0f;
#pragma unroll
        for (int s = 0; s < 16; ++s) q = mfma32(wa[s], bo[s], q);     // Q_j = W_j beta^-1
#pragma unroll
        for (int s = 0; s < 16; ++s) wn = mfma32(ya[s], bo[s], wn);   // Y beta^-1
        if (has_prev) {
#pragma unroll
            for (int s = 0; s < 16; ++s) wn = mfma32(pa[s], po[s], wn);  // - W_{j-1} P1
        }
        const __amdgpu_buffer_rsrc_t nr = ub_rsrc(Wn + (rows ? r0 * 32 : 0), rows);
        if (dbg & 4) {  // (A/B: 4-B stores straight from the result layout)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int64_t rr = (v & 3) + 8 * (v >> 2) + 4 * hh;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(wn[v]), nr, (uint32_t)(rr * 128 + 4 * jr), 0, 0);
            }
        } else {
            rstore_slot<0>(&ust[w][1][0], wn, jr, hh, lane, nr);  // (the Y strip: read above)
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int64_t rr = (v & 3) + 8 * (v >> 2) + 4 * hh;
            if (r0 + rr == lc && rr < rows) qrow[jr] = q[v];
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) slab = mfma32(q[v], wn[v], slab);  // Q_j^T W' (rows past n: 0)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    block_slab32<kF32Waves>(reinterpret_cast<double (*)[1024]>(&ust[0][0][0]), slab, lane, w, part);
}

// blocks per CU: pass E (190 registers: 2 waves per SIMD) 2; pass U 4.
// Measured at C5 (ms, E / U): grid 1x 1.12 / 0.91, 2x 0.96 / 0.78, 3x 1.20 / 0.78, 4x - / 0.76.
static int f32_grid(lz_handle *h, int64_t n, int mult)
{
    return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)(32 * kF32Waves)), (int64_t)h->n_cu * mult));
}

int fused_e32(lz_handle *h, int64_t n, const float *Y, const float *Wj, const float *Wprev, float *Wn,
              const float *binv, const float *P1, int64_t lc, float *qrow, int *nparts)
{
    const int grid = f32_grid(h, n, 2);
    LZ_TRY(ensure_partials(h, (size_t)grid * 1024));
    const int ev = prof_begin(h, PROF_SPMM_PASS);
    const char *ud = getenv("LZ_UB_DMA");  // "0": the register-operand forms (A/B; read per call)
    if (!(ud && ud[0] == '0'))
        hipLaunchKernelGGL(k_fused_e32d, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, Y, Wj, Wprev, Wn, binv, P1,
                           lc, qrow, h->partials, ud ? atoi(ud) >> 1 : 0);
    else
        hipLaunchKernelGGL(k_fused_e32, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, Y, Wj, Wprev, Wn, binv, P1,
                           lc, qrow, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

int fused_el32(lz_handle *h, int64_t n, const float *Wj, const float *U, int *nparts)
{
    const int grid = f32_grid(h, n, 4);  // 2 / 4 / 8 blocks per CU measured alike
    LZ_TRY(ensure_partials(h, (size_t)grid * 1024));
    const int ev = prof_begin(h, PROF_SPMM_PASS);
    hipLaunchKernelGGL(k_fused_el32, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, Wj, U, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

int fused_ub32(lz_handle *h, int64_t n, const float *U, const float *Wj, const float *binv, const float *P2,
               float *Wn, int *nparts, float *Qa, float *Qb)
{
    // 2 blocks per CU: 4.25 ms per C5 step against 4.40 at 4, 4.37 at 3, 4.38 at 1 and 8
    const int grid = f32_grid(h, n, 2);
    LZ_TRY(ensure_partials(h, (size_t)grid * 1024));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    const char *ud = getenv("LZ_UB_DMA");  // "0": the register-operand form (A/B; read per call)
    const bool dma = !(ud && ud[0] == '0');
    // (A/B: LZ_UB_DMA=3 drains every load before each strip, 5 stores W'' with the default policy,
    // 9 stores it by 4-B stores from the result layout instead of whole rows through LDS; 9 in
    // passes E and U too)
    const int dbg = ud ? atoi(ud) >> 1 : 0;
    if (dma && Qa)
        hipLaunchKernelGGL(k_fused_ub32d<true>, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, U, Wj, binv, P2, Wn,
                           h->partials, Qa, Qb, dbg);
    else if (dma)
        hipLaunchKernelGGL(k_fused_ub32d<false>, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, U, Wj, binv, P2,
                           Wn, h->partials, nullptr, nullptr, dbg);
    else if (Qa)
        hipLaunchKernelGGL(k_fused_ub32<true>, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, U, Wj, binv, P2, Wn,
                           h->partials, Qa, Qb);
    else
        hipLaunchKernelGGL(k_fused_ub32<false>, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, U, Wj, binv, P2,
                           Wn, h->partials, nullptr, nullptr);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

int fused_u32(lz_handle *h, int64_t n, float *Wn, const float *Wj, const float *P2, int *nparts)
{
    const int grid = f32_grid(h, n, 4);
    LZ_TRY(ensure_partials(h, (size_t)grid * 1024));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    const char *ud = getenv("LZ_UB_DMA");  // "0": the register-operand forms (A/B; read per call)
    if (!(ud && ud[0] == '0'))
        hipLaunchKernelGGL(k_fused_u32d, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, Wn, Wj, P2, h->partials,
                           ud ? atoi(ud) >> 1 : 0);
    else
        hipLaunchKernelGGL(k_fused_u32, dim3(grid), dim3(64 * kF32Waves), 0, h->stream, n, Wn, Wj, P2, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

// ---------------------------------------------------------------------------
// Any b <= 32, fp64 or fp32 (VALU): 32-row tiles through LDS in fp64, every
// product accumulated in fp64 and rounded to T once (the MFMA path rounds in
// fp32 at b = 32).  Thread t owns slab entries t, t + 256, ... of the b x b slab.
constexpr int kGenRows = 32;

template <typename T>
__global__ __launch_bounds__(256) void k_fused_e_gen(int64_t n, int b, const T *__restrict__ Y,
                                                     const T *__restrict__ Wj, const T *Wprev, T *Wn,
                                                     const T *__restrict__ binv, const T *__restrict__ P1,
                                                     int64_t lc, T *__restrict__ qrow, double *__restrict__ part)
{
    constexpr int TR = kGenRows, MB = 32;
    __shared__ double sb[MB * MB], sp[MB * MB], tj[TR * MB], ty[TR * MB], tp[TR * MB], tq[TR * MB], tw[TR * MB];
    const int t = threadIdx.x, bb = b * b;
    const bool hp = P1 != nullptr;
    for (int e = t; e < bb; e += 256) {
        sb[e] = (double)binv[e];
        sp[e] = hp ? (double)P1[e] : 0.0;
    }
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    XcdSched sch(ceil_div(n, (int64_t)TR));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * TR;
        const int nr = (int)(n - r0 < TR ? n - r0 : TR), ne = nr * b;
        __syncthreads();  // the previous tile's tq / tw reads are done (and sb, sp written)
        for (int e = t; e < ne; e += 256) {
            tj[e] = (double)Wj[r0 * b + e];
            ty[e] = (double)Y[r0 * b + e];
            tp[e] = hp ? (double)Wprev[r0 * b + e] : 0.0;  // Wprev may be Wn: read before any store
        }
        __syncthreads();
        for (int e = t; e < ne; e += 256) {
            const int r = e / b, c = e - r * b;
            double q = 0.0, w = 0.0;
            for (int k = 0; k < b; ++k) {
                q = fma(tj[r * b + k], sb[k * b + c], q);
                w = fma(ty[r * b + k], sb[k * b + c], w);
            }
            for (int k = 0; hp && k < b; ++k) w = fma(-tp[r * b + k], sp[k * b + c], w);
            const T qT = (T)q, wT = (T)w;
            tq[e] = (double)qT;
            tw[e] = (double)wT;
            Wn[r0 * b + e] = wT;
            if (r0 + r == lc) qrow[c] = qT;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int e = t + 256 * kk;
            if (e < bb) {
                const int i = e / b, j = e - i * b;
                for (int r = 0; r < nr; ++r) acc[kk] = fma(tq[r * b + i], tw[r * b + j], acc[kk]);
            }
        }
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (t + 256 * kk < bb) part[(int64_t)blockIdx.x * bb + t + 256 * kk] = acc[kk];
}

// SWAP (the distributed all-gather form): W'' goes to Wj's rows (the rank's
// slot of the gathered block) and W_j to Wn's (the next step's W_{j-1}); the
// tile's rows of both are staged in LDS before any store.
template <typename T, bool SWAP = false>
__global__ __launch_bounds__(256) void k_fused_u_gen(int64_t n, int b, T *Wn, T *Wj, const T *__restrict__ P2,
                                                     double *__restrict__ part)
{
    constexpr int TR = kGenRows, MB = 32;
    __shared__ double sp[MB * MB], tj[TR * MB], tw[TR * MB];
    const int t = threadIdx.x, bb = b * b;
    for (int e = t; e < bb; e += 256) sp[e] = (double)P2[e];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    XcdSched sch(ceil_div(n, (int64_t)TR));
    for (int64_t u = sch.begin; u < sch.end; u += sch.step) {
        const int64_t r0 = u * TR;
        const int nr = (int)(n - r0 < TR ? n - r0 : TR), ne = nr * b;
        __syncthreads();
        for (int e = t; e < ne; e += 256) {
            tj[e] = (double)Wj[r0 * b + e];
            tw[e] = (double)Wn[r0 * b + e];
        }
        __syncthreads();
        double v[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {  // W'' = W' - Wj P2 (ne <= 1024 = 4 per thread)
            const int e = t + 256 * kk;
            if (e < ne) {
                const int r = e / b, c = e - r * b;
                double x = tw[e];
                for (int k = 0; k < b; ++k) x = fma(-tj[r * b + k], sp[k * b + c], x);
                const T xT = (T)x;
                if constexpr (SWAP) {
                    Wj[r0 * b + e] = xT;
                    Wn[r0 * b + e] = (T)tj[e];
                } else {
                    Wn[r0 * b + e] = xT;
                }
                v[kk] = (double)xT;
            }
        }
        __syncthreads();  // every thread's reads of tw are done
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            if (t + 256 * kk < ne) tw[t + 256 * kk] = v[kk];
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int e = t + 256 * kk;
            if (e < bb) {
                const int i = e / b, j = e - i * b;
                for (int r = 0; r < nr; ++r) acc[kk] = fma(tw[r * b + i], tw[r * b + j], acc[kk]);
            }
        }
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (t + 256 * kk < bb) part[(int64_t)blockIdx.x * bb + t + 256 * kk] = acc[kk];
}

template <typename T>
int fused_e_sep(lz_handle *h, int64_t n, int b, const T *Y, const T *Wj, const T *Wprev, T *Wn, const T *binv,
                const T *P1, int64_t lc, T *qrow, int *nparts)
{
    if constexpr (std::is_same<T, float>::value)
        if (b == 32) return fused_e32(h, n, Y, Wj, Wprev, Wn, binv, P1, lc, qrow, nparts);
    LZ_ARG_CHECK(b >= 1 && b <= 32, "fused pass E: 1 <= b <= 32");
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)kGenRows), (int64_t)h->n_cu * 2));
    LZ_TRY(ensure_partials(h, (size_t)grid * b * b));
    const int ev = prof_begin(h, PROF_SPMM_PASS);
    hipLaunchKernelGGL((k_fused_e_gen<T>), dim3(grid), dim3(256), 0, h->stream, n, b, Y, Wj, Wprev, Wn, binv, P1, lc,
                       qrow, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

template <typename T>
int fused_u_sep(lz_handle *h, int64_t n, int b, T *Wn, const T *Wj, const T *P2, int *nparts)
{
    if constexpr (std::is_same<T, float>::value)
        if (b == 32) return fused_u32(h, n, Wn, Wj, P2, nparts);
    LZ_ARG_CHECK(b >= 1 && b <= 32, "fused pass U: 1 <= b <= 32");
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)kGenRows), (int64_t)h->n_cu * 2));
    LZ_TRY(ensure_partials(h, (size_t)grid * b * b));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    hipLaunchKernelGGL((k_fused_u_gen<T>), dim3(grid), dim3(256), 0, h->stream, n, b, Wn, const_cast<T *>(Wj), P2,
                       h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

template <typename T>
int fused_u_swap_sep(lz_handle *h, int64_t n, int b, T *Wn, T *Xown, const T *P2, int *nparts)
{
    LZ_ARG_CHECK(b >= 1 && b <= 32, "fused pass U (swap): 1 <= b <= 32");
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)kGenRows), (int64_t)h->n_cu * 2));
    LZ_TRY(ensure_partials(h, (size_t)grid * b * b));
    const int ev = prof_begin(h, PROF_UPDATE_PASS);
    hipLaunchKernelGGL((k_fused_u_gen<T, true>), dim3(grid), dim3(256), 0, h->stream, n, b, Wn, Xown, P2, h->partials);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

template int fused_u_swap_sep<double>(lz_handle *, int64_t, int, double *, double *, const double *, int *);
template int fused_u_swap_sep<float>(lz_handle *, int64_t, int, float *, float *, const float *, int *);
template int fused_e_sep<double>(lz_handle *, int64_t, int, const double *, const double *, const double *, double *,
                                 const double *, const double *, int64_t, double *, int *);
template int fused_e_sep<float>(lz_handle *, int64_t, int, const float *, const float *, const float *, float *,
                                const float *, const float *, int64_t, float *, int *);
template int fused_u_sep<double>(lz_handle *, int64_t, int, double *, const double *, const double *, int *);
template int fused_u_sep<float>(lz_handle *, int64_t, int, float *, const float *, const float *, int *);

}  // namespace lz
