// lz_spmm.hip -- CSR sparse x tall-skinny kernels for gfx950.
//
// Replaces the reference's ELL-4 kernels ell::SpMM / ell::SpMV
// (kernels/spmv_spmm.hpp:105-199).  Design (see DESIGN.md "SpMM"):
//   * CSR (int64 row_ptr, int32 col, T val); X / Y row-major n x b, so one
//     gathered X row is b*sizeof(T) contiguous bytes (128 B at b=16 fp64)
//     instead of b scattered 8-B loads of the reference's column-major block.
//   * one "group" of LPR = b*sizeof(T)/16 lanes per row, each lane owning a
//     16-byte slice of the row; the group loads LPR consecutive (col,val) pairs
//     with one coalesced load and broadcasts them inside the group with
//     ds_bpermute, then issues LPR independent 16-B X gathers.
//   * XCD-contiguous grid-stride schedule (lz_kernels.hpp XcdSched) so each
//     XCD's L2 holds a sliding window of X for banded operators.
//   * b == 1 (SpMV): CSR-vector, LV lanes per row with a wave64 xor-shuffle
//     reduction per row.
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

template <typename T, int B>
__global__ __launch_bounds__(256) void k_spmm_rm(int64_t n, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ col,
                                                 const T *__restrict__ val,
                                                 const T *__restrict__ X, int64_t ldx,
                                                 T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB;
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int gbase = (tid & 63) / LPR * LPR;
    XcdSched sch(ceil_div(n, RB));
    // Each group walks its rows (u = begin, begin+step, ...) as one stream of
    // LPR-nnz batches, software-pipelined: the (col,val) pair of the NEXT batch
    // and the row_ptr pair of the NEXT row are loaded while the current
    // batch's X rows are gathered, so the only latency on the critical path is
    // the (mostly L2-resident) X gather.  Control flow is group-uniform.
    int64_t u = sch.begin;
    if (u >= sch.end) return;
    int64_t r = u * RB + gi, k = 0, k1 = 0;
    if (r < n) { k = rp[r]; k1 = rp[r + 1]; }
    int64_t un = u + sch.step, rn = un * RB + gi, kn0 = 0, kn1 = 0;
    if (un < sch.end && rn < n) { kn0 = rp[rn]; kn1 = rp[rn + 1]; }
    int cN = 0;
    T vN = T(0);
    if (k + p < k1) { cN = col[k + p]; vN = val[k + p]; }
    T acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = T(0);
    for (;;) {
        const int c = cN;
        const T v = vN;
        const int64_t rem = k1 - k;
        const int cnt = rem < LPR ? (int)rem : LPR;
        const bool last = rem <= LPR;
        const int64_t rcur = r;
        if (!last) {
            k += LPR;
        } else {  // the next row becomes current; fetch row_ptr of the one after
            u = un; r = rn; k = kn0; k1 = kn1;
            un = u + sch.step;
            rn = un * RB + gi;
            kn0 = kn1 = 0;
            if (un < sch.end && rn < n) { kn0 = rp[rn]; kn1 = rp[rn + 1]; }
        }
        cN = 0;
        vN = T(0);
        if (u < sch.end && k + p < k1) { cN = col[k + p]; vN = val[k + p]; }
        Vec<T, VEC> xs[LPR];
        T vs[LPR];
#pragma unroll
        for (int t = 0; t < LPR; ++t) {
            const int ct = (LPR == 1) ? c : __shfl(c, gbase + t, 64);
            vs[t] = (LPR == 1) ? v : __shfl(v, gbase + t, 64);
            xs[t] = ldv<T, VEC>(X + (int64_t)ct * ldx + p * VEC);
        }
#pragma unroll
        for (int t = 0; t < LPR; ++t) {
            if (t < cnt) {
#pragma unroll
                for (int i = 0; i < VEC; ++i) acc[i] = fma(vs[t], xs[t].v[i], acc[i]);
            }
        }
        if (last) {
            if (rcur < n) {
                Vec<T, VEC> o;
#pragma unroll
                for (int i = 0; i < VEC; ++i) o.v[i] = acc[i];
                stv<T, VEC>(Y + rcur * ldy + p * VEC, o);
            }
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[i] = T(0);
            if (u >= sch.end) break;
        }
    }
}

// Tile-per-block SpMM (the default row-major kernel).  A block owns a tile of
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
                                                  const T *__restrict__ X, int64_t ldx,
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

// LDS-DMA gather variant: the X row slices are gathered straight into a
// per-wave LDS landing zone with global_load_lds_dwordx4 (per-lane source
// address, lane-linear destination: group g's 16-B slices land at g*LPR*16),
// so loads in flight cost no VGPRs; one explicit vmcnt(0) per batch, then each
// lane reads back exactly the 16 bytes it fetched.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <typename T, int B, int CAP, int RPG, int UNR>
__global__ __launch_bounds__(256) void k_spmm_dma(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, TR = RB * RPG;
    if constexpr (VEC * sizeof(T) != 16) {
        return;  // never launched: the DMA variant needs 16-byte lane slices
    } else {
    __shared__ int32_t cs[CAP];
    __shared__ T vs[CAP];
    __shared__ __attribute__((aligned(16))) char land[4][UNR][1024];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    if (t < cnt)
                        __builtin_amdgcn_global_load_lds(
                            (gbl_void_t *)(Xp + (int64_t)cs[base + t] * ldx),
                            (lds_void_t *)&land[w][t][0], 16, 0, 0);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int t = 0; t < UNR; ++t) {
                    if (t < cnt) {
                        const Vec<T, VEC> x = *reinterpret_cast<const Vec<T, VEC> *>(&land[w][t][lane * 16]);
                        const T v = vs[base + t];
#pragma unroll
                        for (int i = 0; i < VEC; ++i) acc[j][i] = fma(v, x.v[i], acc[j][i]);
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
}

// Persistent, queue-scheduled, software-pipelined SpMM (the default).
//
// * Work = tiles of RB rows; tiles are split into 8 contiguous ranges, one per
//   "XCD group" g = blockIdx % 8 (blocks b, b+8, ... share an XCD -- observed,
//   speed only).  Blocks of group g take tiles of range g in order from an
//   atomic counter, so the tiles in flight on one XCD stay a narrow window of
//   rows and a banded operator's X gather stays in that XCD's L2.  Any block
//   may take any tile: results do not depend on placement or timing.
// * Per block and tile: the row_ptr slice of tile t+2 and the (col, val) range
//   of tile t+1 are loaded into registers while tile t is gathered from LDS,
//   so HBM latency of the CSR streams is off the critical path.
// * Gather: one group of LPR lanes per row, 16 B per lane, 8 independent X
//   loads per lane per step; (col, val) come from LDS.
// * Tiles with more than 256*PF nnz (very long rows) are gathered straight
//   from global memory by the same groups (no staging).
constexpr int kQueueGroups = 8;

template <typename T, int B, int PF>
__global__ __launch_bounds__(256) void k_spmm_q(int64_t n, const int64_t *__restrict__ rp,
                                                const int32_t *__restrict__ col,
                                                const T *__restrict__ val,
                                                const T *__restrict__ X, int64_t ldx,
                                                T *__restrict__ Y, int64_t ldy,
                                                unsigned *__restrict__ qctr)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, UNR = 8;
    constexpr int CAPF = 256 * PF;                 // staged nnz per tile
    constexpr int RPS = (RB + 1 + 255) / 256;      // row_ptr values per thread
    __shared__ int32_t cs[CAPF];
    __shared__ T vs[CAPF];
    __shared__ int64_t rps[2][RB + 1];
    __shared__ int64_t s_tile[4];
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int64_t ntiles = ceil_div(n, RB);
    const int grp = blockIdx.x % kQueueGroups;
    const int64_t qbeg = ntiles * grp / kQueueGroups, qend = ntiles * (grp + 1) / kQueueGroups;
    // Thread 0 hands out tiles from tickets of TPT consecutive tiles; the next
    // ticket is claimed (atomicAdd) as soon as the previous one is opened, i.e.
    // TPT tiles before its value is needed, so the atomic's latency is hidden
    // and one counter word sees 1/TPT of the tile rate.  A block stops only
    // when an opened ticket lies past its range: no claimed tile is dropped.
    constexpr int TPT = 4;
    int64_t tk_base = 0, tk_end = 0;
    unsigned pend = 0;
    auto next_tile = [&]() -> int64_t {
        if (tk_base >= tk_end) {
            const int64_t b0 = qbeg + (int64_t)pend * TPT;
            if (b0 >= qend) return -1;
            tk_base = b0;
            tk_end = (b0 + TPT < qend) ? b0 + TPT : qend;
            pend = atomicAdd(&qctr[grp], 1u);
        }
        return tk_base++;
    };
    if (tid == 0) {
        pend = atomicAdd(&qctr[grp], 1u);
        s_tile[0] = next_tile();
        s_tile[1] = s_tile[0] >= 0 ? next_tile() : -1;
        s_tile[2] = s_tile[1] >= 0 ? next_tile() : -1;
    }
    __syncthreads();
    int64_t cur = s_tile[0], nxt = s_tile[1], nn = s_tile[2];
    if (cur < 0) return;  // block-uniform
    // registers of the pipeline: row_ptr slice of `nxt`, (col,val) of `cur`
    int64_t rpr[RPS];
    int32_t cr[PF];
    T vr[PF];
    auto load_rp = [&](int64_t t, int64_t *dst) {
#pragma unroll
        for (int i = 0; i < RPS; ++i) {
            const int idx = tid + 256 * i;
            int64_t r = t * RB + idx;
            if (r > n) r = n;
            dst[i] = (t >= 0 && idx <= RB) ? rp[r] : 0;
        }
    };
    // prologue: rp slice of cur -> LDS, (col,val) of cur -> regs, rp slice of nxt -> regs
    {
        int64_t tmp[RPS];
        load_rp(cur, tmp);
#pragma unroll
        for (int i = 0; i < RPS; ++i)
            if (tid + 256 * i <= RB) rps[0][tid + 256 * i] = tmp[i];
    }
    __syncthreads();
    {
        const int64_t kA = rps[0][0], kB = rps[0][RB];
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int64_t k = kA + tid + 256 * i;
            const bool in = k < kB && (kB - kA) <= CAPF;
            cr[i] = in ? col[k] : 0;
            vr[i] = in ? val[k] : T(0);
        }
    }
    load_rp(nxt, rpr);
    const T *Xp = X + p * VEC;
    int cb = 0;  // which rps buffer holds cur's row_ptr slice (block-local toggle)
    for (;;) {
        const int64_t kA = rps[cb][0], kB = rps[cb][RB];
        const bool staged = (kB - kA) <= CAPF;
        // (a) registers -> LDS: (col,val) of cur, row_ptr slice of nxt
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            cs[tid + 256 * i] = cr[i];
            vs[tid + 256 * i] = vr[i];
        }
        if (nxt >= 0) {
#pragma unroll
            for (int i = 0; i < RPS; ++i)
                if (tid + 256 * i <= RB) rps[cb ^ 1][tid + 256 * i] = rpr[i];
        }
        if (tid == 0) s_tile[3] = (nn >= 0) ? next_tile() : -1;
        __syncthreads();
        const int64_t n3 = s_tile[3];
        // (b) issue the loads of the next stages (in flight during the gather)
        if (nxt >= 0) {
            const int64_t kA2 = rps[cb ^ 1][0], kB2 = rps[cb ^ 1][RB];
#pragma unroll
            for (int i = 0; i < PF; ++i) {
                const int64_t k = kA2 + tid + 256 * i;
                const bool in = k < kB2 && (kB2 - kA2) <= CAPF;
                cr[i] = in ? col[k] : 0;
                vr[i] = in ? val[k] : T(0);
            }
        }
        load_rp(nn, rpr);
        // (c) gather tile cur
        const int64_t row = cur * RB + gi;
        const bool valid = row < n && gi < RB;
        const int64_t k0 = valid ? rps[cb][gi] : 0, k1 = valid ? rps[cb][gi + 1] : 0;
        T acc[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = T(0);
        for (int64_t kb = k0; kb < k1; kb += UNR) {  // group-uniform
            const int cnt = (int)((k1 - kb) < UNR ? (k1 - kb) : UNR);
            Vec<T, VEC> xs[UNR];
            T vv[UNR];
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                const int64_t kk = kb + (t < cnt ? t : 0);
                int c;
                if (staged) {
                    const int li = (int)(kk - kA);
                    c = cs[li];
                    vv[t] = vs[li];
                } else {
                    c = col[kk];
                    vv[t] = val[kk];
                }
                xs[t] = ldv<T, VEC>(Xp + (int64_t)c * ldx);
            }
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                if (t < cnt) {
#pragma unroll
                    for (int i = 0; i < VEC; ++i) acc[i] = fma(vv[t], xs[t].v[i], acc[i]);
                }
            }
        }
        if (valid) {
            Vec<T, VEC> o;
#pragma unroll
            for (int i = 0; i < VEC; ++i) o.v[i] = acc[i];
            stv<T, VEC>(Y + row * ldy + p * VEC, o);
        }
        // (d) advance
        if (nxt < 0) break;  // block-uniform
        __syncthreads();     // LDS reads of cur done before (a) overwrites
        cur = nxt;
        nxt = nn;
        nn = n3;
        cb ^= 1;
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
                          const T *val, const T *X, int64_t ldx, T *Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int CAP = S::RB * 32 < 1024 ? 1024 : (S::RB * 32 > 4096 ? 4096 : S::RB * 32);
    const int64_t units = ceil_div(n, S::RB);
    if (units <= 0) return LZ_OK;
    static const char *variant = getenv("LZ_SPMM_KERNEL");  // "stream" / "tile": A/B only
    const int ev = prof_begin(h, PROF_SPMM);
    if (variant && variant[0] == 's') {
        const int grid = (int)std::min<int64_t>(units, (int64_t)h->n_cu * 8);
        hipLaunchKernelGGL((k_spmm_rm<T, B>), dim3(grid), dim3(256), 0, h->stream, n, rp, col,
                           val, X, ldx, Y, ldy);
    } else if (variant && variant[0] == 'q') {
        // persistent queue kernel: grid = resident blocks, 8 queue counters reset per call
        LZ_HIP_TRY(hipMemsetAsync(h->qctr, 0, 64 * sizeof(unsigned), h->stream));
        const int per_cu = h->spmm_blocks_per_cu;
        const int grid = (int)std::max<int64_t>(8, std::min<int64_t>(units, (int64_t)h->n_cu * per_cu));
        hipLaunchKernelGGL((k_spmm_q<T, B, 4>), dim3(grid), dim3(256), 0, h->stream, n, rp, col,
                           val, X, ldx, Y, ldy, h->qctr);
    } else if (variant && variant[0] == 'd' && S::VEC * sizeof(T) == 16) {
        // LDS-DMA gather; LZ_SPMM_KERNEL=d<rpg><unr>, e.g. d28, d24, d18
        const int rpg = variant[1] == '1' ? 1 : 2;
        const int unr = variant[2] == '4' ? 4 : 8;
        const int64_t tiles = ceil_div(n, (int64_t)S::RB * rpg);
        LZ_ARG_CHECK(tiles < (1LL << 31), "too many row tiles");
        constexpr int CAP2 = CAP * 2 < 4096 ? CAP * 2 : 4096;
        if (rpg == 1 && unr == 8)
            hipLaunchKernelGGL((k_spmm_dma<T, B, CAP, 1, 8>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
        else if (rpg == 2 && unr == 8)
            hipLaunchKernelGGL((k_spmm_dma<T, B, CAP2, 2, 8>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
        else if (rpg == 1)
            hipLaunchKernelGGL((k_spmm_dma<T, B, CAP, 1, 4>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_dma<T, B, CAP2, 2, 4>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
    } else {
        static const char *rpg_env = getenv("LZ_SPMM_RPG");
        const int rpg = rpg_env ? atoi(rpg_env) : 2;
        const int64_t tiles = ceil_div(n, (int64_t)S::RB * rpg);
        LZ_ARG_CHECK(tiles < (1LL << 31), "too many row tiles");
        if (rpg == 1)
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP, 1>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
        else if (rpg == 2)
            hipLaunchKernelGGL((k_spmm_lds<T, B, CAP * 2 < 4096 ? CAP * 2 : 4096, 2>),
                               dim3((unsigned)tiles), dim3(256), 0, h->stream, n, rp, col, val, X,
                               ldx, Y, ldy);
        else
            hipLaunchKernelGGL((k_spmm_lds<T, B, 4096, 4>), dim3((unsigned)tiles), dim3(256), 0,
                               h->stream, n, rp, col, val, X, ldx, Y, ldy);
    }
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

template <typename T>
int spmm_rm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, T *Y, int64_t ldy)
{
    switch (b) {
    case 1: return spmv<T>(h, n, rp, col, val, X, Y, 0);
    case 2: return launch_spmm_rm<T, 2>(h, n, rp, col, val, X, ldx, Y, ldy);
    case 4: return launch_spmm_rm<T, 4>(h, n, rp, col, val, X, ldx, Y, ldy);
    case 8: return launch_spmm_rm<T, 8>(h, n, rp, col, val, X, ldx, Y, ldy);
    case 16: return launch_spmm_rm<T, 16>(h, n, rp, col, val, X, ldx, Y, ldy);
    case 32: return launch_spmm_rm<T, 32>(h, n, rp, col, val, X, ldx, Y, ldy);
    case 64: return launch_spmm_rm<T, 64>(h, n, rp, col, val, X, ldx, Y, ldy);
    default:
        set_error("row-major SpMM supports b in {1,2,4,8,16,32,64}, got %d", b);
        return LZ_E_ARG;
    }
}

template <typename T>
int spmm_cm(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const T *val, int b,
            const T *X, int64_t ldx, T *Y, int64_t ldy)
{
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
                             const double *, int, const double *, int64_t, double *, int64_t);
template int spmm_rm<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, float *, int64_t);
template int spmm_cm<double>(lz_handle *, int64_t, const int64_t *, const int32_t *,
                             const double *, int, const double *, int64_t, double *, int64_t);
template int spmm_cm<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                            int, const float *, int64_t, float *, int64_t);
template int spmv<double>(lz_handle *, int64_t, const int64_t *, const int32_t *, const double *,
                          const double *, double *, int64_t);
template int spmv<float>(lz_handle *, int64_t, const int64_t *, const int32_t *, const float *,
                         const float *, float *, int64_t);

}  // namespace lz
