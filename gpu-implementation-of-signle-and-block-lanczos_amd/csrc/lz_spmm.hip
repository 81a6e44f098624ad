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

// Tile-per-block SpMM (the default row-major kernel).  A block owns RB
// consecutive rows (one group of LPR lanes per row): it stages the tile's
// (col, val) range into LDS with coalesced loads, then every group gathers its
// row's X rows 8 nnz at a time (8 independent 16-byte loads per lane in
// flight), reading (col, val) from LDS.  One tile per block with the XCD remap
// keeps each XCD's in-flight tiles contiguous (L2-resident X window).  Tiles
// with more than CAP nnz are staged in CAP-sized chunks.
template <typename T, int B, int CAP>
__global__ __launch_bounds__(256) void k_spmm_lds(int64_t n, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ col,
                                                  const T *__restrict__ val,
                                                  const T *__restrict__ X, int64_t ldx,
                                                  T *__restrict__ Y, int64_t ldy)
{
    using S = SpmmShape<T, B>;
    constexpr int VEC = S::VEC, LPR = S::LPR, RB = S::RB, UNR = 8;
    __shared__ int32_t cs[CAP];
    __shared__ T vs[CAP];
    const int tid = threadIdx.x;
    const int gi = tid / LPR, p = tid % LPR;
    const int64_t r0 = xcd_remap(blockIdx.x, gridDim.x) * RB;
    const int64_t rend = (r0 + RB < n) ? r0 + RB : n;
    const int64_t kA = rp[r0], kB = rp[rend];
    const int64_t row = r0 + gi;
    const bool valid = row < n;
    const int64_t k0 = valid ? rp[row] : kB, k1 = valid ? rp[row + 1] : kB;
    const T *Xp = X + p * VEC;
    T acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = T(0);
    for (int64_t c0 = kA; c0 < kB; c0 += CAP) {  // block-uniform
        const int64_t c1 = (c0 + CAP < kB) ? c0 + CAP : kB;
        if (c0 != kA) __syncthreads();
        for (int64_t k = c0 + tid; k < c1; k += 256) {
            cs[k - c0] = col[k];
            vs[k - c0] = val[k];
        }
        __syncthreads();
        const int64_t a = k0 > c0 ? k0 : c0, e = k1 < c1 ? k1 : c1;
        for (int64_t kb = a; kb < e; kb += UNR) {  // group-uniform
            const int cnt = (int)((e - kb) < UNR ? (e - kb) : UNR);
            const int base = (int)(kb - c0);
            Vec<T, VEC> xs[UNR];
            T vv[UNR];
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                const int li = base + (t < cnt ? t : 0);
                vv[t] = vs[li];
                xs[t] = ldv<T, VEC>(Xp + (int64_t)cs[li] * ldx);
            }
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                if (t < cnt) {
#pragma unroll
                    for (int i = 0; i < VEC; ++i) acc[i] = fma(vv[t], xs[t].v[i], acc[i]);
                }
            }
        }
    }
    if (valid) {
        Vec<T, VEC> o;
#pragma unroll
        for (int i = 0; i < VEC; ++i) o.v[i] = acc[i];
        stv<T, VEC>(Y + row * ldy + p * VEC, o);
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
    static const char *variant = getenv("LZ_SPMM_KERNEL");  // "stream": A/B only
    const int ev = prof_begin(h, PROF_SPMM);
    if (variant && variant[0] == 's') {
        const int grid = (int)std::min<int64_t>(units, (int64_t)h->n_cu * 8);
        hipLaunchKernelGGL((k_spmm_rm<T, B>), dim3(grid), dim3(256), 0, h->stream, n, rp, col,
                           val, X, ldx, Y, ldy);
    } else {
        LZ_ARG_CHECK(units < (1LL << 31), "too many row tiles");
        hipLaunchKernelGGL((k_spmm_lds<T, B, CAP>), dim3((unsigned)units), dim3(256), 0, h->stream,
                           n, rp, col, val, X, ldx, Y, ldy);
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
