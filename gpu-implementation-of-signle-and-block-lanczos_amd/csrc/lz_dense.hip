// lz_dense.hip -- tall-skinny block-orthogonalisation kernels for gfx950.
//
// Replaces the reference's cuBLAS/cuSOLVER calls of block_lanczos_blas
// (utils/lib_utils.hpp:28-202,649-745) and its hand-written float kernels
// tt::mm_tt, tt2::mm_tt2, ts::mm_ts*, sqrtm::My_sqrtm_cusolver
// (kernels/mm_tt.hpp, mm_tt2.hpp, mm_ts.hpp, my_sqrtm_cusolver.hpp).
//
// Layout: n x b row-major blocks.  For b = 16 fp64 the products run on the
// f64 matrix cores (v_mfma_f64_16x16x4_f64):
//   * Gram X^T Y: a 4-row chunk of a row-major block is exactly 64 contiguous
//     doubles, and "lane l holds element l" is both MFMA operand layouts when
//     the contraction runs over rows -- one coalesced 8-B load per operand.
//   * Q*S: the contraction runs over columns, so each wave transposes a
//     16x16 tile through a private LDS tile (row stride 17 doubles, conflict
//     free for ds_read_b64) and the MFMA result lands in the row-major chunk
//     layout again, so W is read/written with coalesced 8-B accesses.
// Other (b, dtype): portable LDS-tiled VALU kernels.
// Every reduction is a fixed-order two-stage reduction (per-workgroup slabs,
// then one workgroup) -- bitwise reproducible run to run, no float atomics.
#include "lz_common.hpp"
#include "lz_internal.hpp"
#include "lz_kernels.hpp"
#include "lz_sqrtm.hpp"

namespace lz {

// ============================================================== Gram slabs
// b = 16 Gram slabs on v_mfma_f64_16x16x4f64; T = double or float (fp32 blocks
// are widened on load and accumulated in fp64, as every other fp32 reduction here).
// fp32 b = 16 Gram slabs: a lane loads 16 B (4 columns of one row), so one
// wave-instruction brings a whole 16-row tile (4x fewer loads than one element
// per lane); the tile goes through the wave's LDS and comes back in MFMA operand
// order.  MFMA step st contracts over rows {4k + st}: lane l supplies row
// 4 (l >> 4) + st, column l & 15, for both operands.  fp64 accumulation.
template <bool SAME>
__global__ __launch_bounds__(512) void k_gram16_f32(int64_t n, const float *__restrict__ X,
                                                    const float *__restrict__ Y,
                                                    double *__restrict__ part)
{
    constexpr int U = 4;  // tiles in flight per wave
    __shared__ float tx[8][U][256];
    __shared__ float ty[SAME ? 1 : 8][U][256];
    __shared__ double red[8][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ntl = ceil_div(n, 16);
    XcdSched s(ceil_div(ntl, 8));
    d4_t acc = {0.0, 0.0, 0.0, 0.0};
    const float4 zero = {0.f, 0.f, 0.f, 0.f};
    for (int64_t u = s.begin; u < s.end; u += U * s.step) {
        float4 xv[U], yv[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int64_t uu = u + t * s.step;
            const int64_t row = (uu * 8 + w) * 16 + (lane >> 2);
            const bool ok = uu < s.end && row < n;
            xv[t] = ok ? *reinterpret_cast<const float4 *>(X + row * 16 + 4 * (lane & 3)) : zero;
            if constexpr (!SAME) yv[t] = ok ? *reinterpret_cast<const float4 *>(Y + row * 16 + 4 * (lane & 3)) : zero;
        }
#pragma unroll
        for (int t = 0; t < U; ++t) {
            *reinterpret_cast<float4 *>(&tx[w][t][4 * lane]) = xv[t];
            if constexpr (!SAME) *reinterpret_cast<float4 *>(&ty[w][t][4 * lane]) = yv[t];
        }
        wave_lds_sync();
#pragma unroll
        for (int t = 0; t < U; ++t)
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int e = (4 * (lane >> 4) + st) * 16 + (lane & 15);
                const double a = (double)tx[w][t][e];
                const double b = SAME ? a : (double)ty[w][t][e];
                acc = mfma16(a, b, acc);
            }
        wave_lds_sync();
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
    __syncthreads();
    if (threadIdx.x < 256) {
        double sum = 0.0;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) sum += red[ww][threadIdx.x];
        part[(int64_t)blockIdx.x * 256 + threadIdx.x] = sum;
    }
}

template <typename T, bool SAME>
__global__ __launch_bounds__(512) void k_gram16_f64(int64_t n, const T *__restrict__ X,
                                                    const T *__restrict__ Y,
                                                    double *__restrict__ part)
{
    __shared__ double red[8][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t nel = n * 16;
    const int64_t nch = ceil_div(n, 4);
    XcdSched s(ceil_div(nch, 8));
    d4_t acc = {0.0, 0.0, 0.0, 0.0};
    constexpr int U = 8;
    for (int64_t u = s.begin; u < s.end; u += U * s.step) {
        double xa[U], ya[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int64_t uu = u + t * s.step;
            const int64_t e = (uu * 8 + w) * 64 + lane;
            const bool ok = (uu < s.end) && (e < nel);
            xa[t] = ok ? (double)X[e] : 0.0;
            ya[t] = SAME ? xa[t] : (ok ? (double)Y[e] : 0.0);
        }
#pragma unroll
        for (int t = 0; t < U; ++t) acc = mfma16(xa[t], ya[t], acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
    __syncthreads();
    if (threadIdx.x < 256) {
        double sum = 0.0;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) sum += red[ww][threadIdx.x];
        part[(int64_t)blockIdx.x * 256 + threadIdx.x] = sum;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_gram_gen(int64_t n, int b, const T *__restrict__ X,
                                                  const T *__restrict__ Y, int64_t ld,
                                                  double *__restrict__ part)
{
    constexpr int TR = 16;
    __shared__ double xs[TR * kMaxB], ys[TR * kMaxB];
    const int bb = b * b, tid = threadIdx.x;
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.0;
    XcdSched s(ceil_div(n, TR));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        for (int e = tid; e < TR * b; e += 256) {
            const int r = e / b, c = e % b;
            const int64_t row = u * TR + r;
            xs[e] = row < n ? (double)X[row * ld + c] : 0.0;
            ys[e] = row < n ? (double)Y[row * ld + c] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int e = tid + 256 * k;
            if (e < bb) {
                const int i = e / b, j = e % b;
                double a = acc[k];
                for (int r = 0; r < TR; ++r) a = fma(xs[r * b + i], ys[r * b + j], a);
                acc[k] = a;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int e = tid + 256 * k;
        if (e < bb) part[(int64_t)blockIdx.x * bb + e] = acc[k];
    }
}

// Fixed-order reduction of P slabs of bb doubles by a 1024-thread workgroup:
// for bb <= 1024 each entry gets G = 1024/bb threads, thread g summing slabs
// g, g+G, ... with four independent accumulators (loads in flight), then the
// G partial sums are added in order g = 0..G-1.  Deterministic for a given
// (P, bb).  Result in out[bb] (LDS); all threads must call it.
constexpr int kRedThreads = 1024;
__device__ void reduce_slabs(const double *__restrict__ part, int P, int bb, double *out,
                             double *scratch)
{
    const int t = threadIdx.x;
    if (bb <= kRedThreads) {
        const int G = kRedThreads / bb;
        const int e = t % bb, g = t / bb;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        if (g < G) {
            int p = g;
            for (; p + 3 * G < P; p += 4 * G) {
                s0 += part[(int64_t)p * bb + e];
                s1 += part[(int64_t)(p + G) * bb + e];
                s2 += part[(int64_t)(p + 2 * G) * bb + e];
                s3 += part[(int64_t)(p + 3 * G) * bb + e];
            }
            for (; p < P; p += G) s0 += part[(int64_t)p * bb + e];
        }
        scratch[t] = (s0 + s1) + (s2 + s3);
        __syncthreads();
        if (t < bb) {
            double s = 0.0;
            for (int gg = 0; gg < G; ++gg) s += scratch[gg * bb + t];
            out[t] = s;
        }
    } else {
        for (int e = t; e < bb; e += kRedThreads) {
            double s = 0.0;
            for (int p = 0; p < P; ++p) s += part[(int64_t)p * bb + e];
            out[e] = s;
        }
    }
    __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(kRedThreads) void k_gram_finish(int b, const double *__restrict__ part,
                                                             int P, int mode, T *__restrict__ R,
                                                             const T *__restrict__ L, T *__restrict__ LR)
{
    __shared__ double g[kMaxB * kMaxB];
    __shared__ double r[kMaxB * kMaxB];
    __shared__ double scratch[kRedThreads];
    const int bb = b * b;
    reduce_slabs(part, P, bb, g, scratch);
    for (int e = threadIdx.x; e < bb; e += kRedThreads) {
        const int i = e / b, j = e % b;
        const double v = mode ? 0.5 * (g[i * b + j] + g[j * b + i]) : g[e];
        R[e] = (T)v;
        r[e] = (double)(T)v;
    }
    if (L) {  // LR = L * R (the Q-free iteration's P2 = beta_j^-1 alpha_j)
        __syncthreads();
        for (int e = threadIdx.x; e < bb; e += kRedThreads) {
            const int i = e / b, j = e % b;
            double s = 0.0;
            for (int k = 0; k < b; ++k) s = fma((double)L[i * b + k], r[k * b + j], s);
            LR[e] = (T)s;
        }
    }
}

// C5 beta^2 step (b = 32, fp32 storage, fp64 arithmetic), one workgroup each:
// k_alpha_b2  X = sum slabs (W_j^T U), Z = beta^-1 X beta^-1, alpha = (Z + Z^T)/2,
//             P2 = beta^-1 alpha, row probe q_j = W_j[lc] beta^-1
// k_m_b2      G = sum slabs (W''^T W''), M = beta^-1 G (the next SpMM's epilogue)
__global__ __launch_bounds__(kRedThreads) void k_alpha_b2(const double *__restrict__ part, int P,
                                                          const float *__restrict__ binv, float *__restrict__ alpha,
                                                          float *__restrict__ P2, const float *__restrict__ Wj,
                                                          int64_t lc_row, float *__restrict__ qrow)
{
    constexpr int B = 32, BB = B * B;
    __shared__ double x[BB], bi[BB], t1[BB];
    __shared__ double scratch[kRedThreads];
    const int t = threadIdx.x;
    reduce_slabs(part, P, BB, x, scratch);
    bi[t] = (double)binv[t];
    __syncthreads();
    const int i = t / B, j = t % B;
    double s = 0.0;  // t1 = beta^-1 X
    for (int k = 0; k < B; ++k) s = fma(bi[i * B + k], x[k * B + j], s);
    t1[t] = s;
    __syncthreads();
    s = 0.0;  // Z = t1 beta^-1
    for (int k = 0; k < B; ++k) s = fma(t1[i * B + k], bi[k * B + j], s);
    x[t] = s;  // each thread reads only t1 and bi here
    __syncthreads();
    const float a = (float)(0.5 * (x[i * B + j] + x[j * B + i]));
    __syncthreads();
    alpha[t] = a;
    t1[t] = (double)a;
    __syncthreads();
    s = 0.0;  // P2 = beta^-1 alpha
    for (int k = 0; k < B; ++k) s = fma(bi[i * B + k], t1[k * B + j], s);
    P2[t] = (float)s;
    if (lc_row >= 0 && t < B) {
        double q = 0.0;
        for (int k = 0; k < B; ++k) q = fma((double)Wj[lc_row * B + k], bi[k * B + t], q);
        qrow[t] = (float)q;
    }
}

__global__ __launch_bounds__(kRedThreads) void k_m_b2(const double *__restrict__ part, int P,
                                                      const float *__restrict__ binv, float *__restrict__ M)
{
    constexpr int B = 32, BB = B * B;
    __shared__ double g[BB], bi[BB];
    __shared__ double scratch[kRedThreads];
    const int t = threadIdx.x;
    reduce_slabs(part, P, BB, g, scratch);
    bi[t] = (double)binv[t];
    __syncthreads();
    const int i = t / B, j = t % B;
    double s = 0.0;
    for (int k = 0; k < B; ++k) s = fma(bi[i * B + k], g[k * B + j], s);
    M[t] = (float)s;
}

int alpha_b2(lz_handle *h, const double *part, int P, const float *binv, float *alpha, float *P2, const float *Wj,
             int64_t lc, int64_t n, float *qrow)
{
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_alpha_b2, dim3(1), dim3(kRedThreads), 0, h->stream, part, P, binv, alpha, P2, Wj,
                       (lc >= 0 && lc < n) ? lc : (int64_t)-1, qrow);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// Wavefront step (lz_wf.hip), b = 16 fp64: S1 = sum of P slabs (V^T Y), S2 =
// sum of the next P (V^T V_prev); X = S1 binv - S2 P1 (P1 null: S1 binv),
// alpha = sym(binv X), P2 = binv alpha, q = V[lc] binv.  (alpha_j = Q_j^T W' =
// beta_j^-1 V_j^T (Y beta_j^-1 - V_{j-1} P1_j), methods/block_lanczos.hpp:155.)
__global__ __launch_bounds__(kRedThreads) void k_alpha_wf16(const double *__restrict__ part, int P,
                                                            const double *__restrict__ binv,
                                                            const double *__restrict__ P1, double *__restrict__ alpha,
                                                            double *__restrict__ P2, const double *__restrict__ V,
                                                            int64_t lc_row, double *__restrict__ qrow)
{
    constexpr int B = 16, BB = 256;
    __shared__ double s1[BB], s2[BB], bi[BB], x[BB];
    __shared__ double scratch[kRedThreads];
    const int t = threadIdx.x;
    reduce_slabs(part, P, BB, s1, scratch);
    if (P1) reduce_slabs(part + (int64_t)P * BB, P, BB, s2, scratch);
    if (t < BB) bi[t] = binv[t];
    __syncthreads();
    const int i = (t & 255) / B, j = t % B;
    if (t < BB) {
        double s = 0.0;
        for (int k = 0; k < B; ++k) s = fma(s1[i * B + k], bi[k * B + j], s);
        if (P1)
            for (int k = 0; k < B; ++k) s = fma(-s2[i * B + k], P1[k * B + j], s);
        x[t] = s;
    }
    __syncthreads();
    double z = 0.0;
    if (t < BB)
        for (int k = 0; k < B; ++k) z = fma(bi[i * B + k], x[k * B + j], z);
    __syncthreads();
    if (t < BB) s1[t] = z;  // Z = binv X
    __syncthreads();
    if (t < BB) {
        const double a = 0.5 * (s1[i * B + j] + s1[j * B + i]);
        alpha[t] = a;
        x[t] = a;
    }
    __syncthreads();
    if (t < BB) {
        double s = 0.0;
        for (int k = 0; k < B; ++k) s = fma(bi[i * B + k], x[k * B + j], s);
        P2[t] = s;
    }
    if (lc_row >= 0 && t < B) {
        double q = 0.0;
        for (int k = 0; k < B; ++k) q = fma(V[lc_row * B + k], bi[k * B + t], q);
        qrow[t] = q;
    }
}

int alpha_wf16(lz_handle *h, const double *part, int P, const double *binv, const double *P1, double *alpha,
               double *P2, const double *V, int64_t lc, int64_t n, double *qrow)
{
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_alpha_wf16, dim3(1), dim3(kRedThreads), 0, h->stream, part, P, binv, P1, alpha, P2, V,
                       (lc >= 0 && lc < n) ? lc : (int64_t)-1, qrow);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

int m_b2(lz_handle *h, const double *part, int P, const float *binv, float *M)
{
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_m_b2, dim3(1), dim3(kRedThreads), 0, h->stream, part, P, binv, M);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ------------------------------------------ b = 32 fp32 on v_mfma_f32_32x32x2_f32
// (BASELINE config 5: block 32, fp32).  Lane l of a 32x32x2 MFMA supplies
// A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]; C/D element (row
// (v&3) + 8(v>>2) + 4(l>>5), col l&31) sits in register v of lane l.
typedef float f16v_t __attribute__((ext_vector_type(16)));

// G = X^T Y: k runs over rows, two per instruction; each wave walks 16-row
// chunks, one accumulator (the 32x32x2 issue interval equals its dependent
// latency, 64 cycles); per-block slabs of 32 x 32 doubles.
template <bool SYM>
__global__ __launch_bounds__(256) void k_gram32_f32(int64_t n, const float *__restrict__ X,
                                                    const float *__restrict__ Y, double *__restrict__ part)
{
    __shared__ double red[4][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    f16v_t acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.0f;
    XcdSched s(ceil_div(n, (int64_t)64));  // 64-row units: 16 rows per wave
    // four units' loads in flight before their MFMAs (one unit at a time, a
    // wave held 2 KB in flight: 0.386 -> 0.313 ms for C5's 10M x 32; eight
    // units measured the same, profiles/r05zd_c5_kernel_stats.csv); the MFMAs run in
    // the same unit order as before
    constexpr int UU = 4;
    for (int64_t u0 = s.begin; u0 < s.end; u0 += UU * s.step) {
        float a[UU][8], bq[UU][8];
#pragma unroll
        for (int uu = 0; uu < UU; ++uu) {
            const int64_t u = u0 + uu * s.step;
            const int64_t r0 = u * 64 + 16 * w;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int64_t row = r0 + 2 * t + (lane >> 5);
                const bool ok = u < s.end && row < n;
                a[uu][t] = ok ? X[row * 32 + (lane & 31)] : 0.0f;
                if constexpr (!SYM) bq[uu][t] = ok ? Y[row * 32 + (lane & 31)] : 0.0f;
            }
        }
#pragma unroll
        for (int uu = 0; uu < UU; ++uu)
#pragma unroll
            for (int t = 0; t < 8; ++t)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[uu][t], SYM ? a[uu][t] : bq[uu][t], acc, 0, 0, 0);
    }
#pragma unroll
    for (int v = 0; v < 16; ++v)
        red[w][((v & 3) + 8 * (v >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = (double)acc[v];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 256)
        part[(int64_t)blockIdx.x * 1024 + e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
}

template <typename T>
int gram_partials(lz_handle *h, int64_t n, int b, const T *X, const T *Y, int64_t ld, int *nparts)
{
    LZ_ARG_CHECK(b >= 1 && b <= kMaxB, "b out of range");
    if (b == 16 && ld == 16) {  // fp64 and fp32
        const bool f32 = std::is_same<T, float>::value;
        const int64_t units = f32 ? ceil_div(ceil_div(n, 16), 8) : ceil_div(ceil_div(n, 4), 8);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, f32 ? h->n_cu * 2 : h->n_cu));
        const int ev_ = prof_begin(h, PROF_GRAM);
        if constexpr (std::is_same<T, float>::value) {
            if (X == Y)
                hipLaunchKernelGGL((k_gram16_f32<true>), dim3(grid), dim3(512), 0, h->stream, n, X, Y, h->partials);
            else
                hipLaunchKernelGGL((k_gram16_f32<false>), dim3(grid), dim3(512), 0, h->stream, n, X, Y, h->partials);
        } else if (X == Y) {
            hipLaunchKernelGGL((k_gram16_f64<T, true>), dim3(grid), dim3(512), 0, h->stream, n, X, Y, h->partials);
        } else {
            hipLaunchKernelGGL((k_gram16_f64<T, false>), dim3(grid), dim3(512), 0, h->stream, n, X, Y, h->partials);
        }
        prof_end(h, ev_);
        LZ_LAUNCH_CHECK();
        *nparts = grid;
        return LZ_OK;
    }
    if constexpr (std::is_same<T, float>::value) {
        if (b == 32 && ld == 32) {
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)64), h->n_cu * 2));
            LZ_TRY(ensure_partials(h, (size_t)grid * 1024));
            const int ev_ = prof_begin(h, PROF_GRAM);
            if (X == Y)
                hipLaunchKernelGGL(k_gram32_f32<true>, dim3(grid), dim3(256), 0, h->stream, n, X, Y, h->partials);
            else
                hipLaunchKernelGGL(k_gram32_f32<false>, dim3(grid), dim3(256), 0, h->stream, n, X, Y, h->partials);
            prof_end(h, ev_);
            LZ_LAUNCH_CHECK();
            *nparts = grid;
            return LZ_OK;
        }
    }
    const int64_t units = ceil_div(n, 16);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, (int64_t)h->n_cu * 2));
    {
    const int ev_ = prof_begin(h, PROF_GRAM);
    hipLaunchKernelGGL((k_gram_gen<T>), dim3(grid), dim3(256), 0, h->stream, n, b, X, Y, ld,
                       h->partials);
    prof_end(h, ev_);
    }
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

template <typename T>
int gram_finish(lz_handle *h, int b, int nparts, int mode, T *R, const double *slabs, const T *L, T *LR)
{
    {
    const int ev_ = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL((k_gram_finish<T>), dim3(1), dim3(kRedThreads), 0, h->stream, b,
                       slabs ? slabs : h->partials, nparts, mode, R, L, LR);
    prof_end(h, ev_);
    }
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ============================================================ sqrtm (Jacobi)
// One workgroup.  All 1024 threads reduce the Gram slabs; then waves 1..15 exit
// and wave 0 alone runs a parallel (round-robin ordered) cyclic Jacobi on the
// b x b symmetric matrix in LDS: each round applies b/2 disjoint rotations at
// once, every element of A' = J^T A J and V' = V J computed from the previous
// buffers (ping-pong; a one-wave barrier is nearly free).  Then
// beta = V sqrt|L| V^T and beta_inv = V |L|^-1/2 V^T as custom_mult2
// (utils/lib_utils.hpp:649-694), which takes |lambda| exactly like this.
template <typename T>
__global__ __launch_bounds__(kRedThreads) void k_sqrtm(int b, const T *__restrict__ Gin,
                                                       const double *__restrict__ part, int P,
                                                       T *__restrict__ beta, T *__restrict__ binv,
                                                       T *__restrict__ eig, const T *__restrict__ L,
                                                       T *__restrict__ LB)
{
    constexpr int MB = 32;
    __shared__ double Abuf[2][MB * MB], Vbuf[2][MB * MB];
    __shared__ double cc[MB], ss[MB];
    __shared__ int partner[MB];
    __shared__ double scratch[kRedThreads];
    const int tid = threadIdx.x, bb = b * b;
    double *A = Abuf[0], *An = Abuf[1], *V = Vbuf[0], *Vn = Vbuf[1];
    if (P > 0) {
        reduce_slabs(part, P, bb, An, scratch);
    } else {
        for (int e = tid; e < bb; e += kRedThreads) An[e] = (double)Gin[e];
        __syncthreads();
    }
    if (tid >= 64) return;  // the rest is one wave: s_barrier waits only for it
    constexpr int NT = 64;
    // symmetrise from the lower triangle (syevj with CUBLAS_FILL_MODE_LOWER)
    for (int e = tid; e < bb; e += NT) {
        const int i = e / b, j = e % b;
        A[e] = (i < j) ? An[j * b + i] : An[e];
        V[e] = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
    const int bo = b + (b & 1);  // even player count (index b = bye when b odd)
    for (int sweep = 0; sweep < 40; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int e = tid; e < bb; e += NT) {
            const double a2 = A[e] * A[e];
            tot += a2;
            if (e / b != e % b) off += a2;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            off += __shfl_xor(off, o, 64);
            tot += __shfl_xor(tot, o, 64);
        }
        if (!(off > 1e-300 + 1e-32 * tot)) break;  // wave-uniform
        for (int rnd = 0; rnd < bo - 1; ++rnd) {
            if (tid < bo / 2) {
                // circle method: position 0 fixed, others rotate
                auto at = [&](int pos) { return pos == 0 ? 0 : 1 + (pos - 1 + rnd) % (bo - 1); };
                int p = at(tid), q = at(bo - 1 - tid);
                if (p > q) { const int t = p; p = q; q = t; }
                if (q < b) {
                    const double apq = A[p * b + q];
                    double c = 1.0, s = 0.0;
                    if (apq != 0.0) {
                        const double tau = (A[q * b + q] - A[p * b + p]) / (2.0 * apq);
                        const double t = (tau >= 0.0 ? 1.0 : -1.0) /
                                         (fabs(tau) + sqrt(1.0 + tau * tau));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = t * c;
                    }
                    partner[p] = q; cc[p] = c; ss[p] = -s;
                    partner[q] = p; cc[q] = c; ss[q] = s;
                } else if (p < b) {
                    partner[p] = p; cc[p] = 1.0; ss[p] = 0.0;
                }
            }
            __syncthreads();
            for (int e = tid; e < bb; e += NT) {
                const int i = e / b, j = e % b;
                const int ip = partner[i], jp = partner[j];
                const double ai = cc[i], bi = (ip == i) ? 0.0 : ss[i];
                const double aj = cc[j], bj = (jp == j) ? 0.0 : ss[j];
                double v = ai * aj * A[i * b + j];
                if (bj != 0.0) v += ai * bj * A[i * b + jp];
                if (bi != 0.0) v += bi * aj * A[ip * b + j];
                if (bi != 0.0 && bj != 0.0) v += bi * bj * A[ip * b + jp];
                if ((jp == i && ip == j && i != j)) v = 0.0;  // annihilated pair
                An[e] = v;
                double vv = aj * V[i * b + j];
                if (bj != 0.0) vv += bj * V[i * b + jp];
                Vn[e] = vv;
            }
            __syncthreads();
            double *t = A; A = An; An = t;
            t = V; V = Vn; Vn = t;
        }
    }
    // beta = V f(L) V^T
    for (int e = tid; e < bb; e += NT) {
        const int i = e / b, j = e % b;
        double s1 = 0.0, s2 = 0.0;
        for (int k = 0; k < b; ++k) {
            const double l = fabs(A[k * b + k]);
            const double sq = sqrt(l);
            const double vv = V[i * b + k] * V[j * b + k];
            s1 += vv * sq;
            s2 += vv * (1.0 / sq);
        }
        if (beta) beta[e] = (T)s1;
        if (binv) binv[e] = (T)s2;
        if (L) An[e] = s1;  // An is dead: park beta for LB
    }
    if (L) {  // LB = L * beta (the Q-free iteration's P1 = beta_{j-1}^-1 beta_j)
        __syncthreads();
        for (int e = tid; e < bb; e += NT) {
            const int i = e / b, j = e % b;
            double s = 0.0;
            for (int k = 0; k < b; ++k) s = fma((double)L[i * b + k], An[k * b + j], s);
            LB[e] = (T)s;
        }
    }
    if (eig && tid < b) {
        const double lk = A[tid * b + tid];
        int rank = 0;
        for (int k = 0; k < b; ++k) {
            const double lm = A[k * b + k];
            rank += (lm < lk) || (lm == lk && k < tid);
        }
        eig[rank] = (T)lk;
    }
}

// Compile-time-B variant (B = 8, 16, 32).  After the slab reduction one wave
// runs the same round-robin (circle method) parallel Jacobi, restructured so
// that a round is short straight-line code: A and U = V^T are kept in
// "position space" -- the entry of index x lives at its round-robin position,
// so the pairs of every round are the fixed positions (p, B-1-p), and after
// each round the rows and columns are written back moved one position along
// the circle (position 0 fixed, pos -> pos-1, 1 -> B-1).  Every LDS address a
// lane touches is then the same in every round; after B-1 rounds (one sweep)
// positions coincide with indices again, so the convergence test and the
// result see the matrix in index order.  Lane t owns the position-space
// entries (t / B + (64/B) k, t % B).  Per round: lanes p < B/2 compute and
// publish the rotation of (p, B-1-p) (one sqrt, one division, a refined rsq),
// then every lane forms A' = R A R^T and U' = R U from four A and two U reads
// and writes them to the other buffer at the moved positions.  The products
// are ordered so that A' stays bit-symmetric (contraction off).  Rotations
// below the relative threshold a_pq^2 <= eps^2 |a_pp a_qq| are skipped and the
// sweeps stop once no pair exceeds it (high relative accuracy for the small
// eigenvalues of a nearly rank-deficient W'^T W').
#ifdef LZ_SQRTM_PROBE
__device__ long long lz_sqrtm_probe[2];  // sweeps, Jacobi clock cycles (scripts/probe)
#endif

template <typename T, int B>
__global__ __launch_bounds__(kRedThreads) void k_sqrtm_b(const T *__restrict__ Gin,
                                                         const double *__restrict__ part, int P,
                                                         T *__restrict__ beta, T *__restrict__ binv,
                                                         T *__restrict__ eig, const T *__restrict__ L,
                                                         T *__restrict__ LB, WfAlpha wa, int ns)
{
#pragma clang fp contract(off)
    static_assert(B == 8 || B == 16 || B == 32, "B in {8, 16, 32}");
    constexpr int BB = B * B, LD = B + 1, NE = BB / 64, RS = 64 / B;
    constexpr int UN = B >= 32 ? 2 : NE;
    constexpr double kTol2 = 2.220446049250313e-16 * 2.220446049250313e-16;
    __shared__ double g[BB];
    __shared__ double scratch[kRedThreads];
    __shared__ double Abuf[2][B * LD], Ubuf[2][B * LD];
    __shared__ double cc[B], ss[B];
    // the wavefront step's alpha kernel folded in (B = 16, wa.part != null):
    // its slabs reduced by the whole block up front, the products at the end
    constexpr int WB = B == 16 ? BB : 1;
    __shared__ double ws1[WB], ws2[WB], wbi[WB], wp1[WB];
    const bool wfa = B == 16 && wa.part != nullptr;
    const int tid = threadIdx.x;
    if (P > 0) {
        reduce_slabs(part, P, BB, g, scratch);
    } else {
        for (int e = tid; e < BB; e += kRedThreads) g[e] = (double)Gin[e];
        __syncthreads();
    }
    if (wfa) {
        reduce_slabs(wa.part, wa.P, BB, ws1, scratch);
        if (L) reduce_slabs(wa.part + (int64_t)wa.P * BB, wa.P, BB, ws2, scratch);
    }
    if constexpr (B == 32) {
        // Newton-Schulz on the MFMA by four waves (sqrtm_ns32) when no
        // eigenvalues are asked for and G is well enough conditioned; the
        // whole workgroup takes part (its barriers), then the one-wave Jacobi
        // route otherwise.  (Abuf / Ubuf: 4 x 32 x 33 doubles of scratch.)
        if (ns && eig == nullptr) {
            double sc = 0.0;
            const bool ok = sqrtm_ns32(g, Abuf[0], Abuf[1], Ubuf[0], scratch, sc, tid);
            if (ok) {
                sqrtm_ns32_tail<T>(Abuf[0], Abuf[1], sc, g, beta, binv, L, LB, tid);
                return;
            }
            __syncthreads();  // the scratch is the Jacobi route's matrices
        }
    }
    if (tid >= 64) return;  // one wave from here on
    const int j = tid % B, r0 = tid / B;  // column, first row of this lane
    const int jq = B - 1 - j;                      // partner position of j
    const int jn = j == 0 ? 0 : (j == 1 ? B - 1 : j - 1);  // moved position of j
    double *Am = Abuf[0], *An = Abuf[1], *Um = Ubuf[0], *Un = Ubuf[1];
    bool done = false;
    if constexpr (B == 16) {
        // Newton-Schulz on the MFMA when no eigenvalues are asked for and G is
        // well enough conditioned (sqrtm_ns16); the Jacobi route otherwise
        if (ns && eig == nullptr) {
            double ya[4], yb[4], za[4], zb[4], sc = 0.0;
            if (sqrtm_ns16(g, Abuf[0], Abuf[1], Ubuf[0], ya, yb, za, zb, sc, tid)) {
                sqrtm_ns16_tail<T>(ya, yb, za, zb, sc, g, beta, binv, L, LB, wfa ? wbi : nullptr,
                                   wfa ? wp1 : nullptr, tid);
                done = true;
            }
            wave_lds_sync();  // the scratch (Abuf, Ubuf) is the Jacobi route's matrices
        }
    }
    if (!done) {
    sqrtm_init<B>(g, Am, Um, tid);  // symmetrised from the lower triangle, U = I
#ifdef LZ_SQRTM_PROBE
    const long long t0 = clock64();
    int nsw = 0;
#endif
    if constexpr (B == 16 || B == 32) {
#ifdef LZ_SQRTM_PROBE
        nsw = jacobi_rr<B>(Am, Um, tid);
#else
        (void)jacobi_rr<B>(Am, Um, tid);
#endif
        (void)An;
        (void)Un;
        (void)jn;
        (void)jq;
    } else {
        for (int sweep = 0; sweep < 60; ++sweep) {
    #ifdef LZ_SQRTM_PROBE
            nsw = sweep;
    #endif
            // converged when no off-diagonal entry exceeds the rotation threshold
            bool need = false;
            const double djj = fabs(Am[j * LD + j]);
    #pragma unroll UN
            for (int k = 0; k < NE; ++k) {
                const int i = r0 + RS * k;
                const double aij = Am[i * LD + j];
                if (i != j && aij != 0.0 && aij * aij > kTol2 * (fabs(Am[i * LD + i]) * djj)) need = true;
            }
            if (__ballot(need) == 0) break;  // wave-uniform
    #pragma unroll 1
            for (int rnd = 0; rnd < B - 1; ++rnd) {
                if (tid < B / 2) {
                    const int p = tid, q = B - 1 - tid;
                    double c, s;
                    jacobi_rot(Am[p * LD + p], Am[q * LD + q], Am[p * LD + q], c, s);
                    cc[p] = c;
                    cc[q] = c;
                    ss[p] = -s;  // R[p][q]
                    ss[q] = s;   // R[q][p]
                }
                wave_lds_sync();
                const double cj = cc[j], sj = ss[j];
                for (int k0 = 0; k0 < NE; k0 += UN) {
                    double v[UN][6], ci[UN], si[UN];
    #pragma unroll
                    for (int kk = 0; kk < UN; ++kk) {  // all reads of the chunk first
                        const int i = r0 + RS * (k0 + kk), iq = B - 1 - i;
                        ci[kk] = cc[i];
                        si[kk] = ss[i];
                        v[kk][0] = Am[i * LD + j];
                        v[kk][1] = Am[i * LD + jq];
                        v[kk][2] = Am[iq * LD + j];
                        v[kk][3] = Am[iq * LD + jq];
                        v[kk][4] = Um[i * LD + j];
                        v[kk][5] = Um[iq * LD + j];
                    }
    #pragma unroll
                    for (int kk = 0; kk < UN; ++kk) {
                        const int i = r0 + RS * (k0 + kk);
                        const int in = i == 0 ? 0 : (i == 1 ? B - 1 : i - 1);
                        const double x1 = v[kk][0] * (ci[kk] * cj), x2 = v[kk][1] * (ci[kk] * sj);
                        const double x3 = v[kk][2] * (si[kk] * cj), x4 = v[kk][3] * (si[kk] * sj);
                        const bool ann = (i == jq) && si[kk] != 0.0;  // the annihilated pair
                        An[in * LD + jn] = ann ? 0.0 : (x1 + x4) + (x2 + x3);
                        Un[in * LD + j] = v[kk][4] * ci[kk] + v[kk][5] * si[kk];
                    }
                }
                {
                    double *t = Am; Am = An; An = t;
                    t = Um; Um = Un; Un = t;
                }
                wave_lds_sync();
            }
        }
    }
#ifdef LZ_SQRTM_PROBE
    if (tid == 0) {
        lz_sqrtm_probe[0] = nsw;
        lz_sqrtm_probe[1] = clock64() - t0;
    }
#endif
    sqrtm_tail<T, B>(Am, Um, cc, ss, g, beta, binv, L, LB, wfa ? wbi : nullptr, wfa ? wp1 : nullptr, tid);
    if (eig && tid < B) {
        const double lk = Am[tid * LD + tid];
        int rank = 0;
        for (int k = 0; k < B; ++k) {
            const double lm = Am[k * LD + k];
            rank += (lm < lk) || (lm == lk && k < tid);
        }
        eig[rank] = (T)lk;
    }
    }  // !done
    if constexpr (B == 16) {
        if (wfa) {  // k_alpha_wf16's products, same order (one wave)
            wave_lds_sync();
            double x[NE];
#pragma unroll
            for (int k = 0; k < NE; ++k) {  // X = S1 binv - S2 P1
                const int i = r0 + RS * k;
                double s = 0.0;
                for (int kk = 0; kk < B; ++kk) s = fma(ws1[i * B + kk], wbi[kk * B + j], s);
                if (L)
                    for (int kk = 0; kk < B; ++kk) s = fma(-ws2[i * B + kk], wp1[kk * B + j], s);
                x[k] = s;
            }
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < NE; ++k) ws2[(r0 + RS * k) * B + j] = x[k];
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < NE; ++k) {  // Z = binv X
                const int i = r0 + RS * k;
                double z = 0.0;
                for (int kk = 0; kk < B; ++kk) z = fma(wbi[i * B + kk], ws2[kk * B + j], z);
                x[k] = z;
            }
#pragma unroll
            for (int k = 0; k < NE; ++k) ws1[(r0 + RS * k) * B + j] = x[k];
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < NE; ++k) {  // alpha = sym(Z)
                const int i = r0 + RS * k;
                x[k] = 0.5 * (ws1[i * B + j] + ws1[j * B + i]);
            }
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const int i = r0 + RS * k;
                wa.alpha[i * B + j] = x[k];
                ws2[i * B + j] = x[k];
            }
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < NE; ++k) {  // P2 = binv alpha
                const int i = r0 + RS * k;
                double s = 0.0;
                for (int kk = 0; kk < B; ++kk) s = fma(wbi[i * B + kk], ws2[kk * B + j], s);
                wa.P2[i * B + j] = s;
            }
            if (wa.lc >= 0 && tid < B) {
                double q = 0.0;
                for (int kk = 0; kk < B; ++kk) q = fma(wa.V[wa.lc * B + kk], wbi[kk * B + tid], q);
                wa.qrow[tid] = q;
            }
        }
    }
}

template <typename T>
int sqrtm_pair(lz_handle *h, int b, const T *G, int nparts, T *beta, T *beta_inv, T *eig,
               const double *slabs, const T *L, T *LB, const WfAlpha *wa)
{
    LZ_ARG_CHECK(b >= 1 && b <= 32, "sqrtm supports b <= 32");
    LZ_ARG_CHECK(!wa || (b == 16 && beta_inv), "the folded alpha products need b = 16 and beta_inv");
    {
    const int ev_ = prof_begin(h, PROF_SMALL);
    const double *sl = slabs ? slabs : h->partials;
    const char *nse = getenv("LZ_SQRTM_NS");  // "0": the Jacobi route at b = 16 and 32 as well (A/B, tests)
    const int ns = (nse && nse[0] == '0') ? 0 : 1;
#define LZ_SQRTM_B(BV)                                                                        \
    case BV:                                                                                  \
        hipLaunchKernelGGL((k_sqrtm_b<T, BV>), dim3(1), dim3(kRedThreads), 0, h->stream, G, sl, \
                           nparts, beta, beta_inv, eig, L, LB, wa ? *wa : WfAlpha{}, ns);      \
        break;
    switch (b) {
        LZ_SQRTM_B(8) LZ_SQRTM_B(16) LZ_SQRTM_B(32)
    default:
        hipLaunchKernelGGL((k_sqrtm<T>), dim3(1), dim3(kRedThreads), 0, h->stream, b, G, sl,
                           nparts, beta, beta_inv, eig, L, LB);
    }
#undef LZ_SQRTM_B
    prof_end(h, ev_);
    }
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ==================================================================== Q * S
// W = sw W + sq Q S at b = 16 on v_mfma_f64_16x16x4f64; T = double or float
// (fp32 operands widened on load, the result rounded once on store).
template <typename T>
__global__ __launch_bounds__(512) void k_tsmm16_f64(int64_t n, double sw, double sq,
                                                    const T *__restrict__ Q,
                                                    const T *__restrict__ S,
                                                    T *__restrict__ W)
{
    __shared__ double tile[8][16 * 17];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double *tl = tile[w];
    double sb[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) sb[kc] = sq * (double)S[(4 * kc + (lane >> 4)) * 16 + (lane & 15)];
    const int64_t ntile = ceil_div(n, 16);
    XcdSched s(ceil_div(ntile, 8));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        const int64_t r0 = (u * 8 + w) * 16;
        if (r0 >= n) continue;  // wave-uniform
        const int64_t qrow = r0 + (lane >> 2);
        double qv[4] = {0.0, 0.0, 0.0, 0.0};
        if (qrow < n) {
            if constexpr (std::is_same<T, double>::value) {
                const double2 *src = reinterpret_cast<const double2 *>(Q + qrow * 16 + 4 * (lane & 3));
                const double2 a = src[0], b2 = src[1];
                qv[0] = a.x; qv[1] = a.y; qv[2] = b2.x; qv[3] = b2.y;
            } else {
                const float4 a = *reinterpret_cast<const float4 *>(Q + qrow * 16 + 4 * (lane & 3));
                qv[0] = a.x; qv[1] = a.y; qv[2] = a.z; qv[3] = a.w;
            }
        }
        d4_t acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + (lane >> 4) + 4 * r;
            acc[r] = (sw != 0.0 && row < n) ? sw * (double)W[r0 * 16 + 64 * r + lane] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) tl[(lane >> 2) * 17 + 4 * (lane & 3) + i] = qv[i];
        wave_lds_sync();
        double a[4];
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) a[kc] = tl[(lane & 15) * 17 + 4 * kc + (lane >> 4)];
        wave_lds_sync();
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) acc = mfma16(a[kc], sb[kc], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + (lane >> 4) + 4 * r;
            if (row < n) W[r0 * 16 + 64 * r + lane] = (T)acc[r];
        }
    }
}

// W = sw*W + sq*(Q S), computed transposed: D = S^T Q^T, so lane l's 16
// accumulator registers are row l&31 of the 32-row tile, columns
// 8g + 4(l>>5) + 0..3 in registers 4g..4g+3 -- four 16-B loads / stores per
// lane.  The contraction is permuted (k = 16(l>>5) + s at step s) so the Q
// operand of a lane is 64 contiguous bytes of its row (four 16-B loads).
__global__ __launch_bounds__(256) void k_tsmm32_f32(int64_t n, float sw, float sq, const float *__restrict__ Q,
                                                    const float *__restrict__ S, float *__restrict__ W)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, jr = lane & 31;
    float sa[16];  // A[i = jr][k = 16 hh + s] = S[k][jr]
#pragma unroll
    for (int st = 0; st < 16; ++st) sa[st] = S[(16 * hh + st) * 32 + jr];
    XcdSched s(ceil_div(n, (int64_t)128));  // 128-row units: 32 rows per wave
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        const int64_t row = u * 128 + 32 * w + jr;
        const bool ok = row < n;
        float qb[16];
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ok) x = *reinterpret_cast<const float4 *>(Q + row * 32 + 16 * hh + 4 * c4);
            qb[4 * c4] = x.x; qb[4 * c4 + 1] = x.y; qb[4 * c4 + 2] = x.z; qb[4 * c4 + 3] = x.w;
        }
        float4 wo[4];
        if (sw != 0.0f) {
#pragma unroll
            for (int g = 0; g < 4; ++g)
                wo[g] = ok ? *reinterpret_cast<const float4 *>(W + row * 32 + 8 * g + 4 * hh)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        f16v_t acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = 0.0f;
#pragma unroll
        for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sa[st], qb[st], acc, 0, 0, 0);
        if (ok) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float4 o;
                if (sw != 0.0f) {
                    o.x = fmaf(sw, wo[g].x, sq * acc[4 * g]);
                    o.y = fmaf(sw, wo[g].y, sq * acc[4 * g + 1]);
                    o.z = fmaf(sw, wo[g].z, sq * acc[4 * g + 2]);
                    o.w = fmaf(sw, wo[g].w, sq * acc[4 * g + 3]);
                } else {
                    o = make_float4(sq * acc[4 * g], sq * acc[4 * g + 1], sq * acc[4 * g + 2], sq * acc[4 * g + 3]);
                }
                *reinterpret_cast<float4 *>(W + row * 32 + 8 * g + 4 * hh) = o;
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_tsmm_gen(int64_t n, int b, T sw, T sq,
                                                  const T *__restrict__ Q, const T *__restrict__ S,
                                                  T *__restrict__ W, int64_t ld)
{
    constexpr int TR = 16;
    __shared__ T ssm[kMaxB * kMaxB];
    __shared__ T qs[TR * kMaxB];
    const int tid = threadIdx.x;
    for (int e = tid; e < b * b; e += 256) ssm[e] = S[e];
    XcdSched s(ceil_div(n, TR));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        __syncthreads();
        for (int e = tid; e < TR * b; e += 256) {
            const int r = e / b, c = e % b;
            const int64_t row = u * TR + r;
            qs[e] = row < n ? Q[row * ld + c] : T(0);
        }
        __syncthreads();
        for (int e = tid; e < TR * b; e += 256) {
            const int r = e / b, j = e % b;
            const int64_t row = u * TR + r;
            if (row >= n) continue;
            T acc = T(0);
            for (int i = 0; i < b; ++i) acc = fma(qs[r * b + i], ssm[i * b + j], acc);
            T *wp = W + row * ld + j;
            *wp = (sw == T(0)) ? sq * acc : fma(sw, *wp, sq * acc);
        }
    }
}

template <typename T>
int tsmm(lz_handle *h, int64_t n, int b, T sw, T sq, const T *Q, const T *S, T *W, int64_t ld)
{
    LZ_ARG_CHECK(b >= 1 && b <= kMaxB && ld >= b, "tsmm shape");
    if (n <= 0) return LZ_OK;
    if (b == 16 && ld == 16) {  // fp64 and fp32
        const int64_t units = ceil_div(ceil_div(n, 16), 8);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, h->n_cu * 2));
        const int ev_ = prof_begin(h, PROF_TSMM);
        hipLaunchKernelGGL((k_tsmm16_f64<T>), dim3(grid), dim3(512), 0, h->stream, n, (double)sw, (double)sq, Q, S,
                           W);
        prof_end(h, ev_);
        LZ_LAUNCH_CHECK();
        return LZ_OK;
    }
    if constexpr (std::is_same<T, float>::value) {
        if (b == 32 && ld == 32) {
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, (int64_t)128), h->n_cu * 4));
            const int ev_ = prof_begin(h, PROF_TSMM);
            hipLaunchKernelGGL(k_tsmm32_f32, dim3(grid), dim3(256), 0, h->stream, n, sw, sq, Q, S, W);
            prof_end(h, ev_);
            LZ_LAUNCH_CHECK();
            return LZ_OK;
        }
    }
    const int64_t units = ceil_div(n, 16);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(units, (int64_t)h->n_cu * 4));
    {
    const int ev_ = prof_begin(h, PROF_TSMM);
    hipLaunchKernelGGL((k_tsmm_gen<T>), dim3(grid), dim3(256), 0, h->stream, n, b, sw, sq, Q, S, W,
                       ld);
    prof_end(h, ev_);
    }
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ============================================================ final state
// The state block_lanczos_blas leaves behind (methods/block_lanczos.hpp:145,
// 159, 162): Q0 = Q1 = Q_{m-1} and W = the last residual W_m.  The Q-free steps
// never store Q, so one row-local pass after the last step makes them:
//   Q = Vq binv                              into Q0 and (Q1 != null) Q1;
//   W = Y binv - Vp P1 - Vq P2  (Y != null; the wavefront form, Vp may be null)
//     or W = Wm (copied unless Wm == Wout).
// Inputs and outputs may alias (every buffer is row-local: a tile's rows are
// staged in LDS before any of them is written).  b <= 32.
template <typename T>
__global__ __launch_bounds__(256) void k_final_state(int64_t n, int b, const T *Y, const T *Vp, const T *Vq,
                                                     const T *Wm, const T *__restrict__ binv,
                                                     const T *__restrict__ P1, const T *__restrict__ P2, T *Wout,
                                                     T *Q0, T *Q1)
{
    constexpr int TR = 16, MB = 32;
    __shared__ T mb[3][MB * MB];
    __shared__ T rs[3][TR * MB];  // the tile's Vq, then Y / Vp (or Wm) rows
    const int tid = threadIdx.x, bb = b * b;
    for (int e = tid; e < bb; e += 256) {
        mb[0][e] = binv[e];
        mb[1][e] = P1 ? P1[e] : T(0);
        mb[2][e] = P2 ? P2[e] : T(0);
    }
    XcdSched s(ceil_div(n, TR));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        const int64_t r0 = u * TR;
        const int nr = (int)(n - r0 < TR ? n - r0 : TR), ne = nr * b;
        __syncthreads();  // the previous tile's rows are no longer read
        for (int e = tid; e < ne; e += 256) {
            const int64_t g = r0 * b + e;
            rs[0][e] = Vq[g];
            rs[1][e] = Y ? Y[g] : Wm[g];
            rs[2][e] = Vp ? Vp[g] : T(0);
        }
        __syncthreads();  // every row of the tile read before any is written
        for (int e = tid; e < ne; e += 256) {
            const int r = e / b, j = e % b;
            const T *vq = &rs[0][r * b], *y = &rs[1][r * b], *vp = &rs[2][r * b];
            T q = T(0), a = T(0), c = T(0), d = T(0);
            for (int i = 0; i < b; ++i) {
                q = fma(vq[i], mb[0][i * b + j], q);
                a = fma(y[i], mb[0][i * b + j], a);
                c = fma(vp[i], mb[1][i * b + j], c);
                d = fma(vq[i], mb[2][i * b + j], d);
            }
            const int64_t g = r0 * b + e;
            if (Y) Wout[g] = (a - c) - d;
            else if (Wm != Wout) Wout[g] = y[j];
            Q0[g] = q;
            if (Q1) Q1[g] = q;
        }
    }
}

// The post-call state when W is already the last residual (Y == null: the
// two-pass and separate-SpMM paths): Q = Vq beta^-1 into Q0 (and Q1), W <- Wm
// when they differ.  Thread (column j, row group) keeps column j of beta^-1 in
// registers and reads each staged row as LDS broadcasts: B multiply-adds per
// output (the general kernel above also formed the three Y-path sums and read
// every matrix entry from LDS: 4.7 ms for C5's 10M x 32 block).  Same products
// in the same order as k_final_state's q.
template <typename T, int B>
__global__ __launch_bounds__(256) void k_final_q(int64_t n, const T *Vq, const T *Wm, const T *__restrict__ binv,
                                                 T *Wout, T *Q0, T *Q1)
{
    constexpr int TR = 64, RG = 256 / B;
    __shared__ T rs[TR * B];
    const int tid = threadIdx.x, j = tid % B, rg = tid / B;
    T mcol[B];
#pragma unroll
    for (int i = 0; i < B; ++i) mcol[i] = binv[i * B + j];
    const bool copyw = Wm != nullptr && Wm != Wout;
    XcdSched s(ceil_div(n, TR));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        const int64_t r0 = u * TR;
        const int nr = (int)(n - r0 < TR ? n - r0 : TR), ne = nr * B;
        __syncthreads();  // the previous tile's rows are no longer read
        for (int e = tid; e < ne; e += 256) rs[e] = Vq[r0 * B + e];
        // (element e is staged and copied by the same thread: a W aliasing Vq is read first)
        if (copyw)
            for (int e = tid; e < ne; e += 256) Wout[r0 * B + e] = Wm[r0 * B + e];
        __syncthreads();  // every row staged (and W copied) before any Q row is written
        for (int r = rg; r < nr; r += RG) {
            T q = T(0);
#pragma unroll
            for (int i = 0; i < B; ++i) q = fma(rs[r * B + i], mcol[i], q);
            const int64_t g = (r0 + r) * B + j;
            Q0[g] = q;
            if (Q1) Q1[g] = q;
        }
    }
}

// b = 16 fp64: thread (column j = t & 15, row group t >> 4) keeps column j of
// binv, P1, P2 in registers and walks 4 of the tile's 64 rows; a row's values
// are LDS broadcasts (16-B reads).  Same products and order as k_final_state.
__global__ __launch_bounds__(256) void k_final_state16(int64_t n, const double *Y, const double *Vp, const double *Vq,
                                                      const double *Wm, const double *__restrict__ binv,
                                                      const double *__restrict__ P1, const double *__restrict__ P2,
                                                      double *Wout, double *Q0, double *Q1)
{
    constexpr int TR = 64;
    __shared__ double2 rs[3][TR * 8];  // the tile's Vq, Y (or Wm), Vp rows
    const int tid = threadIdx.x, j = tid & 15, rg = tid >> 4;
    double mb[16], m1[16], m2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        mb[i] = binv[i * 16 + j];
        m1[i] = P1 ? P1[i * 16 + j] : 0.0;
        m2[i] = P2 ? P2[i * 16 + j] : 0.0;
    }
    const double2 *vq2 = reinterpret_cast<const double2 *>(Vq), *y2 = reinterpret_cast<const double2 *>(Y ? Y : Wm),
                  *vp2 = reinterpret_cast<const double2 *>(Vp);
    XcdSched s(ceil_div(n, TR));
    for (int64_t u = s.begin; u < s.end; u += s.step) {
        const int64_t r0 = u * TR;
        const int nr = (int)(n - r0 < TR ? n - r0 : TR);
        __syncthreads();  // the previous tile's rows are no longer read
        for (int e = tid; e < nr * 8; e += 256) {
            const int64_t g = r0 * 8 + e;
            rs[0][e] = vq2[g];
            rs[1][e] = y2[g];
            rs[2][e] = Vp ? vp2[g] : make_double2(0.0, 0.0);
        }
        __syncthreads();  // every row of the tile read before any is written
#pragma unroll
        for (int k = 0; k < TR / 16; ++k) {
            const int r = rg + 16 * k;
            if (r >= nr) break;
            double q = 0.0, a = 0.0, c = 0.0, d = 0.0;
#pragma unroll
            for (int i2 = 0; i2 < 8; ++i2) {
                const double2 x = rs[0][r * 8 + i2], yv = rs[1][r * 8 + i2], pv = rs[2][r * 8 + i2];
                q = fma(x.x, mb[2 * i2], q);
                q = fma(x.y, mb[2 * i2 + 1], q);
                a = fma(yv.x, mb[2 * i2], a);
                a = fma(yv.y, mb[2 * i2 + 1], a);
                c = fma(pv.x, m1[2 * i2], c);
                c = fma(pv.y, m1[2 * i2 + 1], c);
                d = fma(x.x, m2[2 * i2], d);
                d = fma(x.y, m2[2 * i2 + 1], d);
            }
            const int64_t g = (r0 + r) * 16 + j;
            if (Y) Wout[g] = (a - c) - d;
            else if (Wm != Wout) {
                const double2 yv = rs[1][r * 8 + (j >> 1)];
                Wout[g] = (j & 1) ? yv.y : yv.x;
            }
            Q0[g] = q;
            if (Q1) Q1[g] = q;
        }
    }
}

// The wavefront step's post-call state (Y != null, b = 16 fp64) on the f64
// MFMA, one wave per 16-row strip, no LDS: W = Y beta^-1 - Vp P1 - Vq P2 and
// Q = Vq beta^-1 (Q0, and Q1 when given) as three / one 16 x 16 x 16 products
// per strip.  Lane (c, g) = (l & 15, l >> 4) loads row c's entries 4g .. 4g+3
// of each input (two 16-B loads: the A operand in the permuted contraction
// order of lz_wf.hip's updaters) and keeps B[4g + k][c] of each 16 x 16 matrix;
// a product comes back as D[g + 4 r][c], stored as 4 rows x 128 B per
// instruction.  Row-local: a wave loads its next strip's inputs before it
// stores the current strip (other rows), and no other wave touches its rows,
// so outputs may alias inputs.  A streaming pass: 3 reads + 3 writes of n x 16
// doubles (the LDS form read each row 16 times from LDS and ran at 4.3 TB/s).
__global__ __launch_bounds__(256) void k_final_state16m(int64_t n, const double *Y, const double *Vp,
                                                        const double *Vq, const double *__restrict__ binv,
                                                        const double *__restrict__ P1,
                                                        const double *__restrict__ P2, double *Wout, double *Q0,
                                                        double *Q1)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    double bq[3][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int idx = (4 * g + k) * 16 + c;
        bq[0][k] = binv[idx];
        bq[1][k] = P1 ? -P1[idx] : 0.0;
        bq[2][k] = -P2[idx];
    }
    const int64_t S = (n + 15) / 16;
    const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    typedef double d2v __attribute__((ext_vector_type(2)));
    auto load = [&](const double *X, int64_t s, double out[4]) {
        const int64_t r = s * 16 + c;
        if (X && r < n) {
            const d2v a = *reinterpret_cast<const d2v *>(X + r * 16 + 4 * g);
            const d2v b = *reinterpret_cast<const d2v *>(X + r * 16 + 4 * g + 2);
            out[0] = a.x; out[1] = a.y; out[2] = b.x; out[3] = b.y;
        } else {
            out[0] = out[1] = out[2] = out[3] = 0.0;
        }
    };
    double ya[4], pa[4], ja[4];
    int64_t s = wid;
    if (s < S) {
        load(Y, s, ya);
        load(Vp, s, pa);
        load(Vq, s, ja);
    }
    for (; s < S; s += nw) {
        d4_t w = {0.0, 0.0, 0.0, 0.0}, q = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; ++k) w = mfma16(pa[k], bq[1][k], w);
#pragma unroll
        for (int k = 0; k < 4; ++k) w = mfma16(ya[k], bq[0][k], w);
#pragma unroll
        for (int k = 0; k < 4; ++k) w = mfma16(ja[k], bq[2][k], w);
#pragma unroll
        for (int k = 0; k < 4; ++k) q = mfma16(ja[k], bq[0][k], q);
        const int64_t sn = s + nw;
        if (sn < S) {  // the next strip's rows (not this strip's) before this strip's stores
            load(Y, sn, ya);
            load(Vp, sn, pa);
            load(Vq, sn, ja);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = s * 16 + g + 4 * r;
            if (row < n) {
                Wout[row * 16 + c] = w[r];
                Q0[row * 16 + c] = q[r];
                if (Q1) Q1[row * 16 + c] = q[r];
            }
        }
    }
}

template <typename T>
int final_state(lz_handle *h, int64_t n, int b, const T *Y, const T *Vp, const T *Vq, const T *Wm, const T *binv,
                const T *P1, const T *P2, T *Wout, T *Q0, T *Q1)
{
    LZ_ARG_CHECK(b >= 1 && b <= 32 && Vq && binv && Wout && Q0 && (Y ? P2 != nullptr : Wm != nullptr),
                 "final state (internal)");
    if (n <= 0) return LZ_OK;
    if (!Y && (b == 16 || b == 32)) {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 64), (int64_t)h->n_cu * 4));
        if (b == 16)
            hipLaunchKernelGGL((k_final_q<T, 16>), dim3(grid), dim3(256), 0, h->stream, n, Vq, Wm, binv, Wout, Q0, Q1);
        else
            hipLaunchKernelGGL((k_final_q<T, 32>), dim3(grid), dim3(256), 0, h->stream, n, Vq, Wm, binv, Wout, Q0, Q1);
        LZ_LAUNCH_CHECK();
        return LZ_OK;
    }
    if constexpr (std::is_same<T, double>::value) {
        const char *fm = getenv("LZ_FS_MFMA");  // "0": the LDS form for the wavefront's call too (A/B)
        if (b == 16 && Y && !(fm && fm[0] == '0')) {
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ceil_div(n, 16), 4), (int64_t)h->n_cu * 8));
            hipLaunchKernelGGL(k_final_state16m, dim3(grid), dim3(256), 0, h->stream, n, Y, Vp, Vq, binv, P1, P2, Wout,
                               Q0, Q1);
            LZ_LAUNCH_CHECK();
            return LZ_OK;
        }
        if (b == 16) {
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 64), (int64_t)h->n_cu * 4));
            hipLaunchKernelGGL(k_final_state16, dim3(grid), dim3(256), 0, h->stream, n, Y, Vp, Vq, Wm, binv, P1, P2,
                               Wout, Q0, Q1);
            LZ_LAUNCH_CHECK();
            return LZ_OK;
        }
    }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 16), (int64_t)h->n_cu * 4));
    hipLaunchKernelGGL((k_final_state<T>), dim3(grid), dim3(256), 0, h->stream, n, b, Y, Vp, Vq, Wm, binv, P1, P2,
                       Wout, Q0, Q1);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// row-major rows x b (ld b) -> column-major (leading dimension ld >= rows), a
// 64-row tile through LDS: coalesced reads, one column piece of 64 per store
template <typename T>
__global__ __launch_bounds__(256) void k_rm_to_cm(int64_t rows, int b, const T *__restrict__ src, int64_t ld,
                                                  T *__restrict__ dst)
{
    constexpr int TR = 64;
    __shared__ T t[TR * kMaxB];
    const int tid = threadIdx.x;
    for (int64_t u = blockIdx.x; u * TR < rows; u += gridDim.x) {
        const int64_t r0 = u * TR;
        const int nr = (int)(rows - r0 < TR ? rows - r0 : TR);
        __syncthreads();
        for (int e = tid; e < nr * b; e += 256) t[e] = src[r0 * b + e];
        __syncthreads();
        for (int e = tid; e < nr * b; e += 256) {
            const int c = e / nr, r = e % nr;
            dst[(int64_t)c * ld + r0 + r] = t[r * b + c];
        }
    }
}

template <typename T>
int to_col_major(lz_handle *h, int64_t rows, int b, const T *src, int64_t ld, T *dst)
{
    LZ_ARG_CHECK(b >= 1 && b <= kMaxB && ld >= rows && src != dst, "to_col_major shape");
    if (rows <= 0) return LZ_OK;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, 64), (int64_t)h->n_cu * 4));
    hipLaunchKernelGGL((k_rm_to_cm<T>), dim3(grid), dim3(256), 0, h->stream, rows, b, src, ld, dst);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

// ================================================================ row probe
template <typename T>
__global__ void k_copy_row(int b, const T *__restrict__ Q, int64_t ld, int col_major, int64_t lc,
                           T *__restrict__ q)
{
    const int c = threadIdx.x;
    if (c < b) q[c] = col_major ? Q[lc + c * ld] : Q[lc * ld + c];
}

template <typename T>
int copy_row(lz_handle *h, int b, const T *Q, int64_t ld, int col_major, int64_t lc, T *q)
{
    hipLaunchKernelGGL((k_copy_row<T>), dim3(1), dim3(64), 0, h->stream, b, Q, ld, col_major, lc,
                       q);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

#define LZ_DENSE_INST(T)                                                                       \
    template int gram_partials<T>(lz_handle *, int64_t, int, const T *, const T *, int64_t,    \
                                  int *);                                                      \
    template int gram_finish<T>(lz_handle *, int, int, int, T *, const double *, const T *, T *); \
    template int sqrtm_pair<T>(lz_handle *, int, const T *, int, T *, T *, T *, const double *, const T *, T *,  \
                               const WfAlpha *);\
    template int tsmm<T>(lz_handle *, int64_t, int, T, T, const T *, const T *, T *, int64_t); \
    template int copy_row<T>(lz_handle *, int, const T *, int64_t, int, int64_t, T *);             \
    template int final_state<T>(lz_handle *, int64_t, int, const T *, const T *, const T *, const T *, const T *, \
                                const T *, const T *, T *, T *, T *);                             \
    template int to_col_major<T>(lz_handle *, int64_t, int, const T *, int64_t, T *);
LZ_DENSE_INST(double)
LZ_DENSE_INST(float)

}  // namespace lz
