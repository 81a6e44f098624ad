// Does an HBM-latency share of the requests set the 128-B gather rate?
// Waves gather 128-B rows (8 lanes x 16 B, 8 loads in flight per lane) from an
// L2-resident 1 MB window; in mode "mix", every F-th load instead reads a
// random 128-B row of a 4 GB table (an HBM miss, the SpMM's compulsory X
// misses and CSR stream); in mode "split", the same HBM loads are issued by
// separate blocks (other CUs' waves) that do nothing else.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int F, int SPLIT>
__global__ __launch_bounds__(256) void k_mix(const double *__restrict__ X, uint32_t wmask, const double *__restrict__ Z,
                                             uint32_t zmask, int iters, double *__restrict__ out, uint32_t salt)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)((wmask + 1) * 128u), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    // SPLIT: blocks with blockIdx % F == 0 issue only HBM loads (one in F of all loads), the rest only L2 gathers
    const bool hbm_block = SPLIT && (blockIdx.x % F) == 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            h = h * 1664525u + 1013904223u;
            const bool far = SPLIT ? hbm_block : (F > 0 && ((it * 8 + t) % F) == 0);
            if (far) {
                const uint64_t row = ((uint64_t)h * 2654435761ull) & zmask;
                xs[t] = *reinterpret_cast<const double2 *>(Z + row * 16 + 2 * p);
            } else {
                const uint32_t row = (h >> 8) & wmask;
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
                __builtin_memcpy(&xs[t], &u, 16);
            }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int F, int SPLIT>
static void run(const double *X, const double *Z, uint32_t zrows, int bpc, double *out)
{
    const int grid = 256 * bpc, iters = 1000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_mix<F, SPLIT>), dim3(grid), dim3(256), 0, 0, X, 8191u, Z, zrows - 1, 20, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_mix<F, SPLIT>), dim3(grid), dim3(256), 0, 0, X, 8191u, Z, zrows - 1, iters, out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double lines = (double)grid * 4 * iters * 8 * 8;
    printf("%s F=%2d blocks/CU %d : %.3f ms  %.1f G lines/s (%.1f G L2-window lines/s)\n", SPLIT ? "split" : "mix  ", F,
           bpc, ms, lines / ms / 1e6, (F ? lines * (F - 1) / F : lines) / ms / 1e6);
}

int main()
{
    double *X, *Z, *out;
    const uint32_t zrows = 1u << 25;  // 4 GB of 128-B rows
    hipMalloc(&X, (size_t)1 << 20);
    hipMemset(X, 0, (size_t)1 << 20);
    hipMalloc(&Z, (size_t)zrows * 128);
    hipMemset(Z, 0, (size_t)zrows * 128);
    hipMalloc(&out, 64);
    run<0, 0>(X, Z, zrows, 4, out);
    run<20, 0>(X, Z, zrows, 4, out);
    run<10, 0>(X, Z, zrows, 4, out);
    run<5, 0>(X, Z, zrows, 4, out);
    run<10, 0>(X, Z, zrows, 8, out);
    run<10, 1>(X, Z, zrows, 4, out);
    run<5, 1>(X, Z, zrows, 4, out);
    run<10, 1>(X, Z, zrows, 8, out);
    return 0;
}
