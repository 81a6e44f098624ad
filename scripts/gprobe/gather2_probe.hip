// Chip-wide gather rate from an L2-resident window (8,192 x 1 KB = 8 MB split
// per XCD... rows_mask picks the window) as a function of the gathered row
// size: ROWB = 128 (8 lanes x 16 B per row, 8 rows per wave-instruction: the
// SpMM's X gather at b = 16 fp64), 256, 512 or 1024 B (64 lanes, one row).
// Same number of 128-B lines per wave-instruction (8) in every case.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int ROWB, int UNR>
__global__ __launch_bounds__(256) void k_g(const double *__restrict__ X, uint32_t rows_mask, int iters,
                                           double *__restrict__ out, uint32_t salt)
{
    constexpr int LPR = ROWB / 16;  // lanes per row
    const int lane = threadIdx.x & 63, p = lane % LPR;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double *>(X), (short)0, (int)((rows_mask + 1) * (uint32_t)ROWB), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / LPR * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 8) & rows_mask;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * (uint32_t)ROWB + 16u * p, 0, 0);
            __builtin_memcpy(&xs[t], &u, 16);
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int ROWB, int UNR>
static void run(const double *X, uint32_t bytes_window, int bpc, double *out)
{
    const uint32_t rows = bytes_window / ROWB;
    const int grid = 256 * bpc, iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_g<ROWB, UNR>), dim3(grid), dim3(256), 0, 0, X, rows - 1, 20, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_g<ROWB, UNR>), dim3(grid), dim3(256), 0, 0, X, rows - 1, iters, out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double lines = (double)grid * 4 * iters * UNR * 8;  // 4 waves, 8 lines per wave-instruction
    printf("row %4d B  window %5u KB  UNR %d  blocks/CU %d : %.3f ms  %.1f G lines/s  %.2f TB/s\n", ROWB,
           bytes_window >> 10, UNR, bpc, ms, lines / ms / 1e6, lines * 128 / ms / 1e9);
}

int main()
{
    double *X, *out;
    hipMalloc(&X, (size_t)64 << 20);
    hipMemset(X, 0, (size_t)64 << 20);
    hipMalloc(&out, 64);
    for (uint32_t w : {1u << 20, 2u << 20}) {
        for (int bpc : {4, 8}) {
            run<128, 8>(X, w, bpc, out);
            run<256, 8>(X, w, bpc, out);
            run<512, 8>(X, w, bpc, out);
            run<1024, 8>(X, w, bpc, out);
        }
    }
    run<128, 16>(X, 1u << 20, 4, out);
    run<1024, 16>(X, 1u << 20, 4, out);
    return 0;
}
