// Does address-translation reach bound the X gathers?  The same chip-wide gather
// as gather2_probe (128-B rows, 8 lanes x 16 B, 8 rows per wave-instruction, 8
// loads in flight per lane) over a fixed set of 8,192 distinct rows (1 MB of
// lines, L2-resident), but row r placed at r * STRIDE: STRIDE = 128 packs the
// set into one 1 MB range, larger strides spread the same lines over more pages
// (4 KB + 128: one line per 4 KB page; 64 KB + 128; 2 MB + 128).  A falling
// rate with the stride means the gathers pay for translation misses.
//   hipcc --offload-arch=gfx950 -O3 -o tlb_probe tlb_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int UNR>
__global__ __launch_bounds__(256) void k_g(const char *__restrict__ X, uint64_t stride, uint32_t rows_mask,
                                           int iters, double *__restrict__ out, uint32_t salt)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint64_t row = (h >> 8) & rows_mask;
            xs[t] = *reinterpret_cast<const double2 *>(X + row * stride + 16u * p);
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1 + lane;
}

static void run(const char *X, uint64_t stride, uint32_t rows, int bpc, double *out)
{
    const int grid = 256 * bpc, iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_g<8>), dim3(grid), dim3(256), 0, 0, X, stride, rows - 1, 20, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_g<8>), dim3(grid), dim3(256), 0, 0, X, stride, rows - 1, iters, out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double lines = (double)grid * 4 * iters * 8 * 8;
    printf("rows %5u  stride %8llu B  span %8.1f MB  blocks/CU %d : %.3f ms  %.1f G lines/s\n", rows,
           (unsigned long long)stride, rows * (double)stride / 1048576.0, bpc, ms, lines / ms / 1e6);
    hipEventDestroy(e0); hipEventDestroy(e1);
}

int main()
{
    const uint64_t bytes = (uint64_t)8192 * ((2u << 20) + 128) + 4096;
    char *X; double *out;
    if (hipMalloc(&X, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(X, 0, bytes);
    hipMalloc(&out, 64);
    for (int bpc : {4, 7}) {
        for (uint64_t s : {128ull, 4096ull + 128, 65536ull + 128, (2ull << 20) + 128}) run(X, s, 8192, bpc, out);
        for (uint64_t s : {128ull, 4096ull + 128, 65536ull + 128}) run(X, s, 2048, bpc, out);
    }
    hipDeviceSynchronize();
    return 0;
}
