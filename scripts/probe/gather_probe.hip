// Chip-wide rate of 128-B row gathers (8 lanes x 16 B per row) from an
// L2-resident window, vs loads in flight per lane and waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int UNR>
__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ X, uint32_t rows_mask,
                                                int iters, double *__restrict__ out, uint32_t salt)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)((rows_mask + 1) * 128), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 8) & rows_mask;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
            __builtin_memcpy(&xs[t], &u, 16);
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int UNR>
static void run(const double *X, uint32_t rows, int blocks_per_cu, double *out)
{
    const int grid = 256 * blocks_per_cu, iters = 2000 / UNR * 8;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k_gather<UNR>, dim3(grid), dim3(256), 0, 0, X, rows - 1, 10, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_gather<UNR>, dim3(grid), dim3(256), 0, 0, X, rows - 1, iters, out, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double bytes = (double)grid * 256 / 8 * iters * UNR * 128;
    printf("rows=%u (%.1f MB) UNR=%d blocks/CU=%d : %.3f ms  %.2f TB/s  (%.1f B/clk/CU @2.4GHz)\n", rows,
           rows * 128 / 1e6, UNR, blocks_per_cu, ms, bytes / ms / 1e9, bytes / ms / 1e9 * 1e12 / 256 / 2.4e9 / 1e3 * 1e3 / 1e3);
}

int main()
{
    double *X, *out;
    const uint32_t maxrows = 1u << 24;  // 2 GiB
    hipMalloc(&X, (size_t)maxrows * 128);
    hipMemset(X, 0, (size_t)maxrows * 128);
    hipMalloc(&out, 64);
    for (uint32_t rows : {1u << 10, 1u << 13, 1u << 16, 1u << 20, 1u << 24}) {
        run<8>(X, rows, 4, out);
    }
    for (int bpc : {2, 4, 8}) { run<4>(X, 1u << 13, bpc, out); run<8>(X, 1u << 13, bpc, out); run<16>(X, 1u << 13, bpc, out); }
    return 0;
}
