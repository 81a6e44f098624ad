// Chip-wide rate of 128-B row gathers (8 lanes x 16 B per row) from an
// L2-resident window, vs loads in flight per lane and waves per CU; and the
// same gathers with an HBM stream mixed into the same waves (S stream loads of
// 16 B/lane per 8 gathers) or into separate waves (stream-only blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int UNR, int S>
__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ X, uint32_t rows_mask,
                                                const double *__restrict__ Z, int iters,
                                                double *__restrict__ out, uint32_t salt, int mode)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)((rows_mask + 1) * 128), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    // stream: each block walks its own contiguous slice of Z (16 B per lane per load)
    const int64_t per_block = (int64_t)iters * (S > 0 ? S : 1) * 256 * 2;
    const double *zb = Z + (int64_t)blockIdx.x * per_block + threadIdx.x * 2;
    // mode 1: odd blocks stream (they land on other XCDs); mode 2: waves 2,3 of
    // every block stream (same CU as the gathering waves 0,1)
    const bool stream_only = (mode == 1 && (blockIdx.x & 1)) || (mode == 2 && (threadIdx.x >> 7));
    for (int it = 0; it < iters; ++it) {
        double2 xs[UNR > 0 ? UNR : 1];
        if (!stream_only) {
#pragma unroll
            for (int t = 0; t < UNR; ++t) {
                h = h * 1664525u + 1013904223u;
                const uint32_t row = (h >> 8) & rows_mask;
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
                __builtin_memcpy(&xs[t], &u, 16);
            }
        }
        double2 zs[S > 0 ? S : 1];
        if (mode == 0 || stream_only) {
#pragma unroll
            for (int s = 0; s < S; ++s) zs[s] = *reinterpret_cast<const double2 *>(zb + ((int64_t)it * S + s) * 512);
        }
        if (!stream_only) {
#pragma unroll
            for (int t = 0; t < UNR; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
        }
        if (mode == 0 || stream_only) {
#pragma unroll
            for (int s = 0; s < S; ++s) { a0 += zs[s].x; a1 += zs[s].y; }
        }
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int UNR, int S>
static void run(const double *X, uint32_t rows, const double *Z, int blocks_per_cu, int mode, double *out)
{
    const int grid = 256 * blocks_per_cu, iters = 1000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_gather<UNR, S>), dim3(grid), dim3(256), 0, 0, X, rows - 1, Z, 10, out, 1u, mode);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_gather<UNR, S>), dim3(grid), dim3(256), 0, 0, X, rows - 1, Z, iters, out, 7u, mode);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double gblocks = mode ? grid / 2.0 : grid, sblocks = mode ? grid / 2.0 : grid;
    const double gbytes = gblocks * 256 / 8 * iters * UNR * 128;
    const double sbytes = S ? sblocks * 256 * 16.0 * iters * S : 0;
    printf("rows=%u UNR=%d S=%d mode=%s blocks/CU=%d : %.3f ms  gather %.2f TB/s  stream %.2f TB/s\n", rows, UNR, S,
           mode == 2 ? "wave-split(same CU)" : mode ? "block-split(other XCD)" : "mixed", blocks_per_cu, ms, gbytes / ms / 1e9, sbytes / ms / 1e9);
}

int main()
{
    double *X, *Z, *out;
    hipMalloc(&X, (size_t)(1u << 20) * 128);
    hipMemset(X, 0, (size_t)(1u << 20) * 128);
    const size_t zbytes = (size_t)256 * 8 * 1010 * 8 * 256 * 16 + (1 << 20);  // 8 blocks/CU, S<=8
    hipMalloc(&Z, zbytes);
    hipMemset(Z, 0, zbytes);
    hipMalloc(&out, 64);
    printf("Z %.2f GB\n", zbytes / 1e9);
    run<8, 0>(X, 1u << 13, Z, 4, 0, out);
    run<8, 1>(X, 1u << 13, Z, 4, 0, out);
    run<8, 2>(X, 1u << 13, Z, 4, 0, out);
    run<8, 4>(X, 1u << 13, Z, 4, 0, out);
    run<8, 8>(X, 1u << 13, Z, 4, 0, out);
    run<8, 2>(X, 1u << 13, Z, 4, 1, out);
    run<8, 8>(X, 1u << 13, Z, 4, 1, out);
    run<8, 2>(X, 1u << 13, Z, 4, 2, out);
    run<8, 8>(X, 1u << 13, Z, 4, 2, out);
    run<0, 8>(X, 1u << 13, Z, 4, 0, out);
    return 0;
}
