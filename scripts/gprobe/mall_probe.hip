// How fast can the chip gather 128-B rows (8 lanes x 16 B, 8 rows per
// wave-instruction: the X gather at b = 16 fp64) when each XCD's gathers fall
// in a window of its own that is larger than its 4 MB L2?  C4's per-rank
// wavefront step gathers inside +-65,536 rows (16.8 MB) of the rows an XCD is
// working on, the 8 XCDs' windows disjoint (DESIGN.md 4, C4 per-rank share).
// Window per XCD = 1 .. 32 MB (8 .. 256 MB in all: L2 -> Infinity Cache), and a
// 2 GB table (HBM).  Blocks are dealt to the XCDs round-robin, so block b
// gathers in window (b mod 8).
//   mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int UNR>
__global__ __launch_bounds__(256) void k_g(const double *__restrict__ X, uint64_t win_bytes, uint32_t rows_mask,
                                           int iters, double *__restrict__ out, uint32_t salt)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    const char *base = reinterpret_cast<const char *>(X) + (blockIdx.x & 7) * win_bytes;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char *>(base), (short)0, (int)((rows_mask + 1u) * 128u), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 4) & rows_mask;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
            __builtin_memcpy(&xs[t], &u, 16);
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
}

static void run(const double *X, uint64_t win, int bpc, double *out)
{
    const uint32_t rows = (uint32_t)(win / 128);
    const int grid = 256 * bpc, iters = 1500;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k_g<8>, dim3(grid), dim3(256), 0, 0, X, win, rows - 1, 200, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_g<8>, dim3(grid), dim3(256), 0, 0, X, win, rows - 1, iters, out, 7u);
    hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return; }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double lines = (double)grid * 4 * iters * 8 * 8;  // 4 waves, 8 loads, 8 lines per wave-instruction
    printf("window per XCD %6.1f MB (all %7.1f MB)  blocks/CU %d : %.3f ms  %6.1f G lines/s  %.2f TB/s\n",
           win / 1048576.0, 8 * win / 1048576.0, bpc, ms, lines / ms / 1e6, lines * 128 / ms / 1e9);
}

int main()
{
    double *X, *out;
    const size_t total = (size_t)2 << 30;
    if (hipMalloc(&X, total) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(X, 0, total);
    hipMalloc(&out, 64);
    for (int bpc : {4, 3}) {
        for (uint64_t mb : {1, 2, 4, 8, 16, 32}) run(X, mb << 20, bpc, out);
        run(X, total / 8, bpc, out);
    }
    return 0;
}
