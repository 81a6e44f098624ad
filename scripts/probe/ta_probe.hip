// TA cost of partially-useful gather instructions: 8 gathers per step, each a
// wave-instruction of 64 lanes x 16 B over 8 rows of 128 B (L2-resident);
// lanes beyond `act` (of 64) are either out-of-range (buffer OOB offset) or
// exec-masked.  Reports wave-instructions per microsecond per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>  // 0: OOB lanes, 1: exec-masked lanes
__global__ __launch_bounds__(256) void k_ta(const double *__restrict__ X, uint32_t rows_mask, int iters, int act,
                                            double *__restrict__ out)
{
    const int lane = threadIdx.x & 63, p = lane & 7;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)((rows_mask + 1) * 128), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + 7;
    double a0 = 0, a1 = 0;
    const bool on = lane < act;
    for (int it = 0; it < iters; ++it) {
        double2 xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 8) & rows_mask;
            if (MODE == 0) {
                const uint32_t off = on ? row * 128u + 16u * p : 0x80000000u;
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
                __builtin_memcpy(&xs[t], &u, 16);
            } else {
                xs[t] = double2{0.0, 0.0};
                if (on) {
                    const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
                    __builtin_memcpy(&xs[t], &u, 16);
                }
            }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int MODE>
static void run(const double *X, int act, double *out)
{
    const int grid = 256 * 4, iters = 1000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_ta<MODE>), dim3(grid), dim3(256), 0, 0, X, (1u << 13) - 1, 10, act, out);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_ta<MODE>), dim3(grid), dim3(256), 0, 0, X, (1u << 13) - 1, iters, act, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double instr = (double)grid * 4 * iters * 8;  // wave-instructions
    printf("%s act=%2d lanes: %.3f ms  %.1f wave-instr/us/CU  useful %.2f TB/s\n", MODE ? "exec-mask" : "OOB      ", act,
           ms, instr / 256 / (ms * 1e3), instr * act * 16 / ms / 1e9);
}

int main()
{
    double *X, *out;
    hipMalloc(&X, (size_t)(1u << 13) * 128);
    hipMemset(X, 0, (size_t)(1u << 13) * 128);
    hipMalloc(&out, 64);
    for (int act : {64, 48, 32, 16, 8}) { run<0>(X, act, out); run<1>(X, act, out); }
    return 0;
}
