// Where should the HBM stream of a gather-bound kernel be issued?  Every block
// runs for the same wall-clock time (s_memrealtime) and counts its iterations.
//   mode 0: every wave gathers 128-B rows from an L2-resident 1 MB window
//   mode 1: every wave gathers, and one load in F is a coalesced 1-KB piece of a
//           sequential 4 GB stream (the CSR stream / compulsory X in the SpMM)
//   mode 2: the stream moves to dedicated blocks: blocks whose XCD-local index
//           (blockIdx / 8) is a multiple of F stream only (8 loads in flight per
//           lane), the others gather only
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(256) void k_split(const double *__restrict__ X, const double *__restrict__ Z,
                                               uint64_t zlines, int mode, int F, long long ticks,
                                               unsigned long long *__restrict__ cnt, double *__restrict__ out)
{
    const int lane = threadIdx.x & 63, p = lane & 7, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)(8192u * 128u), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + 11u;
    const bool streamer = mode == 2 && ((blockIdx.x >> 3) % F) == 0;
    // each block streams its own region: 1 KB per wave-instruction, sequential
    uint64_t zpos = ((uint64_t)blockIdx.x * 4 + w) * 1048576ull % zlines;  // in 128-B lines, 1 KB steps
    double a0 = 0, a1 = 0;
    unsigned long long it = 0, glines = 0, slines = 0;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        double2 xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const bool st = streamer || (mode == 1 && ((it * 8 + t) % F) == 0);
            if (st) {
                const uint64_t line = (zpos + (uint64_t)(lane >> 3)) % zlines;  // 8 consecutive lines per wave-instr
                xs[t] = *reinterpret_cast<const double2 *>(Z + line * 16 + 2 * p);
                zpos += 8;
            } else {
                h = h * 1664525u + 1013904223u;
                const uint32_t row = (h >> 8) & 8191u;
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
                __builtin_memcpy(&xs[t], &u, 16);
            }
            if (st) slines += 8; else glines += 8;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
        ++it;
    }
    if (a0 == 12345.0) out[0] = a1;
    if (lane == 0) {
        atomicAdd(&cnt[0], glines);
        atomicAdd(&cnt[1], slines);
    }
}

int main()
{
    double *X, *Z, *out;
    unsigned long long *cnt;
    const uint64_t zlines = 1ull << 25;  // 4 GB
    hipMalloc(&X, (size_t)1 << 20); hipMemset(X, 0, (size_t)1 << 20);
    hipMalloc(&Z, zlines * 128); hipMemset(Z, 0, zlines * 128);
    hipMalloc(&out, 64); hipMalloc(&cnt, 16);
    const long long ticks = 200000;  // 2 ms at 100 MHz
    struct Cfg { int mode, F, bpc; };
    for (Cfg c : std::vector<Cfg>{{0, 1, 4}, {1, 10, 4}, {1, 5, 4}, {2, 10, 4}, {2, 5, 4}, {2, 10, 8}, {1, 10, 8}}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(cnt, 0, 16);
            hipLaunchKernelGGL(k_split, dim3(256 * c.bpc), dim3(256), 0, 0, X, Z, zlines, c.mode, c.F, ticks, cnt, out);
            hipDeviceSynchronize();
            unsigned long long hc[2];
            hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost);
            if (rep)
                printf("mode %d F=%2d blocks/CU %d : gather %.1f G lines/s (%.1f TB/s)  stream %.2f TB/s\n", c.mode, c.F,
                       c.bpc, hc[0] / 2e-3 / 1e9, hc[0] * 128 / 2e-3 / 1e12, hc[1] * 128 / 2e-3 / 1e12);
        }
    }
    return 0;
}
