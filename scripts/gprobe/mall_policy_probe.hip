// Does a stream's cache policy decide whether a gather window stays in the
// Infinity Cache?  C4's per-rank wavefront step gathers inside per-XCD windows
// of 16.8 MB (134 MB for the 8 XCDs: Infinity-Cache sized, not L2 sized) while
// the same CUs stream ~4.6 GB per launch; the launch gathers at ~52 G lines/s,
// the HBM rate of mall_probe, not its 81 G lines/s Infinity-Cache rate.
//
// Part 1: gathers in the 8 windows (8 rows x 128 B per wave-instruction, as the
// step's X gather) interleaved with 16-B-per-lane streaming loads of a 4 GB
// buffer, 1 stream instruction per 4 gather instructions (the step's ratio),
// the stream's buffer-instruction cache policy: 0 plain, 2 nt, 16 sc1, 18 sc1|nt.
// Part 2: the windows written (16-B stores, policy 0 / 2 / 16 / 18) by one
// kernel, then gathered once (plain loads) by the next: the gather rate says
// whether the written lines are still on the die.  Baselines: gathers with no
// stream, and after a 2 GB plain stream between the write and the gather.
//   hipcc -O3 --offload-arch=gfx950 mall_policy_probe.hip -o mall_policy_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr uint64_t kWin = 16800ull * 1024;   // bytes per XCD window
constexpr uint32_t kRows = kWin / 128;       // rows per window

template <int AUX>
__global__ __launch_bounds__(256) void k_mix(const double *__restrict__ X, const double *__restrict__ S,
                                             uint64_t sbytes, int iters, int stream, double *__restrict__ out,
                                             uint32_t salt)
{
    const int lane = threadIdx.x & 63, p = lane & 7, w = threadIdx.x >> 6;
    const char *base = reinterpret_cast<const char *>(X) + (blockIdx.x & 7) * kWin;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), (short)0, (int)kWin, 0x00020000);
    // this wave's stream: 1 KB per instruction, consecutive, wrapping inside its share
    const uint64_t waves = (uint64_t)gridDim.x * 4, share = (sbytes / waves) & ~(uint64_t)1023;
    const char *sb = reinterpret_cast<const char *>(S) + ((uint64_t)blockIdx.x * 4 + w) * share;
    const auto sr = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(sb), (short)0, (int)share, 0x00020000);
    uint32_t soff = 0;
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + salt;
    double a0 = 0, a1 = 0;
    for (int it = 0; it < iters; ++it) {
        double2 xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 4) % kRows;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
            __builtin_memcpy(&xs[t], &u, 16);
        }
        double2 ss[2] = {};
        if (stream) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(sr, soff + 16u * lane, 0, AUX);
                __builtin_memcpy(&ss[t], &u, 16);
                soff += 1024;
                if (soff >= share) soff = 0;
            }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
        a0 += ss[0].x + ss[1].y;
    }
    if (a0 == 12345.0) out[0] = a1;
}

template <int AUX>
__global__ __launch_bounds__(256) void k_write(double *X, uint64_t bytes, double v)
{
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(X, (short)0, (int)bytes, 0x00020000);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    for (uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; o < bytes; o += (uint64_t)gridDim.x * 256 * 16) {
        const double2 d = make_double2(v, v + 1.0);
        u4 u;
        __builtin_memcpy(&u, &d, 16);
        __builtin_amdgcn_raw_buffer_store_b128(u, xr, (uint32_t)o, 0, AUX);
    }
}

// every row of the 8 windows gathered exactly once, in a scrambled order
// (1,000,003 is prime and does not divide the row count: a bijection)
__global__ __launch_bounds__(256) void k_perm_gather(const double *__restrict__ X, double *__restrict__ out)
{
    constexpr uint32_t N = 8 * kRows;
    const int lane = threadIdx.x & 63, p = lane & 7, g = lane >> 3;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)(8 * kWin), 0x00020000);
    const uint32_t waves = gridDim.x * 4, wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    double a = 0;
    for (uint32_t ins = wv; ins < N / 8; ins += waves) {
        const uint32_t row = (uint32_t)(((uint64_t)(ins * 8 + g) * 1000003ull) % N);
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
        double2 d;
        __builtin_memcpy(&d, &u, 16);
        a += d.x;
    }
    if (a == 12345.0) out[0] = a;
}

__global__ __launch_bounds__(256) void k_stream(const double *__restrict__ S, uint64_t bytes, double *out)
{
    double a = 0;
    const double2 *s2 = reinterpret_cast<const double2 *>(S);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < bytes / 16; i += (uint64_t)gridDim.x * 256)
        a += s2[i].x;
    if (a == 12345.0) out[0] = a;
}

static float timed(hipEvent_t e0, hipEvent_t e1)
{
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

template <int AUX>
static void mix(const double *X, const double *S, uint64_t sbytes, double *out, int stream, const char *name)
{
    const int grid = 256 * 4, iters = 1200;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_mix<AUX>, dim3(grid), dim3(256), 0, 0, X, S, sbytes, 200, stream, out, 1u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mix<AUX>, dim3(grid), dim3(256), 0, 0, X, S, sbytes, iters, stream, out, 7u);
    hipEventRecord(e1);
    const float ms = timed(e0, e1);
    const double lines = (double)grid * 4 * iters * 8 * 8, sb = stream ? (double)grid * 4 * iters * 2 * 1024 : 0;
    printf("part 1  stream %-9s : %.3f ms  gathers %6.1f G lines/s  stream %.2f TB/s\n", name, ms, lines / ms / 1e6,
           sb / ms / 1e9);
}

template <int AUX>
static void wr_then_gather(double *X, const double *S, double *out, int flush, const char *name)
{
    const int grid = 256 * 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // fill the die with something else first
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, S, (uint64_t)2 << 30, out);
    hipLaunchKernelGGL(k_write<AUX>, dim3(grid), dim3(256), 0, 0, X, 8 * kWin, 1.0);
    if (flush) hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, S + (1ull << 27), (uint64_t)2 << 30, out);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_perm_gather, dim3(grid), dim3(256), 0, 0, X, out);
    hipEventRecord(e1);
    const float ms = timed(e0, e1);
    const double lines = 8.0 * kRows;
    printf("part 2  write %-9s%s: gather %.4f ms  %6.1f G lines/s\n", name, flush ? " + 2 GB stream" : "             ",
           ms, lines / ms / 1e6);
}

int main()
{
    double *X, *S, *out;
    const uint64_t sbytes = (uint64_t)4 << 30;
    if (hipMalloc(&X, 8 * kWin) != hipSuccess || hipMalloc(&S, sbytes) != hipSuccess ||
        hipMalloc(&out, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(X, 0, 8 * kWin);
    hipMemset(S, 0, sbytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        mix<0>(X, S, sbytes, out, 0, "none");
        mix<0>(X, S, sbytes, out, 1, "plain");
        mix<2>(X, S, sbytes, out, 1, "nt");
        mix<16>(X, S, sbytes, out, 1, "sc1");
        mix<18>(X, S, sbytes, out, 1, "sc1|nt");
    }
    for (int rep = 0; rep < 2; ++rep) {
        wr_then_gather<0>(X, S, out, 0, "plain");
        wr_then_gather<2>(X, S, out, 0, "nt");
        wr_then_gather<16>(X, S, out, 0, "sc1");
        wr_then_gather<18>(X, S, out, 0, "sc1|nt");
        wr_then_gather<0>(X, S, out, 1, "plain");
    }
    return 0;
}
