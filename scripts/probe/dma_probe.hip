// Streaming rate of one LDS-DMA loader wave per CU (60 x 1 KB buffer_load...lds
// per tile, two LDS stages, counted vmcnt wait for the previous tile), alone and
// with NG gather waves on the same CU (8 x 16-B loads per lane in flight, random
// 128-B rows of an L2-resident 1 MB window).  One block per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_t;
constexpr int TILE_KB = 60;

template <int NG>
__global__ __launch_bounds__(64 * (NG + 1)) void k_dma(const char *__restrict__ S, int64_t per_block, int tiles,
                                                       const double *__restrict__ X, double *__restrict__ out,
                                                       int prio, int lwaves)
{
    extern __shared__ char lds[];  // 2 x 60 KB stages + flag
    int *flag = reinterpret_cast<int *>(lds + 2 * TILE_KB * 1024);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) *flag = 0;
    __syncthreads();
    if (w < lwaves) {
        if (prio) __builtin_amdgcn_s_setprio(3);
        const char *base = S + blockIdx.x * per_block;
        for (int t = 0; t < tiles; ++t) {
            const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base + (int64_t)t * TILE_KB * 1024),
                                                             (short)0, TILE_KB * 1024, 0x00020000);
            char *dst = lds + (t & 1) * TILE_KB * 1024;
#pragma unroll
            for (int q = w; q < TILE_KB; q += 1) {
                if ((q % lwaves) != w) continue;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t *)(dst + q * 1024), 16, q * 1024 + lane * 16, 0, 0, 0);
            }
            if (t) asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0 && w == 0) asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)(lds_t *)flag), "v"(1) : "memory");
        return;
    }
    // gather waves: until the loader is done
    const int p = lane & 7;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, 1 << 20, 0x00020000);
    uint32_t h = (blockIdx.x * 1024 + threadIdx.x) / 8 * 2654435761u + 7;
    double a0 = 0, a1 = 0;
    long it = 0;
    for (;; ++it) {
        if ((it & 3) == 0) {
            int v;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_t *)flag) : "memory");
            if (__builtin_amdgcn_readfirstlane(v)) break;
        }
        double2 xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            h = h * 1664525u + 1013904223u;
            const uint32_t row = (h >> 8) & 8191;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
            __builtin_memcpy(&xs[t], &u, 16);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
    }
    if (a0 == 12345.0) out[0] = a1;
    if (lane == 0) atomicAdd(reinterpret_cast<unsigned long long *>(out + 1), (unsigned long long)it);
}

template <int NG>
static void run(const char *S, int tiles, const double *X, double *out, int prio, int lwaves)
{
    const int grid = 256;
    const int64_t per_block = (int64_t)tiles * TILE_KB * 1024;
    const size_t lds = 2 * TILE_KB * 1024 + 64;
    hipFuncSetAttribute((const void *)k_dma<NG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_dma<NG>), dim3(grid), dim3(64 * (NG + 1)), lds, 0, S, per_block, 4, X, out, prio, lwaves);
    hipMemset(out, 0, 16);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_dma<NG>), dim3(grid), dim3(64 * (NG + 1)), lds, 0, S, per_block, tiles, X, out, prio, lwaves);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long its[2];
    hipMemcpy(its, out, 16, hipMemcpyDeviceToHost);
    const double sbytes = (double)grid * per_block;
    const double gbytes = (double)its[1] * 8 * 1024;
    printf("NG=%2d loaders=%d prio=%d: %.3f ms  stream %.2f TB/s (%.1f KB/us/CU, %.2f us/tile)  gather %.2f TB/s\n", NG,
           lwaves, prio, ms, sbytes / ms / 1e9, sbytes / 256 / ms / 1e6, ms * 1e3 / tiles, gbytes / ms / 1e9);
}

int main()
{
    const int tiles = 200;
    char *S; double *X, *out;
    hipMalloc(&S, (size_t)256 * tiles * TILE_KB * 1024);
    hipMemset(S, 0, (size_t)256 * tiles * TILE_KB * 1024);
    hipMalloc(&X, 1 << 20); hipMemset(X, 0, 1 << 20);
    hipMalloc(&out, 64);
    run<0>(S, tiles, X, out, 0, 1);
    run<0>(S, tiles, X, out, 0, 1);
    run<4>(S, tiles, X, out, 1, 1);
    run<8>(S, tiles, X, out, 1, 1);
    run<15>(S, tiles, X, out, 1, 1);
    run<15>(S, tiles, X, out, 0, 1);
    run<15>(S, tiles, X, out, 1, 2);
    run<15>(S, tiles, X, out, 1, 4);
    return 0;
}
