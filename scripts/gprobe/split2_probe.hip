// Can an L2 gather stream and a near-peak HBM stream run at the same time on
// the same CUs?  (The SpMM needs ~1e8 gathered 128-B rows AND 3.84 GB of HBM
// traffic per launch: 0.8 ms means ~125 G lines/s beside ~4.8 TB/s.)
// Every block runs for the same wall-clock time (s_memrealtime) and counts its
// work.  Blocks whose XCD-local index (blockIdx / 8) is a multiple of F are
// streamers: each wave walks its own sequential region, 1 KB per
// wave-instruction, 8 loads in flight per lane (VGPR loads, or LDS-DMA when
// DMA = 1), and stores W x 1 KB to a second region per 8 KB read.  The
// other blocks gather random 128-B rows (8 lanes x 16 B, 8 loads in flight per
// lane) from a 2 MB window (resident in every XCD's L2).
//   split2_probe            (sweeps F, blocks per CU, DMA, write share)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((address_space(3))) void lds_t;

template <int DMA>
__global__ __launch_bounds__(256) void k_split2(const double *__restrict__ X, const double *__restrict__ Z,
                                                double *__restrict__ Zw, uint64_t zlines, int F, int W, int M, long long ticks,
                                                unsigned long long *__restrict__ cnt, double *__restrict__ out)
{
    __shared__ double lds[4][8][128];  // 32 KB: 4 blocks per CU  // DMA landing area (per wave: 8 pieces of 1 KB)
    const int lane = threadIdx.x & 63, p = lane & 7, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)(16384u * 128u), 0x00020000);
    uint32_t h = (blockIdx.x * 256 + threadIdx.x) / 8 * 2654435761u + 11u;
    // M = 0: by XCD-local index mod F (with 4 blocks per CU and 32 CUs per XCD,
    // F | 32 puts streamers and gatherers on different CUs); M = 1: by
    // (XCD-local index / 32) mod F (each CU holds both kinds)
    const int kx = blockIdx.x >> 3;
    const bool streamer = F > 0 && ((M ? kx / 32 : kx) % F) == 0;
    // each wave streams its own, never repeated, partition of Z (and of Zw)
    const uint64_t nwaves = (uint64_t)gridDim.x * 4, wid = (uint64_t)blockIdx.x * 4 + w;
    const uint64_t part = zlines * 128 / nwaves & ~(uint64_t)1023;  // bytes
    const char *zb = (const char *)Z + wid * part;
    char *zwb = (char *)Zw + wid * part / 2;
    uint64_t zpos = 0;
    double a0 = 0, a1 = 0;
    unsigned long long glines = 0, rbytes = 0, wbytes = 0;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    if (streamer) {
        const __amdgpu_buffer_rsrc_t zr =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(zb), (short)0, (int)part, 0x00020000);
        int it = 0;
        while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
            double2 xs[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t off = (uint32_t)(((zpos + t) * 1024u) % part) + 16u * lane;
                if constexpr (DMA) {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(zr, (lds_t *)&lds[w][t][0], 16, off, 0, 0, 0);
                } else {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(zr, off, 0, 0);
                    __builtin_memcpy(&xs[t], &v, 16);
                }
            }
            zpos += 8;
            rbytes += 8 * 1024;
            if constexpr (DMA) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
#pragma unroll
                for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
            }
            for (int t = 0; t < W; ++t) {  // W x 1 KB stored per 8 KB read
                const uint64_t u = ((zpos / 8 * W + t) * 1024u) % (part / 2);
                double2 v = {a0, a1};
                *reinterpret_cast<double2 *>(zwb + u + 16 * lane) = v;
                wbytes += 1024;
            }
            ++it;
        }
    } else {
        while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
            double2 xs[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                h = h * 1664525u + 1013904223u;
                const uint32_t row = (h >> 8) & 16383u;
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, row * 128u + 16u * p, 0, 0);
                __builtin_memcpy(&xs[t], &u, 16);
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
            glines += 8 * 8;
        }
    }
    if (a0 == 12345.0) out[0] = a1 + lds[w][lane & 7][lane];
    if (lane == 0) {
        atomicAdd(&cnt[0], glines);
        atomicAdd(&cnt[1], rbytes);
        atomicAdd(&cnt[2], wbytes);
    }
}

int main()
{
    double *X, *Z, *Zw, *out;
    unsigned long long *cnt;
    const uint64_t zlines = 1ull << 28;  // 32 GB read region (16 GB written): no stream repeats in 2 ms
    hipMalloc(&X, (size_t)16384 * 128); hipMemset(X, 0, (size_t)16384 * 128);
    hipMalloc(&Z, zlines * 128); hipMemset(Z, 0, zlines * 128);
    hipMalloc(&Zw, zlines * 64);
    hipMalloc(&out, 64); hipMalloc(&cnt, 24);
    const long long ticks = 200000;  // 2 ms at 100 MHz
    struct Cfg { int F, bpc, dma, W, M; };
    std::vector<Cfg> cfgs = {{0, 4, 0, 0, 0}, {1, 4, 0, 0, 0}, {1, 4, 1, 0, 0}, {1, 4, 0, 4, 0},
                             {4, 4, 0, 0, 0}, {4, 4, 0, 0, 1}, {4, 4, 0, 4, 0}, {4, 4, 0, 4, 1},
                             {2, 4, 0, 0, 0}, {2, 4, 0, 0, 1}, {2, 4, 0, 4, 0}, {2, 4, 0, 4, 1},
                             {2, 4, 1, 4, 0}, {2, 4, 1, 4, 1}, {8, 4, 0, 4, 0}};
    for (Cfg c : cfgs) {
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(cnt, 0, 24);
            if (c.dma)
                hipLaunchKernelGGL(k_split2<1>, dim3(256 * c.bpc), dim3(256), 0, 0, X, Z, Zw, zlines, c.F, c.W, c.M, ticks, cnt, out);
            else
                hipLaunchKernelGGL(k_split2<0>, dim3(256 * c.bpc), dim3(256), 0, 0, X, Z, Zw, zlines, c.F, c.W, c.M, ticks, cnt, out);
            hipDeviceSynchronize();
            unsigned long long hc[3];
            hipMemcpy(hc, cnt, 24, hipMemcpyDeviceToHost);
            if (rep)
                printf("F=%d %s blocks/CU %d dma %d W=%d : gather %6.1f G lines/s  read %.2f TB/s  write %.2f TB/s\n", c.F,
                       c.M ? "in-CU " : "per-CU", c.bpc, c.dma, c.W, hc[0] / 2e-3 / 1e9, hc[1] / 2e-3 / 1e12, hc[2] / 2e-3 / 1e12);
        }
    }
    return 0;
}
