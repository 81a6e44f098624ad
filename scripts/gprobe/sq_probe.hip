// Does an HBM stream carried by SCALAR loads (the scalar data cache path, its
// own miss tracking and lgkmcnt) leave a CU's vector gathers alone, where a
// vector-load stream on the same CU halves them (split2_probe)?
// Block = NG gather waves (random 128-B rows from a 2 MB window, 8 lanes x
// 16 B, 8 loads in flight per lane: the SpMM's X gather) + NS streamer waves.
// Streamer kind 0: 64-B scalar loads (NB in flight), each wave its own
// sequential region; kind 1: 16-B-per-lane vector loads (8 in flight).  Every
// wave runs for the same wall-clock time (s_memrealtime) and counts its work.
//   sq_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int i16v __attribute__((ext_vector_type(16)));

template <int NB>
__device__ __forceinline__ void sload_batch(const char *pv)
{
    const uint64_t a = (uint64_t)pv;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const char *p = (const char *)(((uint64_t)hi << 32) | lo);
    i16v r[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(r[b]) : "s"(p), "n"(b * 64));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("" ::"s"(r[b]));
}

template <int KIND, int NB>
__global__ void k_sq(const double *__restrict__ X, const char *__restrict__ Z, uint64_t zbytes, int NG, int NS,
                     long long ticks, unsigned long long *__restrict__ cnt, double *__restrict__ out)
{
    const int lane = threadIdx.x & 63, p = lane & 7, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(X), (short)0, (int)(16384u * 128u), 0x00020000);
    uint32_t h = (blockIdx.x * 512 + threadIdx.x) / 8 * 2654435761u + 11u;
    double a0 = 0, a1 = 0;
    unsigned long long glines = 0, rbytes = 0;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    if (w >= NG) {
        const uint64_t nsw = (uint64_t)gridDim.x * NS, wid = (uint64_t)blockIdx.x * NS + (w - NG);
        const uint64_t part = zbytes / nsw & ~(uint64_t)4095;
        const char *zb = Z + wid * part;
        uint64_t pos = 0;
        if constexpr (KIND == 0) {
            while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
                sload_batch<NB>(zb + pos);
                pos = (pos + NB * 64) % (part - NB * 64);
                rbytes += NB * 64;
            }
        } else {
            const __amdgpu_buffer_rsrc_t zr =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(zb), (short)0, (int)part, 0x00020000);
            while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
                double2 xs[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const uint32_t off = (uint32_t)((pos + t * 1024u) % part) + 16u * lane;
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(zr, off, 0, 0);
                    __builtin_memcpy(&xs[t], &v, 16);
                }
#pragma unroll
                for (int t = 0; t < 8; ++t) { a0 += xs[t].x; a1 += xs[t].y; }
                pos += 8 * 1024;
                rbytes += 8 * 1024;
            }
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
    if (a0 == 12345.0) out[0] = a1;
    if (lane == 0) {
        atomicAdd(&cnt[0], glines);
        atomicAdd(&cnt[1], rbytes);
    }
}

int main()
{
    double *X, *out;
    char *Z;
    unsigned long long *cnt;
    const uint64_t zbytes = 16ull << 30;  // 16 GB: no stream repeats in 2 ms
    hipMalloc(&X, (size_t)16384 * 128); hipMemset(X, 0, (size_t)16384 * 128);
    hipMalloc(&Z, zbytes); hipMemset(Z, 0, zbytes);
    hipMalloc(&out, 64); hipMalloc(&cnt, 16);
    const long long ticks = 200000;  // 2 ms at 100 MHz
    struct Cfg { int kind, nb, NG, NS, bpc; };
    std::vector<Cfg> cfgs = {
        {0, 4, 4, 0, 4},                                  // gathers alone
        {0, 4, 0, 1, 4}, {0, 4, 0, 2, 4}, {0, 4, 0, 4, 4}, // scalar streams alone (4, 8, 16 waves / CU)
        {0, 6, 0, 4, 4}, {0, 2, 0, 4, 4},
        {1, 4, 0, 1, 4}, {1, 4, 0, 2, 4},                 // vector streams alone
        {0, 4, 4, 1, 4}, {0, 4, 4, 2, 4}, {0, 6, 4, 2, 4}, // gathers + scalar streams on the same CU
        {1, 4, 4, 1, 4}, {1, 4, 4, 2, 4},                 // gathers + vector streams on the same CU
    };
    for (Cfg c : cfgs) {
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(cnt, 0, 16);
            const dim3 grid(256 * c.bpc), blk(64 * (c.NG + c.NS));
            if (c.kind == 1) hipLaunchKernelGGL((k_sq<1, 4>), grid, blk, 0, 0, X, Z, zbytes, c.NG, c.NS, ticks, cnt, out);
            else if (c.nb == 2) hipLaunchKernelGGL((k_sq<0, 2>), grid, blk, 0, 0, X, Z, zbytes, c.NG, c.NS, ticks, cnt, out);
            else if (c.nb == 6) hipLaunchKernelGGL((k_sq<0, 6>), grid, blk, 0, 0, X, Z, zbytes, c.NG, c.NS, ticks, cnt, out);
            else hipLaunchKernelGGL((k_sq<0, 4>), grid, blk, 0, 0, X, Z, zbytes, c.NG, c.NS, ticks, cnt, out);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            unsigned long long hc[2];
            hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost);
            if (rep)
                printf("%s nb %d  gather waves %d + streamers %d per block, %d blocks/CU : gather %6.1f G lines/s  stream %.2f TB/s\n",
                       c.kind ? "vector" : "scalar", c.nb, c.NG, c.NS, c.bpc, hc[0] / 2e-3 / 1e9, hc[1] / 2e-3 / 1e12);
        }
    }
    return 0;
}
