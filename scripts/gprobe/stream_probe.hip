// STREAM-style HBM ceilings on MI355X for the access mixes this build's passes
// use ("verify [the 8 TB/s nominal] with a STREAM-copy
// measurement on the box").  Arrays of 2 GiB each (far past the 256 MB
// Infinity Cache), 16-B accesses, grid-stride, U = 4 or 8 independent 16-B
// accesses in flight per lane per array, 256-thread blocks, 8 or 16 per CU:
//   read     sum of one array                      (EL-like: reads only)
//   write    fill one array                        (stores only)
//   copy     b = a                                 (1 read : 1 write)
//   r2w1     c = a + b                             (pass UB: 2 reads : 1 write)
//   r3w2     d = a + b + c, e = a - b              (the wavefront step's streams: 3 : 2)
//   r3w3     d = a + b, e = b + c, f = a + c       (the post-call state pass: 3 : 3)
// each with the default cache policy and with non-temporal (nt) loads and stores.
// Bytes moved / time (median of 7 after 2 warm-ups), HIP events.
//   hipcc -O3 --offload-arch=gfx950 stream_probe.hip -o stream_probe && ./stream_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4 *p, f4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int R, int W, bool NT, int U>
__global__ __launch_bounds__(256) void k_mix(int64_t n4, const f4 *__restrict__ a, const f4 *__restrict__ b,
                                             const f4 *__restrict__ c, f4 *__restrict__ d, f4 *__restrict__ e,
                                             f4 *__restrict__ f, float *__restrict__ sink)
{
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x); i0 < n4; i0 += stride) {
        f4 x[U], y[U], z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * gridDim.x * 256;
            const bool ok = i < n4;
            const f4 zero = {0.f, 0.f, 0.f, 0.f};
            x[u] = (R >= 1 && ok) ? ld<NT>(a + i) : zero;
            y[u] = (R >= 2 && ok) ? ld<NT>(b + i) : zero;
            z[u] = (R >= 3 && ok) ? ld<NT>(c + i) : zero;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * gridDim.x * 256;
            if (i >= n4) continue;
            if constexpr (W == 0) {
                acc += x[u] + y[u] + z[u];
            } else if constexpr (R == 0) {
                const f4 v = {(float)i, 1.f, 2.f, 3.f};
                st<NT>(d + i, v);
            } else {
                st<NT>(d + i, x[u] + y[u] + z[u]);
                if constexpr (W >= 2) st<NT>(e + i, x[u] - y[u]);
                if constexpr (W >= 3) st<NT>(f + i, x[u] + z[u]);
            }
        }
    }
    if constexpr (W == 0)
        if (acc.x == 12345.678f) sink[0] = acc.y;  // keep the loads
}

template <int R, int W, bool NT, int U = 4>
static void run(const char *name, int64_t n4, f4 *const *buf, float *sink, int grid)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ms;
    for (int it = 0; it < 9; ++it) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_mix<R, W, NT, U>), dim3(grid), dim3(256), 0, 0, n4, buf[0], buf[1], buf[2], buf[3], buf[4],
                           buf[5], sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float t = 0;
        hipEventElapsedTime(&t, e0, e1);
        if (it >= 2) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double t = ms[ms.size() / 2] * 1e-3;
    const double bytes = (double)n4 * 16.0 * (R + W);
    std::printf("%-6s %-7s U %d grid %5d %6.2f GB in %8.3f ms = %5.2f TB/s (min %.3f, max %.3f ms)\n", name,
                NT ? "nt" : "default", U, grid, bytes / 1e9, t * 1e3, bytes / t / 1e12, ms.front(), ms.back());
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main()
{
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t bytes = 2LL << 30, n4 = bytes / 16;
    f4 *buf[6];
    for (auto &p : buf) {
        if (hipMalloc(&p, bytes) != hipSuccess) {
            std::printf("hipMalloc failed\n");
            return 1;
        }
        hipMemset(p, 0, bytes);
    }
    float *sink;
    hipMalloc(&sink, 64);
    hipDeviceSynchronize();
    std::printf("%d CUs, 256-thread blocks, arrays of %.1f GiB\n", cus, bytes / double(1 << 30));
    for (int g : {cus * 8, cus * 16}) {
        run<1, 0, false, 4>("read", n4, buf, sink, g);
        run<1, 0, true, 4>("read", n4, buf, sink, g);
        run<1, 0, true, 8>("read", n4, buf, sink, g);
        run<0, 1, false, 4>("write", n4, buf, sink, g);
        run<0, 1, true, 4>("write", n4, buf, sink, g);
        run<0, 1, false, 8>("write", n4, buf, sink, g);
        run<1, 1, false, 4>("copy", n4, buf, sink, g);
        run<1, 1, true, 4>("copy", n4, buf, sink, g);
        run<1, 1, false, 8>("copy", n4, buf, sink, g);
        run<2, 1, false, 4>("r2w1", n4, buf, sink, g);
        run<2, 1, true, 4>("r2w1", n4, buf, sink, g);
        run<2, 1, false, 8>("r2w1", n4, buf, sink, g);
        run<2, 1, true, 8>("r2w1", n4, buf, sink, g);
        run<3, 2, false, 4>("r3w2", n4, buf, sink, g);
        run<3, 2, false, 8>("r3w2", n4, buf, sink, g);
        run<3, 3, false, 4>("r3w3", n4, buf, sink, g);
        run<3, 3, false, 8>("r3w3", n4, buf, sink, g);
    }
    for (auto p : buf) hipFree(p);
    hipFree(sink);
    return 0;
}
