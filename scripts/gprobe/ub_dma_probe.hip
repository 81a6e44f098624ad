// Layout check of k_fused_ub32d's operand staging (lz_fused32.hip): one wave
// DMAs a 32 x 32 fp32 strip into LDS with the per-lane swizzled global pieces
// (16 B per lane, 1 KB per instruction) and reads each lane's MFMA A-operands
// back (row lane & 31, floats 16 (lane >> 5) .. + 15) with ds_read_b128; the
// values must equal the strip's.  Also the same with the builtin LDS loads
// instead of inline asm, and with the per-strip buffer resource offset.
//   hipcc -O3 --offload-arch=gfx950 ub_dma_probe.hip -o ub_dma_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_t;

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char *)p;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_probe(const float *M, int64_t r0, int rows, float *out)
{
    __shared__ __attribute__((aligned(16))) float st[2][2][1024];
    const int lane = threadIdx.x & 63, hh = lane >> 5, jr = lane & 31;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(M + r0 * 32), (short)0, rows * 128, 0x00020000);
    const uint32_t goff = (uint32_t)((lane >> 3) * 128 + 16 * ((lane & 7) ^ ((lane >> 3) & 7)));
    for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t *)&st[1][0][256 * k], 16, goff + 1024 * k, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float a[16];
    if constexpr (MODE == 0) {
        const uint32_t sb = lds_addr(&st[1][0][0]), rb = (uint32_t)(jr * 128);
        float4 u4[4];
        const uint32_t o0 = sb + rb + 16u * (uint32_t)((4 * hh + 0) ^ (jr & 7)),
                       o1 = sb + rb + 16u * (uint32_t)((4 * hh + 1) ^ (jr & 7)),
                       o2 = sb + rb + 16u * (uint32_t)((4 * hh + 2) ^ (jr & 7)),
                       o3 = sb + rb + 16u * (uint32_t)((4 * hh + 3) ^ (jr & 7));
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %5\n\t"
            "ds_read_b128 %2, %6\n\t"
            "ds_read_b128 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(u4[0]), "=&v"(u4[1]), "=&v"(u4[2]), "=&v"(u4[3])
            : "v"(o0), "v"(o1), "v"(o2), "v"(o3)
            : "memory");
        for (int c = 0; c < 4; ++c) {
            a[4 * c] = u4[c].x; a[4 * c + 1] = u4[c].y; a[4 * c + 2] = u4[c].z; a[4 * c + 3] = u4[c].w;
        }
    } else {  // plain C++ LDS reads of the same positions
        __syncthreads();
        for (int c = 0; c < 4; ++c) {
            const int pos = 8 * jr + ((4 * hh + c) ^ (jr & 7));
            for (int i = 0; i < 4; ++i) a[4 * c + i] = st[1][0][4 * pos + i];
        }
    }
    for (int s = 0; s < 16; ++s) out[lane * 16 + s] = a[s];
}

int main()
{
    const int n = 100;
    std::vector<float> h(n * 32);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < 32; ++c) h[r * 32 + c] = (float)(r * 100 + c);
    float *dM, *dout;
    hipMalloc(&dM, h.size() * 4);
    hipMalloc(&dout, 64 * 16 * 4);
    hipMemcpy(dM, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> o(64 * 16);
    for (int mode = 0; mode < 2; ++mode)
        for (int r0 : {0, 32, 96}) {
            const int rows = n - r0 < 32 ? n - r0 : 32;
            hipMemset(dout, 0xff, 64 * 16 * 4);
            if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(64), 0, 0, dM, (int64_t)r0, rows, dout);
            else hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(64), 0, 0, dM, (int64_t)r0, rows, dout);
            hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
            int bad = 0, shown = 0;
            for (int lane = 0; lane < 64; ++lane)
                for (int s = 0; s < 16; ++s) {
                    const int row = lane & 31, col = 16 * (lane >> 5) + s;
                    const float want = row < rows ? (float)((r0 + row) * 100 + col) : 0.0f;
                    if (o[lane * 16 + s] != want) {
                        ++bad;
                        if (shown++ < 6) printf("  mode %d r0 %d lane %d s %d: got %g want %g\n", mode, r0, lane, s,
                                                o[lane * 16 + s], want);
                    }
                }
            printf("mode %d (%s) r0 %d rows %d: %d of 1024 wrong\n", mode, mode ? "C++ reads" : "asm reads", r0, rows, bad);
        }
    return 0;
}
