// k_fused_ub32d (DMA operand staging) against k_fused_ub32 (register operands)
// on random data: the stored W'' and the slabs must be the same bits.  Prints
// where they differ (row within the 32-row strip, column, wave).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include \
//     -I../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc ub_kernel_probe.hip -o ub_kernel_probe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_fused32.hip"

#include <cstdio>
#include <random>
#include <vector>

namespace lz {  // (host helpers of the library the included file's launchers name; unused here)
int ensure_partials(lz_handle *, size_t) { return 0; }
int prof_begin(lz_handle *, int) { return -1; }
void prof_end(lz_handle *, int) {}
void set_error(const char *, ...) {}
}  // namespace lz
using namespace lz;

int main()
{
    for (int64_t n : {(int64_t)128, (int64_t)20011}) {
        std::mt19937 g(5);
        std::uniform_real_distribution<float> u(-1.f, 1.f);
        std::vector<float> hU(n * 32), hW(n * 32), hb(1024), hp(1024);
        for (auto &x : hU) x = u(g);
        for (auto &x : hW) x = u(g);
        for (auto &x : hb) x = u(g);
        for (auto &x : hp) x = u(g);
        float *U, *W, *b, *p, *o1, *o2;
        double *s1, *s2;
        const int grid = (int)std::min<int64_t>(ceil_div(n, (int64_t)128), 512);
        hipMalloc(&U, n * 128); hipMalloc(&W, n * 128); hipMalloc(&b, 4096); hipMalloc(&p, 4096);
        hipMalloc(&o1, n * 128); hipMalloc(&o2, n * 128);
        hipMalloc(&s1, (size_t)grid * 8192); hipMalloc(&s2, (size_t)grid * 8192);
        hipMemcpy(U, hU.data(), n * 128, hipMemcpyHostToDevice);
        hipMemcpy(W, hW.data(), n * 128, hipMemcpyHostToDevice);
        hipMemcpy(b, hb.data(), 4096, hipMemcpyHostToDevice);
        hipMemcpy(p, hp.data(), 4096, hipMemcpyHostToDevice);
        hipMemset(o1, 0, n * 128); hipMemset(o2, 0, n * 128);
        hipLaunchKernelGGL(k_fused_ub32<false>, dim3(grid), dim3(256), 0, 0, n, U, W, b, p, o1, s1, nullptr, nullptr);
        hipLaunchKernelGGL(k_fused_ub32d<false>, dim3(grid), dim3(256), 0, 0, n, U, W, b, p, o2, s2, nullptr, nullptr, 0);
        hipDeviceSynchronize();
        std::vector<float> r1(n * 32), r2(n * 32);
        std::vector<double> q1((size_t)grid * 1024), q2((size_t)grid * 1024);
        hipMemcpy(r1.data(), o1, n * 128, hipMemcpyDeviceToHost);
        hipMemcpy(r2.data(), o2, n * 128, hipMemcpyDeviceToHost);
        hipMemcpy(q1.data(), s1, q1.size() * 8, hipMemcpyDeviceToHost);
        hipMemcpy(q2.data(), s2, q2.size() * 8, hipMemcpyDeviceToHost);
        int64_t bad = 0, shown = 0;
        for (int64_t i = 0; i < n * 32; ++i)
            if (r1[i] != r2[i]) {
                ++bad;
                if (shown++ < 12)
                    printf("  n %ld row %ld (strip row %ld, wave %ld) col %ld: reg %g dma %g\n", (long)n, (long)(i / 32),
                           (long)(i / 32 % 32), (long)(i / 32 / 32 % 4), (long)(i % 32), r1[i], r2[i]);
            }
        int64_t sbad = 0;
        for (size_t i = 0; i < q1.size(); ++i) sbad += q1[i] != q2[i];
        printf("n %ld: %ld of %ld W'' values differ, %ld of %zu slab values\n", (long)n, (long)bad, (long)(n * 32),
               (long)sbad, q1.size());
    }
    return 0;
}
