// Which CUs does a stream made by hipExtStreamCreateWithCUMask run on?
// For a few masks, launch 4096 blocks that each record (XCC id, HW_ID) and
// count the distinct CUs per XCC.  Mask layouts tried:
//   all            every bit set
//   lo(k)          bit i set when (i / 8) % 8 <  k  -- if bit i is CU i / 8 of XCC i % 8
//   hi(k)          the complement of lo(k)
//   low32          bits 0..31 only (the first 32 CUs in the runtime's order)
// Then the pair lo(2) / hi(2) is launched together (two streams) to check
// that both kernels run at the same time on disjoint CUs.
//   hipcc -O3 --offload-arch=gfx950 cumask_probe.hip -o cumask_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(uint32_t *out, long long spin)
{
    if (threadIdx.x == 0) {
        const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 15u;  // HW_REG_XCC_ID
        const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));         // HW_REG_HW_ID
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
        out[3 * blockIdx.x] = xcc;
        out[3 * blockIdx.x + 1] = hw;
        out[3 * blockIdx.x + 2] = (uint32_t)(__builtin_amdgcn_s_memrealtime() & 0xffffffffu);
    }
}

static void report(const char *name, const std::vector<uint32_t> &h, int nb)
{
    std::set<uint32_t> cus[16];
    for (int b = 0; b < nb; ++b) {
        const uint32_t xcc = h[3 * b], hw = h[3 * b + 1];
        const uint32_t cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
        cus[xcc & 15].insert(se * 32 + sh * 16 + cu);
    }
    printf("%-10s CUs per XCC:", name);
    int tot = 0;
    for (int x = 0; x < 8; ++x) {
        printf(" %zu", cus[x].size());
        tot += (int)cus[x].size();
    }
    printf("  (total %d)  XCC0 se/cu:", tot);
    for (uint32_t v : cus[0]) printf(" %u.%u", v / 32, v % 32);
    printf("\n");
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("multiProcessorCount %d\n", ncu);
    const int nb = 4096;
    uint32_t *d;
    hipMalloc(&d, sizeof(uint32_t) * 3 * nb * 2);
    std::vector<uint32_t> h(3 * nb * 2);
    auto mask_of = [&](int kind, int k) {
        std::vector<uint32_t> m(8, 0);
        for (int i = 0; i < 256; ++i) {
            bool on = false;
            if (kind == 0) on = true;
            if (kind == 1) on = (i / 8) % 8 < k;
            if (kind == 2) on = (i / 8) % 8 >= k;
            if (kind == 3) on = i < 32;
            if (on) m[i / 32] |= 1u << (i % 32);
        }
        return m;
    };
    struct M { const char *name; int kind, k; };
    std::vector<M> ms = {{"all", 0, 0}, {"lo(2)", 1, 2}, {"hi(2)", 2, 2}, {"lo(1)", 1, 1}, {"hi(1)", 2, 1}, {"low32", 3, 0}};
    for (auto &mm : ms) {
        auto m = mask_of(mm.kind, mm.k);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, 8, m.data()) != hipSuccess) {
            printf("%s: hipExtStreamCreateWithCUMask failed\n", mm.name);
            continue;
        }
        std::vector<uint32_t> got(8);
        hipExtStreamGetCUMask(s, 8, got.data());
        hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d, 200LL);
        hipStreamSynchronize(s);
        hipMemcpy(h.data(), d, sizeof(uint32_t) * 3 * nb, hipMemcpyDeviceToHost);
        report(mm.name, h, nb);
        printf("           mask back: %08x %08x ...\n", got[0], got[1]);
        hipStreamDestroy(s);
    }
    // the complementary pair at once: both kernels spin 1 ms per block
    auto m1 = mask_of(1, 2), m2 = mask_of(2, 2);
    hipStream_t s1, s2;
    hipExtStreamCreateWithCUMask(&s1, 8, m1.data());
    hipExtStreamCreateWithCUMask(&s2, 8, m2.data());
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s1, d, 100000LL);
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s2, d + 3 * nb, 100000LL);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, sizeof(uint32_t) * 3 * nb * 2, hipMemcpyDeviceToHost);
    uint32_t a0 = ~0u, a1 = 0, b0 = ~0u, b1 = 0;
    for (int b = 0; b < nb; ++b) {
        a0 = std::min(a0, h[3 * b + 2]); a1 = std::max(a1, h[3 * b + 2]);
        b0 = std::min(b0, h[3 * nb + 3 * b + 2]); b1 = std::max(b1, h[3 * nb + 3 * b + 2]);
    }
    printf("pair: lo(2) ends %u..%u, hi(2) ends %u..%u (100 MHz ticks): %s\n", a0, a1, b0, b1,
           (b0 < a1 && a0 < b1) ? "overlapping" : "serial");
    std::vector<uint32_t> hh(h.begin(), h.begin() + 3 * nb), hb(h.begin() + 3 * nb, h.end());
    report("pair lo(2)", hh, nb);
    report("pair hi(2)", hb, nb);
    return 0;
}
