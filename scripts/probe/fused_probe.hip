// Phase timing of k_fused_spmm16 on the C3 operator (build: scripts/probe/Makefile).
// Compiled under a private namespace so its kernels cannot alias liblz_hip.so's.
#define LZ_FUSED_PROBE 1
#define lz lzprobe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_fused.hip"
#undef lz
#include <algorithm>
#include <cstdlib>
#include <vector>
#include "lz_host.h"
namespace lzprobe {
void set_error(const char *, ...) {}
int prof_begin(lz_handle *, int) { return -1; }
void prof_end(lz_handle *, int) {}
int ensure_partials(lz_handle *, size_t) { return 0; }
}  // namespace lzprobe

int main(int argc, char **argv)
{
    const int64_t n = argc > 1 ? (int64_t)atof(argv[1]) : 10000000;
    const int64_t hw = argc > 2 ? atoll(argv[2]) : 4096;
    std::vector<int64_t> rp(n + 1);
    const int64_t nnz = lzh_gen_banded_count(n, 10.0, hw, 20261015ull, rp.data());
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    lzh_gen_banded_fill(n, 10.0, hw, 20261015ull, rp.data(), col.data(), val.data(), nullptr);
    int64_t *drp; int32_t *dcol; double *dval, *W, *Q, *Wn, *bi, *be, *qrow, *part;
    const int64_t tiles = (n + 127) / 128;
    hipMalloc(&drp, (n + 1) * 8); hipMalloc(&dcol, nnz * 4); hipMalloc(&dval, nnz * 8);
    hipMalloc(&W, n * 128); hipMalloc(&Q, n * 128); hipMalloc(&Wn, n * 128);
    hipMalloc(&bi, 256 * 8); hipMalloc(&be, 256 * 8); hipMalloc(&qrow, 16 * 8); hipMalloc(&part, tiles * 256 * 8);
    hipMemcpy(drp, rp.data(), (n + 1) * 8, hipMemcpyHostToDevice);
    hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemcpy(dval, val.data(), nnz * 8, hipMemcpyHostToDevice);
    hipMemset(W, 0, n * 128); hipMemset(Q, 0, n * 128);
    std::vector<double> eye(256, 0.0);
    for (int i = 0; i < 16; ++i) eye[i * 17] = 1.0;
    hipMemcpy(bi, eye.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(be, eye.data(), 2048, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    long long *rec;
    hipMalloc(&rec, tiles * 64);
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_fused_probe), &rec, sizeof(rec));
    std::vector<long long> h(tiles * 8);
    for (int it = 0; it < 3; ++it) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(lzprobe::k_fused_spmm16<true>, dim3((unsigned)tiles), dim3(512), 0, 0, n, drp, dcol, dval,
                           W, n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h.data(), rec, tiles * 64, hipMemcpyDeviceToHost);
        double s0 = 0, s1 = 0, s2 = 0;
        long long wmin = h[3], wmax = h[4];
        for (int64_t b = 0; b < tiles; ++b) {
            s0 += h[8 * b]; s1 += h[8 * b + 1]; s2 += h[8 * b + 2];
            wmin = std::min(wmin, h[8 * b + 3]); wmax = std::max(wmax, h[8 * b + 4]);
        }
        // residency profile: blocks alive at 20 sample points
        int alive[20] = {0};
        for (int64_t b = 0; b < tiles; ++b)
            for (int k = 0; k < 20; ++k) {
                const long long t = wmin + (wmax - wmin) * (2 * k + 1) / 40;
                alive[k] += (h[8 * b + 3] <= t && t < h[8 * b + 4]);
            }
        const double nb = (double)tiles;
        printf("n=%ld hw=%ld  %.3f ms  avg cycles: staging %.0f gather %.0f epilogue %.0f total %.0f; span %.3f ms; alive:",
               (long)n, (long)hw, ms, s0 / nb, s1 / nb, s2 / nb, (s0 + s1 + s2) / nb, (wmax - wmin) / 100e3);
        for (int k = 0; k < 20; ++k) printf(" %d", alive[k]);
        printf("\n");
    }
    return 0;
}
