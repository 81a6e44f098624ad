// Loader / consumer wait breakdown of k_spmm_ws on the C3 operator.
#define LZ_WS_PROBE 1
#define lz lzprobe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_spmm.hip"
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

template <int NC, int KS, int D, int CAP>
static void run(int64_t n, const int64_t *drp, const int32_t *dcol, const double *dval, const double *X, double *Y,
                int *err, long long *rec, int bpc)
{
    const int grid = 256 * bpc;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int it = 0; it < 2; ++it) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((lzprobe::k_spmm_ws<NC, KS, D, CAP>), dim3(grid), dim3(64 * (NC + 1)), 0, 0, n, drp, dcol,
                           dval, X, Y, err);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(grid * 8);
    hipMemcpy(h.data(), rec, grid * 64, hipMemcpyDeviceToHost);
    double s[6] = {0};
    for (int b = 0; b < grid; ++b) for (int j = 0; j < 6; ++j) s[j] += h[8 * b + j];
    long long w0 = h[6], w1 = h[7], smin = h[6], smax = h[6];
    for (int b = 0; b < grid; ++b) {
        w0 = std::min(w0, h[8 * b + 6]); w1 = std::max(w1, h[8 * b + 7]);
        smax = std::max(smax, h[8 * b + 6]);
    }
    printf("  wall: span %.3f ms, last block start at +%.3f ms, in-kernel clock %.2f GHz\n", (w1 - w0) / 1e5,
           (smax - w0) / 1e5, s[3] / grid / ((double)(w1 - w0) / 1e8) / 1e9);
    printf("NC=%d K=%d D=%d CAP=%d bpc=%d: %.3f ms; per block avg: loader total %.0f cyc, consumer0 total %.0f "
           "(ready-wait %.0f, gather %.0f over %.0f steps = %.0f cyc/step), tiles %.1f\n", NC, KS, D, CAP, bpc, ms,
           s[4] / grid, s[3] / grid, s[2] / grid, s[1] / grid, s[0] / grid, s[1] / s[0], s[5] / grid);
}

int main(int argc, char **argv)
{
    const int64_t n = 10000000, hw = argc > 1 ? atoll(argv[1]) : 4096;
    std::vector<int64_t> rp(n + 1);
    const int64_t nnz = lzh_gen_banded_count(n, 10.0, hw, 20261015ull, rp.data());
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    lzh_gen_banded_fill(n, 10.0, hw, 20261015ull, rp.data(), col.data(), val.data(), nullptr);
    int64_t *drp; int32_t *dcol; double *dval, *X, *Y; int *err; long long *rec;
    hipMalloc(&drp, (n + 1) * 8); hipMalloc(&dcol, nnz * 4); hipMalloc(&dval, nnz * 8);
    hipMalloc(&X, n * 128); hipMalloc(&Y, n * 128); hipMalloc(&err, 64); hipMalloc(&rec, 4096 * 64);
    hipMemcpy(drp, rp.data(), (n + 1) * 8, hipMemcpyHostToDevice);
    hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemcpy(dval, val.data(), nnz * 8, hipMemcpyHostToDevice);
    hipMemset(X, 0, n * 128); hipMemset(err, 0, 64);
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_probe), &rec, sizeof(rec));
    run<8, 4, 3, 1784>(n, drp, dcol, dval, X, Y, err, rec, 1);
    run<8, 3, 2, 1784>(n, drp, dcol, dval, X, Y, err, rec, 1);
    run<12, 3, 2, 2680>(n, drp, dcol, dval, X, Y, err, rec, 1);
    run<15, 3, 2, 3360>(n, drp, dcol, dval, X, Y, err, rec, 1);
    int e; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    printf("err=%d\n", e);
    return 0;
}
