// Loader / consumer wait breakdown of the wave-specialised fused pass (k_fused_ws16).
#define LZ_WS_PROBE 1
#define lz lzprobe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_fused.hip"
#undef lz
#include <algorithm>
#include <vector>
#include "lz_host.h"
namespace lzprobe {
void set_error(const char *, ...) {}
int prof_begin(lz_handle *, int) { return -1; }
void prof_end(lz_handle *, int) {}
int ensure_partials(lz_handle *, size_t) { return 0; }
}  // namespace lzprobe

template <int NC, int CAP, int KS, bool QREG = false>
static void run(int64_t n, const int64_t *drp, const int32_t *dcol, const double *dval, const double *W, double *Q,
                double *Wn, const double *bi, const double *be, double *qrow, double *part, int *err, long long *rec)
{
    const int grid = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((lzprobe::k_fused_ws16<NC, CAP, KS, QREG>), dim3(grid), dim3(64 * (NC + 1)), 0, 0, n, drp, dcol, dval,
                           W, n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part, err);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(grid * 8);
    hipMemcpy(h.data(), rec, grid * 64, hipMemcpyDeviceToHost);
    double s[6] = {0};
    for (int b = 0; b < grid; ++b) for (int j = 0; j < 6; ++j) s[j] += h[8 * b + j];
    printf("NC=%d CAP=%d K=%d QREG=%d: %.3f ms; per block: loader %.0f cyc (done-wait %.0f); consumer0 %.0f (ready-wait %.0f, "
           "gather %.0f); tiles %.1f\n", NC, CAP, KS, (int)QREG, ms, s[4] / grid, s[1] / grid, s[3] / grid, s[2] / grid, s[0] / grid,
           s[5] / grid);
}

int main()
{
    const int64_t n = 10000000;
    std::vector<int64_t> rp(n + 1);
    const int64_t nnz = lzh_gen_banded_count(n, 10.0, 4096, 20261015ull, rp.data());
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    lzh_gen_banded_fill(n, 10.0, 4096, 20261015ull, rp.data(), col.data(), val.data(), nullptr);
    int64_t *drp; int32_t *dcol; double *dval, *W, *Q, *Wn, *bi, *be, *qrow, *part; int *err; long long *rec;
    hipMalloc(&drp, (n + 1) * 8); hipMalloc(&dcol, nnz * 4); hipMalloc(&dval, nnz * 8);
    hipMalloc(&W, n * 128); hipMalloc(&Q, n * 128); hipMalloc(&Wn, n * 128);
    hipMalloc(&bi, 2048); hipMalloc(&be, 2048); hipMalloc(&qrow, 128); hipMalloc(&part, 256 * 16 * 2048);
    hipMalloc(&err, 64); hipMalloc(&rec, 4096 * 64);
    hipMemcpy(drp, rp.data(), (n + 1) * 8, hipMemcpyHostToDevice);
    hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemcpy(dval, val.data(), nnz * 8, hipMemcpyHostToDevice);
    hipMemset(W, 0, n * 128); hipMemset(Q, 0, n * 128); hipMemset(err, 0, 64);
    std::vector<double> eye(256, 0.0);
    for (int i = 0; i < 16; ++i) eye[i * 17] = 1.0;
    hipMemcpy(bi, eye.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(be, eye.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_probe), &rec, sizeof(rec));
    // dbg masks (timing only): 1 = no Q DMA, 4 = no stores, 8 = no gathers
    for (int dbg : {0, 8}) {
        hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_dbg), &dbg, sizeof(dbg));
        printf("dbg=%2d (gathers %s)\n  ", dbg, dbg & 8 ? "off" : "on");
        run<15, 2536, 2>(n, drp, dcol, dval, W, Q, Wn, bi, be, qrow, part, err, rec);
        printf("  ");
        run<15, 2536, 3, true>(n, drp, dcol, dval, W, Q, Wn, bi, be, qrow, part, err, rec);
    }
    int e; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    printf("err=%d\n", e);
    return 0;
}
