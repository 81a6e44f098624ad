// Per-tile timeline of the wave-specialised fused pass (k_fused_ws16<15,2536,2>):
// loader DMA issue and ready stamps, each consumer's start (after its ready
// wait) and end, for block 0-3, tiles < 256.
#define LZ_WS_PROBE 1
#define LZ_WS_PROBE_TL 1
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

int main()
{
    const int64_t n = 10000000;
    std::vector<int64_t> rp(n + 1);
    const int64_t nnz = lzh_gen_banded_count(n, 10.0, 4096, 20261015ull, rp.data());
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    lzh_gen_banded_fill(n, 10.0, 4096, 20261015ull, rp.data(), col.data(), val.data(), nullptr);
    int64_t *drp; int32_t *dcol; double *dval, *W, *Q, *Wn, *bi, *be, *qrow, *part; int *err; long long *rec, *tl;
    hipMalloc(&drp, (n + 1) * 8); hipMalloc(&dcol, nnz * 4); hipMalloc(&dval, nnz * 8);
    hipMalloc(&W, n * 128); hipMalloc(&Q, n * 128); hipMalloc(&Wn, n * 128);
    hipMalloc(&bi, 2048); hipMalloc(&be, 2048); hipMalloc(&qrow, 128); hipMalloc(&part, 256 * 16 * 2048);
    hipMalloc(&err, 64); hipMalloc(&rec, 4096 * 64);
    const size_t tlb = (size_t)4 * 256 * 32 * 8;
    hipMalloc(&tl, tlb); hipMemset(tl, 0, tlb);
    hipMemcpy(drp, rp.data(), (n + 1) * 8, hipMemcpyHostToDevice);
    hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice);
    hipMemcpy(dval, val.data(), nnz * 8, hipMemcpyHostToDevice);
    hipMemset(W, 0, n * 128); hipMemset(Q, 0, n * 128); hipMemset(err, 0, 64);
    std::vector<double> eye(256, 0.0);
    for (int i = 0; i < 16; ++i) eye[i * 17] = 1.0;
    hipMemcpy(bi, eye.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(be, eye.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_probe), &rec, sizeof(rec));
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_tl), &tl, sizeof(tl));
    int dbg = getenv("TL_DBG") ? atoi(getenv("TL_DBG")) : 0;
    hipMemcpyToSymbol(HIP_SYMBOL(lzprobe::lz_ws_dbg), &dbg, sizeof(dbg));
    const bool qreg = getenv("TL_QREG") != nullptr;
    for (int it = 0; it < 3; ++it) {
        if (getenv("TL_PP"))
            hipLaunchKernelGGL((lzprobe::k_fused_pp16<14, 2376, 3, 2>), dim3(256), dim3(1024), 0, 0, n, drp, dcol,
                               dval, W, n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part, err);
        else if (getenv("TL_NL2"))
            hipLaunchKernelGGL((lzprobe::k_fused_ws16<14, 2376, 3, true, 2>), dim3(256), dim3(1024), 0, 0, n, drp,
                               dcol, dval, W, n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part, err);
        else if (qreg)
            hipLaunchKernelGGL((lzprobe::k_fused_ws16<15, 2536, 3, true>), dim3(256), dim3(1024), 0, 0, n, drp, dcol,
                               dval, W, n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part, err);
        else
            hipLaunchKernelGGL((lzprobe::k_fused_ws16<15, 2536, 2>), dim3(256), dim3(1024), 0, 0, n, drp, dcol, dval, W,
                               n, W, Q, Wn, bi, be, (int64_t)-1, qrow, part, err);
    }
    hipDeviceSynchronize();
    std::vector<long long> h(tlb / 8);
    hipMemcpy(h.data(), tl, tlb, hipMemcpyDeviceToHost);
    const int NC = (getenv("TL_NL2") || getenv("TL_PP")) ? 14 : 15;
    for (int b = 0; b < 2; ++b) {
        const long long *B = h.data() + (size_t)b * 256 * 32;
        const long long t0 = B[0];
        printf("block %d (cycles from tile-0 issue): tile issue ready | consumer start min/max end min/max | "
               "busy min/avg/max\n", b);
        double s_lat = 0, s_span = 0, s_bmax = 0, s_bavg = 0, s_period = 0;
        int cnt = 0;
        for (int i = 0; i < 160; ++i) {
            const long long *R = B + i * 32;
            long long smin = LLONG_MAX, smax = 0, emin = LLONG_MAX, emax = 0, bmin = LLONG_MAX, bmax = 0;
            double bsum = 0;
            for (int c = 0; c < NC; ++c) {
                const long long st = R[2 + 2 * c], en = R[3 + 2 * c];
                smin = std::min(smin, st); smax = std::max(smax, st);
                emin = std::min(emin, en); emax = std::max(emax, en);
                bmin = std::min(bmin, en - st); bmax = std::max(bmax, en - st); bsum += en - st;
            }
            if (i >= 10 && i < 150) {
                s_lat += R[1] - R[0]; s_span += emax - smin; s_bmax += bmax; s_bavg += bsum / NC;
                s_period += B[(i + 1) * 32] - R[0];
                ++cnt;
            }
            if (i < 8 || (i >= 40 && i < 46))
                printf("  %3d  %8lld %8lld | %8lld %8lld  %8lld %8lld | %6lld %6.0f %6lld\n", i, R[0] - t0, R[1] - t0,
                       smin - t0, smax - t0, emin - t0, emax - t0, bmin, bsum / NC, bmax);
        }
        printf("  per-consumer avg busy:");
        for (int c = 0; c < NC; ++c) {
            double sb = 0;
            for (int i = 10; i < 150; ++i) sb += B[i * 32 + 3 + 2 * c] - B[i * 32 + 2 + 2 * c];
            printf(" %.0f", sb / 140);
        }
        printf("\n");
        printf("  avg over tiles 10-149: DMA issue->ready %.0f, tile period %.0f, consumer span %.0f, busy avg %.0f max %.0f\n",
               s_lat / cnt, s_period / cnt, s_span / cnt, s_bavg / cnt, s_bmax / cnt);
    }
    if (getenv("TL_PP")) {
        std::vector<long long> r(256 * 8);
        hipMemcpy(r.data(), rec, 256 * 64, hipMemcpyDeviceToHost);
        double a[8] = {0};
        for (int b = 0; b < 256; ++b) for (int j = 0; j < 8; ++j) a[j] += r[8 * b + j];
        const double nt = a[7];
        printf("consumer0 per tile (cycles): ready-wait %.0f, offsets %.0f, step0 issue %.0f, epilogue %.0f, "
               "step0 fma(wait) %.0f, later steps %.0f, total %.0f\n", a[0] / nt, a[1] / nt, a[2] / nt, a[3] / nt,
               a[4] / nt, a[5] / nt, a[6] / nt);
    }
    return 0;
}
