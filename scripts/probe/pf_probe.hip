// Timing of the per-wave prefetching fused pass (k_fused_pf16) with the X
// gathers and/or the HBM streams masked (dbg bits), and vs grid size.
#define lz lzprobe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_fused.hip"
#undef lz
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
    int64_t *drp; int32_t *dcol; double *dval, *W, *Q, *Wn, *bi, *be, *qrow, *part;
    hipMalloc(&drp, (n + 1) * 8); hipMalloc(&dcol, nnz * 4); hipMalloc(&dval, nnz * 8);
    hipMalloc(&W, n * 128); hipMalloc(&Q, n * 128); hipMalloc(&Wn, n * 128);
    hipMalloc(&bi, 2048); hipMalloc(&be, 2048); hipMalloc(&qrow, 128); hipMalloc(&part, 4096 * 8 * 2048);
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
    const int grids[] = {512, 256};
    const int dbgs[] = {0, 1, 2, 3, 7};
    for (int unr : {4, 8})
    for (int grid : grids)
        for (int dbg : dbgs) {
            float best = 1e9;
            for (int it = 0; it < 4; ++it) {
                hipEventRecord(e0);
                if (unr == 4)
                    hipLaunchKernelGGL(lzprobe::k_fused_pf16<4>, dim3(grid), dim3(512), 0, 0, n, drp, dcol, dval, W, n,
                                       W, Q, Wn, bi, be, (int64_t)-1, qrow, part, dbg);
                else
                    hipLaunchKernelGGL(lzprobe::k_fused_pf16<8>, dim3(grid), dim3(512), 0, 0, n, drp, dcol, dval, W, n,
                                       W, Q, Wn, bi, be, (int64_t)-1, qrow, part, dbg);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (it && ms < best) best = ms;
            }
            printf("UNR=%d grid=%d dbg=%d (gather %s, streams %s, stores %s): %.3f ms\n", unr, grid, dbg, dbg & 1 ? "off" : "on",
                   dbg & 2 ? "off" : "on", dbg & 4 ? "off" : dbg & 8 ? "nt" : "on", best);
        }
    return 0;
}
