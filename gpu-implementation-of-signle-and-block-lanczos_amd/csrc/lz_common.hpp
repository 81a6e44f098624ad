// lz_common.hpp -- shared definitions of liblz_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "lz_hip.h"

namespace lz {

class Comm;  // lz_comm.hpp

// thread-local last error (lz_last_error)
void set_error(const char *fmt, ...);

#define LZ_HIP_TRY(expr)                                                          \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess) {                                                   \
            ::lz::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,          \
                            hipGetErrorString(e_));                               \
            return LZ_E_HIP;                                                      \
        }                                                                         \
    } while (0)

#define LZ_ARG_CHECK(cond, msg)                                                   \
    do {                                                                          \
        if (!(cond)) {                                                            \
            ::lz::set_error("argument error: %s (%s)", msg, #cond);             \
            return LZ_E_ARG;                                                      \
        }                                                                         \
    } while (0)

#define LZ_LAUNCH_CHECK()                                                         \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) {                                                   \
            ::lz::set_error("%s:%d kernel launch -> %s", __FILE__, __LINE__,      \
                            hipGetErrorString(e_));                               \
            return LZ_E_HIP;                                                      \
        }                                                                         \
    } while (0)

#define LZ_TRY(expr)                                                              \
    do {                                                                          \
        int rc_ = (expr);                                                         \
        if (rc_ != LZ_OK) return rc_;                                             \
    } while (0)

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kMaxPartials = 2048;  // per-workgroup partial b x b slabs kept in the handle
constexpr int kMaxB = 64;

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace lz

// The opaque handle (lz_handle in the C ABI).
struct lz_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    // a second stream for one-workgroup kernels that overlap a streaming pass
    // (the b = 32 sqrtm beside the next SpMM), joined back by events
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int n_cu = 256;
    int grid_cap = 0;  // > 0: at most this many blocks for kernels whose blocks wait on each other
    // device workspace: per-workgroup partial b x b sums (double), b x b
    // scratch matrices and a few scalars.
    double *partials = nullptr;   // per-workgroup / per-tile slabs (grown on demand)
    size_t partials_cap = 0;      // doubles
    double *partials2 = nullptr;  // first-level folded slabs: 256 * kMaxB * kMaxB doubles
    double *scratch = nullptr;    // 8 * kMaxB * kMaxB doubles
    int *err_flag = nullptr;      // device: nonzero if a persistent kernel gave up a bounded spin
    lz::Comm *comm = nullptr;     // lz_comm_init (RCCL) or lz_comm_init_local (virtual ranks)
    int nranks = 1, rank = 0;
    // the Krylov-block exchange of the distributed iteration runs on its own
    // stream, beside the interior rows' pass 1 (ev_cx: main -> exchange stream,
    // ev_xd: exchange done -> main)
    hipStream_t xstream = nullptr;
    hipEvent_t ev_cx = nullptr, ev_xd = nullptr;
    hipEvent_t ev_bd = nullptr;  // the wavefront step's second boundary launch (exchange stream) -> main
    int64_t last_split[2] = {-1, -1};  // lz_debug_last_split
    int last_wf = 0, last_wf_pre = 0;  // lz_debug_last_wf: wavefront step, pass-2-first overlap
    // lz_block_lanczos leaves Q0 = Q1 = Q_{m-1}, W = W_m as the reference does
    // (one row-local pass per solve); lz_set_final_state(h, 0) skips that pass
    int final_state = 1;
    int dbg_setup_fail = 0;       // lz_debug_fail_next_setup: the next distributed set-up's forced status
    // fixed-nnz SpMM format (experiment, lz_spmm.hip fnz_prepare): the operator's
    // columns with row-end flags and each tile's first row, keyed by the operator
    void *c16buf = nullptr;       // pass 1's 16-bit columns (col16_plan), nnz int16
    size_t c16_cap = 0;           // bytes
    int32_t *fnz_colf = nullptr, *fnz_trow = nullptr;
    int64_t fnz_key[4] = {0, 0, 0, 0};
    bool fnz_ok = false;
    // wavefront step (lz_wf.hip): per-tile dependency ranges (int2) and
    // pass-2 tile flags, T + 64 entries each
    void *wf_deps = nullptr;
    int *wf_flags = nullptr;
    size_t wf_cap = 0;
    void *ybuf = nullptr;         // distributed generic-b iteration: the local SpMM result
    size_t ybuf_cap = 0;          // bytes
    void *halo = nullptr;         // lz::HaloPlan when lz_halo_init was called
    uint64_t *pairs = nullptr;    // per-16-row-strip row order by length (k_strip_pairs)
    int *longq = nullptr;         // k_spmm_seg long-tile queue: [0], [1] counts (alternate calls), [2..] tile ids
    size_t longq_cap = 0;         // ints
    int longq_parity = 0;         // the count slot of the next call
    // the long-tile pass of a planned SpMM (the list an earlier call of the
    // same solve queued) runs on its own stream beside the tile pass
    hipStream_t lstream = nullptr;
    hipEvent_t ev_lfork = nullptr, ev_ljoin = nullptr;
    // CU-partitioned SpMM (LZ_SPMM_PF, lz_spmm.hip launch_seg_pf): the tile
    // kernel's and the prefetch kernel's CU-masked streams, their fork / join
    // events, the control words, the mask split they were made for
    hipStream_t pf_sg = nullptr, pf_sp = nullptr;
    hipEvent_t ev_pff = nullptr, ev_pfg = nullptr, ev_pfp = nullptr;
    int *pf_ctl = nullptr;
    int pf_key = -1;
    int pf_band = 0;                 // the operator's max |column - row| (k_band), for pf_band_key
    int64_t pf_band_key[3] = {0, 0, -1};
    size_t pairs_cap = 0;         // entries
    void *cm_buf = nullptr;       // column-major SpMM: row-major copies of X and Y
    size_t cm_cap = 0;            // bytes
    // optional per-kernel-class timing with hipEvents on the handle's stream
    // (lz_prof_enable / lz_prof_read): events recorded around each launch of
    // the class, elapsed times summed at read time.
    bool prof = false;
    unsigned prof_mask = ~0u;     // classes recorded while prof is on
    hipEvent_t *ev_pool = nullptr;
    int ev_cap = 0, ev_used = 0;
    int ev_class[4096];
};

namespace lz {
enum ProfClass { PROF_SPMM_PASS = 0, PROF_UPDATE_PASS = 1, PROF_SMALL = 2, PROF_GRAM = 3,
                 PROF_TSMM = 4, PROF_SPMM = 5, PROF_NCLASS = 6 };
// bracket one launch: returns the event index of the start (-1 when off)
int prof_begin(lz_handle *h, int cls);
// grow h->partials to hold at least `doubles` (outside any timed/captured loop)
int ensure_partials(lz_handle *h, size_t doubles);
void prof_end(lz_handle *h, int idx);
}  // namespace lz
