// lz_wf.hip -- the wavefront block-Lanczos step: b = 16, fp64, one GPU.
//
// The two-pass Q-free step (lz_fused.hip) runs pass 1 (the SpMM plus its MFMA
// epilogue) and pass 2 (W'' = W' - W_j P2) as separate launches, because pass
// 2 needs alpha_j, a sum over every row of pass 1's output.  Pass 1 of the
// NEXT step needs no such global value if it is written in the unnormalised
// (beta^2) form, so here one launch runs pass 2 of step j and pass 1 of step
// j + 1 together, as a wavefront over the rows:
//
//   V_j  = W''_{j-1} (unnormalised; Q_j = V_j beta_j^-1), Y_j = A V_j,
//   V_{j+1} = Y_j beta_j^-1 - V_{j-1} P1_j - V_j P2_j        (pass 2, "updaters")
//   Y_{j+1} = A V_{j+1};  S1 = V_{j+1}^T Y_{j+1}              (pass 1, "consumers")
//   G_{j+1} = V_{j+1}^T V_{j+1};  S2 = V_{j+1}^T V_j          (slabs, updaters)
//
// and after the launch (a 12-workgroup fold of the block slabs, then one
// one-workgroup kernel): beta_{j+1} = sqrtm(G),
// P1_{j+1} = beta_j^-1 beta_{j+1}, alpha_{j+1} = sym(beta^-1 (S1 beta^-1 -
// S2 P1)), P2 = beta^-1 alpha, q = V_{j+1}[lc] beta^-1.  The products are the
// reference's (methods/block_lanczos.hpp:137-165: W = A Q1 - Q0 beta,
// alpha = Q1^T W, W -= Q1 alpha, beta = sqrtm(W^T W)) reassociated:
// A Q = (A V) beta^-1, Q_{j-1} beta_j = V_{j-1} (beta_{j-1}^-1 beta_j).
//
// Bytes per step: A + 5 n b s (Y_j, V_{j-1}, V_j read; V_{j+1}, Y_{j+1}
// written) against A + 6 n b s for the two passes, and the V_{j+1} rows that
// pass 1 gathers were written a few hundred rows earlier in the same launch.
//
// One block per CU, wave-specialised: NL loaders stage pass-1 tiles' CSR runs
// (k_fused_pp16's ring), NU updaters run pass 2 on 16-row strips streamed
// into LDS slots by LDS-DMA, NC consumers gather and run the S1 epilogue.  Hand-off inside the launch (MI355X_MICROARCH.md, "Valid forms"
// table, first row): updaters store V_{j+1} write-through (16-B sc1 stores),
// drain (counted s_waitcnt vmcnt) and publish a per-tile flag with an sc1
// store; a loader polls the flags of every pass-2 tile its pass-1 tile reads
// (sc1 loads), then publishes the staged tile through its LDS ready word;
// every load of V_{j+1} is an sc1 load.  Results do not depend on placement;
// liveness needs every block resident (one block per CU, grid <= CUs), and
// every wait is bounded (a timeout sets the device error word).
#include <climits>
#include <mutex>
#include <unordered_map>

#include "lz_internal.hpp"
#include "lz_kernels.hpp"

namespace lz {

// block shapes (LZ_WF_SHAPE): 111 (default) = 1 loader + 11 consumers + 4
// updaters (one per SIMD); "NC" = 10, 11, 12 for 2 loaders + NC consumers +
// 14 - NC updaters; tiles of 16 NC rows. An updater wave is bound by its
// SIMD's MFMA pipe: at C3 2 + 13 + 1 took 3.1 ms, 2 + 12 + 2 1.93, 2 + 11 + 3
// 1.87, 2 + 10 + 4 1.86, 1 + 11 + 4 1.82, 1 + 12 + 3 1.87, 1 + 10 + 5 1.94
// (scripts/ab_c3.py); one loader wave keeps up with 11 consumers.
constexpr int kWfK = 3, kWfNL = 2;
constexpr int kWfCapPerRow = 11;  // stage entries per row (C3: 10 +- 2.2 nnz per row)
// the wide shape (rows of up to ~27 entries on average, C4's density): 1 loader
// + 10 consumers + 2 (32-bit columns) or 3 (16-bit) updaters, two stages of
// 4400 entries (k_fused_pp16's wide stage).  At C4's per-rank share (n = 5M,
// 25 per row, half width 65,536) 2.52-2.55 ms per step against 2.67 for the
// two passes: the launch takes pass 1 + pass 2 (2.37-2.40 against 2.08 +
// 0.35), the gain is the kernels it replaces.  Its gathers miss L2 (a 16 MB
// window per XCD) and share the fabric with the updaters' streams; 2 loaders,
// or 9 consumers + 3 updaters, measured the same.
constexpr int kWfWideCap = 4400;
constexpr double kWfWideRow = 27.0;
constexpr int kWfMaxSpan = 1024;    // pass-2 tiles one pass-1 tile may read (flag polls per tile)
constexpr int kWfAux = 16;          // buffer-instruction cache policy: sc1
constexpr long kWfSpin = 1L << 21;  // flag polls per tile before the loader gives up (about 2 s)

// Once per solve, one pass over the CSR columns: per pass-1 tile t (TR rows)
// [lo, hi], the tiles holding its columns, t itself included (pass 1 of tile t
// overwrites Y rows pass 2 of tile t reads); spans[0..2] = max(t - lo),
// max(hi - t), max(hi - lo + 1); and, when col16 != null, pass 1's 16-bit
// columns (col16_plan's encoding: the offset from the row's 16-row strip),
// spans[3] != 0 if one is out of int16 reach.  Columns >= ncol (a rank's halo
// rows) are left out of the ranges.  A wave walks one strip's run
// (coalesced); one atomic per block and quantity.
// xoff: the gather-source row of local row 0 (the all-gather form's slot
// offset; 0 otherwise); own rows are [xoff, xoff + n), the others are left out
// of the ranges.  win: the gather source has 2^24+ rows, so every column must
// lie within kWinRows / 2 of its strip's own row (spans[3] bit 1 otherwise).
__global__ __launch_bounds__(256) void k_wf_deps(int64_t n, int TR, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ col, int2 *__restrict__ deps,
                                                 int16_t *__restrict__ col16, int *__restrict__ spans, int64_t xoff,
                                                 int win)
{
    __shared__ int smin[4], smax[4];
    const int64_t T = ceil_div(n, (int64_t)TR);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ns = TR / 16;
    int sb = 0, sf = 0, sw = 0, bad = 0, far = 0;  // span maxima (thread 0), int16 / window range flags
    for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
        int mn = INT_MAX, mx = -1;
        for (int s = w; s < ns; s += 4) {
            const int64_t s0 = t * TR + 16 * s;
            if (s0 >= n) break;
            const int64_t s1 = s0 + 16 < n ? s0 + 16 : n;
            for (int64_t k = rp[s0] + lane, e = rp[s1]; k < e; k += 64) {
                const int64_t c = (int64_t)col[k] - xoff;  // local row (own rows: [0, n))
                if (c >= 0 && c < n) {  // (other columns: a rank's halo / peers' slots, boundary tiles)
                    mn = c < mn ? (int)c : mn;
                    mx = c > mx ? (int)c : mx;
                }
                const int64_t d = c - s0;
                if (win) far |= (d < -(kWinRows / 2) + 32) | (d > kWinRows / 2 - 32);
                if (col16) {
                    bad |= (d < -32768) | (d > 32767);
                    col16[k] = (int16_t)d;
                }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        if (lane == 0) {
            smin[w] = mn;
            smax[w] = mx;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < 4; ++i) {
                mn = smin[i] < mn ? smin[i] : mn;
                mx = smax[i] > mx ? smax[i] : mx;
            }
            int lo = (int)t, hi = (int)t;
            if (mx >= 0) {
                const int a = (int)(mn / TR), b = (int)(mx / TR);
                lo = a < lo ? a : lo;
                hi = b > hi ? b : hi;
            }
            deps[t] = make_int2(lo, hi);
            sb = (int)t - lo > sb ? (int)t - lo : sb;
            sf = hi - (int)t > sf ? hi - (int)t : sf;
            sw = hi - lo + 1 > sw ? hi - lo + 1 : sw;
        }
        __syncthreads();
    }
    if (__ballot(bad) != 0 && lane == 0) atomicOr(&spans[3], 1);
    if (__ballot(far) != 0 && lane == 0) atomicOr(&spans[3], 2);
    if (threadIdx.x == 0) {
        atomicMax(&spans[0], sb);
        atomicMax(&spans[1], sf);
        atomicMax(&spans[2], sw);
    }
}

typedef unsigned v4u32_t __attribute__((ext_vector_type(4)));
typedef double d2_t __attribute__((ext_vector_type(2)));

// swap a double with the neighbouring lane (l ^ 1) by DPP (quad_perm 1,0,3,2)
__device__ __forceinline__ double dpp_swap1(double x)
{
    int2 v;
    __builtin_memcpy(&v, &x, 8);
    v.x = __builtin_amdgcn_mov_dpp(v.x, 0xB1, 0xF, 0xF, false);
    v.y = __builtin_amdgcn_mov_dpp(v.y, 0xB1, 0xF, 0xF, false);
    double r;
    __builtin_memcpy(&r, &v, 8);
    return r;
}

// The step kernel.  P2 == nullptr: pass 1 only (the first launch of a solve,
// on Vg = B, or a distributed rank's boundary tiles; no flags); Vj != nullptr
// there (the one-GPU solve's first launch, shapes with NU * DU * 3 >= NC):
// the consumers also sum G = Vg^T Vg over their own rows (beta_0's Gram, from
// the registers the S1 epilogue already holds) into the G slabs.  P1 ==
// nullptr: no V_{j-1} term (step 0).  Vprev and Vout may alias (V_{j+1} over
// V_{j-1}: each strip is read, then written, by one wave).  With P2, Vout is
// the gather source's own rows: Vg + 16 xoff.  part: S1 slabs at [0, G), S2
// at [G, 2G), G at [2G, 3G) (256 doubles each, one per block).
// Distributed forms: pass 1 over tiles [p1a, p1b) and pass 2 over the tiles
// [q0, q1) u [q2, q3) (a pass-2-only launch may take two ranges; with pass-1
// tiles q2 == q3); xoff = the gather-source row of local row 0 (the
// all-gather form's slot), a gather source of 2^24+ rows read through a
// per-strip window of kWinRows rows (the plan proved every column inside);
// SW: pass 2 also stores V_j's rows into Vsave (over V_{j-1}, read earlier by
// the same wave), so V_{j+1} can take V_j's place in the all-gather slot.
// GEN: the general form above; false: the one-GPU solve's launch (pass 2 over
// every tile, xoff = 0, the whole gather source below 2^24 rows, no SW), whose
// range arithmetic then folds away at compile time.
// XO, extra outputs (own instantiations, so the step launch carries none of
// their registers): 1, a solve's first launch (pass 1 only, Vj != nullptr)
// whose consumers also sum beta_0's Gram (see above); 2, the one-GPU solve's
// post-call state (a pass-2-only launch): pass 2 also stores Q = V_j beta^-1
// into Vsave and (when not null) Yo -- the reference's Q0 = Q1 = Q_{m-1} --
// beside V_m = W_m into Vout.
template <int NC, int CAP, int K, int NL, int NU, int DU, bool C16, bool SW = false, bool GEN = true, int XO = 0>
__global__ __launch_bounds__(64 * (NC + NL + NU)) void k_wf16(
    int64_t n, const int64_t *__restrict__ rp, const int32_t *__restrict__ col, const int16_t *__restrict__ col16,
    const double *__restrict__ val, const uint64_t *__restrict__ pairs, const double *Yj, const double *Vprev,
    const double *Vj, double *Vout, const double *__restrict__ binv, const double *__restrict__ P1,
    const double *__restrict__ P2, const double *Vg, double *Yo, const int2 *__restrict__ deps, int *flags, int epoch,
    int64_t hback, int lead, double *__restrict__ part, int *__restrict__ err, int dbg, int64_t nx, int64_t p1a,
    int64_t p1b, int64_t Th, int cpol, int64_t xoff, int64_t q0, int64_t q1, int64_t q2, int64_t q3, double *Vsave)
{
    using CT = typename std::conditional<C16, int16_t, int32_t>::type;
    using C = FwCfg<NC, CAP, true, true, CT>;
    constexpr int TR = C::TR;
    constexpr int GA = kWfAux, SA = kWfAux;  // gathers / V stores: sc1
    static_assert(NC > 3 && NC <= kPairPad, "strips per tile");
    __shared__ typename C::Stage st[K];
    __shared__ double scr[NC][256];     // per consumer: the parked Y tile (swizzled), then its slab
    __shared__ double ust[NU][DU + 1][3][256];  // per updater: strip slots (Y_j, V_{j-1}, V_j rows)
    __shared__ int ready[K], done[K], cons_in, upd_in;
    __shared__ int p1pub;  // pass-1 tiles this block's loaders have published
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool has_p2 = P2 != nullptr, has_prev = P1 != nullptr;
    // beta_0's Gram by the consumers (the first launch; their slabs parked in
    // the idle updaters' strip slots 1 .. DU)
    constexpr bool kG0 = XO == 1 && DU >= 1 && NU * DU * 3 >= NC;
    constexpr bool QO = XO == 2;
    const bool g0 = kG0 && !has_p2 && Vj != nullptr;
    if (threadIdx.x < K) {
        ready[threadIdx.x] = -1;
        done[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) {
        cons_in = 0;
        p1pub = 0;
        upd_in = 0;
    }
    __syncthreads();  // the only block barrier
    const int64_t T = ceil_div(n, (int64_t)TR);
    static_assert(GEN || !SW, "SW stores are a distributed form");
    static_assert(!(SW && XO == 2), "Vsave carries either V_j (SW) or Q (XO 2)");
    if constexpr (!GEN) {  // the host launches this form only for these values
        xoff = 0;
        q0 = 0;
        q1 = q2 = q3 = T;
        nx = n;
    }
    if (T != Th || blockDim.x != 64 * (NC + NL + NU) || (kG0 != (!has_p2 && Vj != nullptr))) {
        // the host planned other tiles (flags, ranges) or launched another
        // block shape (waves past the roles would index past the tile), or asked
        // a shape without the slot room for beta_0's Gram: refuse loudly
        if (threadIdx.x == 0) *err = 7;
        return;
    }
    const int64_t G = gridDim.x, bid = blockIdx.x;
    // regions: pass-1 tiles [begin, end) of region x go to the blocks b = x
    // (mod 8), interleaved; the region's pass-2 tiles are [pbeg, pend), the
    // same range moved hback tiles down, so the pass-2 wavefront leads
    // (pass-1 tiles: [p1a, p1b) -- all of them, or the interior ones of a
    // distributed rank; pass 2 covers every tile)
    // (pass-2 tiles by a virtual index v in [0, NQ): v < nq1 -> tile q0 + v,
    // else q2 + v - nq1; region bounds pbeg / pend are virtual)
    int64_t begin, end, kb, KB, pbeg, pend;
    const int64_t NP1 = p1b - p1a, nq1 = q1 - q0, NQ = nq1 + (q3 - q2);
    auto ptile = [&](int64_t v) {
        if constexpr (!GEN) return v;
        return v < nq1 ? q0 + v : q2 + (v - nq1);
    };
    auto clampq = [&](int64_t v) { return v < 0 ? (int64_t)0 : (v > NQ ? NQ : v); };
    if (G < 8) {
        begin = p1a; end = p1b; kb = bid; KB = G; pbeg = 0; pend = NQ;
    } else {
        const int64_t x = bid & 7;
        begin = p1a + NP1 * x / 8;
        end = p1a + NP1 * (x + 1) / 8;
        kb = bid >> 3;
        KB = (G - x + 7) >> 3;
        if (NP1 > 0) {  // (one pass-2 range)
            pbeg = x == 0 ? 0 : clampq(begin - hback - q0);
            pend = x == 7 ? NQ : clampq(end - hback - q0);
        } else {  // pass 2 only: the (virtual) range split evenly
            pbeg = NQ * x / 8;
            pend = NQ * (x + 1) / 8;
        }
    }
    int64_t nt = (end - begin - kb + KB - 1) / KB > 0 ? (end - begin - kb + KB - 1) / KB : 0;
    if (dbg & 4) nt = 0;  // timing diagnostics (LZ_WF_DBG): no pass-1 tiles
    auto tile_of = [&](int64_t i) { return begin + kb + i * KB; };
    if (w < NL) {
        // ------------------------------------------------------------ loaders
        __builtin_amdgcn_s_setprio(3);
        const int64_t nnz = rp[n];
        for (int64_t i = w; i < nt; i += NL) {
            const int s = (int)(i % K);
            const int64_t t = tile_of(i);
            const int64_t r0 = t * TR, r1 = (r0 + TR < n) ? r0 + TR : n;
            const int64_t kA = rp[r0];
            if (i >= K) {
                long spin = 0;
                const uint32_t da = ws_lds_addr(&done[s]);
                while (ws_lds_read(da) < NC * (int)(i / K) && ++spin < kWsSpin) __builtin_amdgcn_s_sleep(1);
                if (spin >= kWsSpin) { *err = 3; break; }
            }
            const int64_t ca = kA & ~(int64_t)(C::CPP - 1), va = kA & ~(int64_t)1;
            const int64_t cb = ((nnz - ca) * (int64_t)sizeof(CT) + 3) & ~(int64_t)3, vb = (nnz - va) * 8;
            const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int64_t *>(rp + r0), (short)0,
                                                              (int)((r1 - r0 + 1) * 8), 0x00020000);
            const CT *cbase = C16 ? reinterpret_cast<const CT *>(col16) : reinterpret_cast<const CT *>(col);
            const auto cr = __builtin_amdgcn_make_buffer_rsrc(const_cast<CT *>(cbase + ca), (short)0,
                                                              (int)(cb < 0x7fffffff ? cb : 0x7fffffff), 0x00020000);
            const auto vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(val + va), (short)0,
                                                              (int)(vb < 0x7fffffff ? vb : 0x7fffffff), 0x00020000);
            const int64_t s0i = r0 / 16, ns = (n + 15) / 16 + kPairPad;
            const auto pr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(pairs + s0i), (short)0,
                                                              (int)((ns - s0i) * 8), 0x00020000);
            if (cpol & 2) {  // streaming (nt) CSR reads
                ws_dma<2>(rr, st[s].rp, C::RP_PIECES, lane);
                ws_dma<2>(cr, st[s].col, C::COL_PIECES, lane);
                ws_dma<2>(vr, st[s].val, C::VAL_PIECES, lane);
                ws_dma<2>(pr, st[s].pr, C::PR_PIECES, lane);
            } else {
                ws_dma(rr, st[s].rp, C::RP_PIECES, lane);
                ws_dma(cr, st[s].col, C::COL_PIECES, lane);
                ws_dma(vr, st[s].val, C::VAL_PIECES, lane);
                ws_dma(pr, st[s].pr, C::PR_PIECES, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (has_p2 && !(dbg & 1)) {
                // every pass-2 tile this tile reads (and its own: its Y rows
                // are overwritten below) must have published this epoch
                const int2 d = deps[t];
                long spin = 0;
                for (int lo = d.x; lo <= d.y && spin < kWfSpin; lo += 64) {
                    const int idx = lo + lane;
                    for (;;) {
                        const int f = idx <= d.y
                                          ? __hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                          : epoch;
                        if (__ballot(f != epoch) == 0) break;
                        if (++spin >= kWfSpin) break;
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                if (spin >= kWfSpin) { *err = 5; break; }
            }
            if (lane == 0) {
                ws_lds_write(ws_lds_addr(&ready[s]), (int)i);
                asm volatile("ds_add_u32 %0, %1" ::"v"(ws_lds_addr(&p1pub)), "v"(1) : "memory");
            }
        }
        return;
    }
    if (w < NL + NU) {
        // ----------------------------------------------------------- updaters
        // Each updater streams its tiles' 16-row strips through DU + 1 LDS
        // slots (LDS-DMA: DU strips in flight without holding registers).  A
        // slot holds the strip's Y_j, V_{j-1} and V_j rows, 16-B pieces
        // XOR-swizzled (piece p of row r at p ^ ((r >> 1) & 7)), so both the
        // MFMA A-operand reads (row l & 15, pieces 2 (l >> 4) + hh) and the
        // accumulator-layout reads of V_j (row 4r + (l >> 4), column l & 15)
        // are free of bank conflicts.  The slot reads are inline asm: after an
        // LDS-DMA the compiler would put vmcnt(0) before any LDS access.
        const int uw = w - NL;
        d4_t gacc = {0.0, 0.0, 0.0, 0.0}, sacc = {0.0, 0.0, 0.0, 0.0};
        if (has_p2 && !(dbg & 2)) {
            if (dbg & 8) __builtin_amdgcn_s_setprio(0);
            else if (dbg & 64) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(2);
            const int c = lane & 15, g = lane >> 4;
            // B operands (permuted contraction order): beta^-1, -P1, -P2
            double bq[3][4];
#pragma unroll
            for (int kc = 0; kc < 4; ++kc) {
                const int idx = (4 * g + kc) * 16 + c;
                bq[0][kc] = binv[idx];
                bq[1][kc] = has_prev ? -P1[idx] : 0.0;
                bq[2][kc] = -P2[idx];
            }
            const int64_t ut0 = pbeg + kb + uw * KB, ustep = (int64_t)NU * KB;  // (virtual indices)
            const int64_t ntl = ut0 < pend ? (pend - ut0 + ustep - 1) / ustep : 0;
            const int64_t ns = ntl * NC;  // strips of this wave's tiles, in order
            const int bytes = (int)(n * 128);
            const __amdgpu_buffer_rsrc_t rs[3] = {
                __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Yj), (short)0, bytes, 0x00020000),
                __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(has_prev ? Vprev : Vj), (short)0,
                                                  has_prev ? bytes : 0, 0x00020000),
                __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Vj), (short)0, bytes, 0x00020000)};
            const auto Or = __builtin_amdgcn_make_buffer_rsrc(Vout, (short)0, bytes, 0x00020000);
            const auto Sr = __builtin_amdgcn_make_buffer_rsrc(SW || QO ? Vsave : Vout, (short)0, SW || QO ? bytes : 0,
                                                              0x00020000);
            // QO: the second Q output (Q1; out of range, so dropped, when null)
            const auto Qr = __builtin_amdgcn_make_buffer_rsrc(QO && Yo ? Yo : Vout, (short)0, QO && Yo ? bytes : 0,
                                                              0x00020000);
            auto strip_r0 = [&](int64_t s) { return ptile(ut0 + (s / NC) * ustep) * TR + 16 * (s % NC); };
            // this lane's DMA pieces: LDS piece q = 64 k + lane holds row q >> 3,
            // global piece (q & 7) ^ swizzle
            uint32_t goff[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int q = 64 * k + lane, row = q >> 3;
                goff[k] = (uint32_t)(row * 128 + 16 * ((q & 7) ^ ((row >> 1) & 7)));
            }
            // six DMA instructions per strip, always issued (out of range past
            // the stream), so the counted waits below hold
            // pace: the strips of this wave's tile m (its m-th in the block's
            // tile order) are fetched once the block's loaders have published
            // pass-1 tile m - lead, so V_{j+1} rows are gathered soon after
            // they are written (in L2 / the MALL), not a region later.  lead
            // exceeds the tiles a pass-1 tile reaches ahead, so the pass-1
            // tiles the wait is for never wait on this wave (no cycle).
            // A region whose pass-1 range starts more than hback tiles after its
            // pass-2 range (region 0 of a distributed rank's interior launch, whose
            // pass 1 starts at p1a while its pass 2 starts at tile 0) counts its
            // pace from the pass-1 start: the host's lead covers an offset of
            // hback between the two ranges, and the first pass-1 tile needs the
            // pass-2 tiles at block positions up to (p1a + hfwd) / KB.
            const int64_t gap = begin - (NQ > 0 ? ptile(pbeg < NQ ? pbeg : NQ - 1) : 0) - hback;
            const int64_t poff = gap > 0 ? (gap + KB - 1) / KB : 0;
            int64_t paced = -1;  // last tile cleared
            auto pace = [&](int64_t s) {
                const int64_t m = uw + (s / NC) * NU - poff;
                if (s >= ns || s / NC <= paced) return;
                paced = s / NC;
                const uint32_t pa = ws_lds_addr(&p1pub);
                // (never more than the block's pass-1 tiles: a distributed rank's
                // pass 1 here covers only the interior)
                const int target = (int)(m - lead < nt ? m - lead : nt);
                long spin = 0;
                while (ws_lds_read(pa) < target && ++spin < kWsSpin) __builtin_amdgcn_s_sleep(2);
                if (spin >= kWsSpin) *err = 6;
            };
            auto dma = [&](int64_t s) {
                const int slot = (int)(s % (DU + 1));
                const bool live = s < ns;
                if (!(dbg & 32)) pace(s);
                const uint32_t rb = live ? (uint32_t)(strip_r0(s) * 128) : 0u;
#pragma unroll
                for (int m = 0; m < 3; ++m)
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        ws_lds_t *dst = (ws_lds_t *)((char *)&ust[uw][slot][m][0] + 1024 * k);
                        const uint32_t off = live ? rb + goff[k] : 0x80000000u;
                        if (cpol & 1) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[m], dst, 16, off, 0, 0, 2);
                        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[m], dst, 16, off, 0, 0, 0);
                    }
            };
            // byte offsets of this lane's slot reads (from the slot base)
            const int ra = c;
            const uint32_t oa0 = (uint32_t)(ra * 128 + 16 * ((2 * g) ^ ((ra >> 1) & 7)));
            const uint32_t oa1 = (uint32_t)(ra * 128 + 16 * ((2 * g + 1) ^ ((ra >> 1) & 7)));
            uint32_t oc[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * r + g;
                oc[r] = (uint32_t)(2 * 2048 + row * 128 + 16 * ((c >> 1) ^ ((row >> 1) & 7)) + 8 * (c & 1));
            }
            const bool ev = (c & 1) == 0;
#pragma unroll
            for (int s = 0; s < DU; ++s) dma(s);
            for (int64_t s = 0; s < ns; ++s) {
                dma(s + DU);
                // strip s landed: DU younger strips' six DMAs each, and from the
                // steady state on also DU strips' two (SW: four) stores, were
                // issued after it
                constexpr int ST = SW ? 4 : QO ? 6 : 2;
                if (s < DU) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * DU) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((6 + ST) * DU) : "memory");
                if (s % NC == DU && s >= NC && lane == 0)
                    // tile s / NC - 1 ended with strip s - DU - 1, whose stores
                    // are older than strip s's DMA: drained
                    __hip_atomic_store(flags + ptile(ut0 + (s / NC - 1) * ustep), epoch, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t sb = ws_lds_addr(reinterpret_cast<int *>(&ust[uw][(int)(s % (DU + 1))][0][0]));
                d2_t y0, y1, p0, p1, j0, j1;
                double vc0, vc1, vc2, vc3;
                asm volatile(
                    "ds_read_b128 %0, %10\n\t"
                    "ds_read_b128 %1, %11\n\t"
                    "ds_read_b128 %2, %10 offset:2048\n\t"
                    "ds_read_b128 %3, %11 offset:2048\n\t"
                    "ds_read_b128 %4, %10 offset:4096\n\t"
                    "ds_read_b128 %5, %11 offset:4096\n\t"
                    "ds_read_b64 %6, %12\n\t"
                    "ds_read_b64 %7, %13\n\t"
                    "ds_read_b64 %8, %14\n\t"
                    "ds_read_b64 %9, %15\n\t"
                    "s_waitcnt lgkmcnt(0)"
                    // early-clobber: the reads are issued before the inputs are dead
                    : "=&v"(y0), "=&v"(y1), "=&v"(p0), "=&v"(p1), "=&v"(j0), "=&v"(j1), "=&v"(vc0), "=&v"(vc1),
                      "=&v"(vc2), "=&v"(vc3)
                    : "v"(sb + oa0), "v"(sb + oa1), "v"(sb + oc[0]), "v"(sb + oc[1]), "v"(sb + oc[2]),
                      "v"(sb + oc[3])
                    : "memory");
                const double ya[4] = {y0.x, y0.y, y1.x, y1.y}, pa[4] = {p0.x, p0.y, p1.x, p1.y},
                             ja[4] = {j0.x, j0.y, j1.x, j1.y}, vjc[4] = {vc0, vc1, vc2, vc3};
                d4_t acc = {0.0, 0.0, 0.0, 0.0};
                if (dbg & 16) {  // timing diagnostics: no MFMA work
                    acc = d4_t{pa[0] + ya[0], pa[1] + ya[1], ja[2] + vjc[2], ja[3] + vjc[3]};
                } else {
#pragma unroll
                for (int kc = 0; kc < 4; ++kc) acc = mfma16(pa[kc], bq[1][kc], acc);
#pragma unroll
                for (int kc = 0; kc < 4; ++kc) acc = mfma16(ya[kc], bq[0][kc], acc);
#pragma unroll
                for (int kc = 0; kc < 4; ++kc) acc = mfma16(ja[kc], bq[2][kc], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) gacc = mfma16(acc[r], acc[r], gacc);
#pragma unroll
                for (int r = 0; r < 4; ++r) sacc = mfma16(acc[r], vjc[r], sacc);
                }
                // V_{j+1}: the lane pairs (c, c ^ 1) swap one value per row pair
                // so each lane stores 16 contiguous bytes (write-through)
                const uint32_t r0b = (uint32_t)(strip_r0(s) * 128);
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const double a0 = acc[2 * h2], a1 = acc[2 * h2 + 1];
                    const double y = dpp_swap1(ev ? a1 : a0);
                    const double2 v = ev ? make_double2(a0, y) : make_double2(y, a1);
                    const int row = 4 * (2 * h2 + (ev ? 0 : 1)) + g;
                    const uint32_t off = r0b + (uint32_t)(row * 128 + (ev ? c : c - 1) * 8);
                    if (cpol & 8) __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&v), Or, off, 0, SA | 2);
                    else if (dbg & 128)  // (diagnostic: plain stores keep the line in this XCD's L2)
                        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&v), Or, off, 0, 0);
                    else __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&v), Or, off, 0, SA);
                }
                if constexpr (QO) {  // Q = V_j beta^-1, the same pair swap, two outputs
                    d4_t qa = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int kc = 0; kc < 4; ++kc) qa = mfma16(ja[kc], bq[0][kc], qa);
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2) {
                        const double a0 = qa[2 * h2], a1 = qa[2 * h2 + 1];
                        const double y = dpp_swap1(ev ? a1 : a0);
                        const double2 v = ev ? make_double2(a0, y) : make_double2(y, a1);
                        const int row = 4 * (2 * h2 + (ev ? 0 : 1)) + g;
                        const uint32_t off = r0b + (uint32_t)(row * 128 + (ev ? c : c - 1) * 8);
                        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&v), Sr, off, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&v), Qr, off, 0, 0);
                    }
                }
                if constexpr (SW) {
                    // V_j's strip (slot part 2, as the DMA laid it out) to Vsave:
                    // the DMA's own global offsets, so the pieces land unswizzled
                    v4u32_t vp0, vp1;
                    asm volatile(
                        "ds_read_b128 %0, %2 offset:4096\n\t"
                        "ds_read_b128 %1, %2 offset:5120\n\t"
                        "s_waitcnt lgkmcnt(0)"
                        : "=&v"(vp0), "=&v"(vp1)
                        : "v"(sb + 16u * (uint32_t)lane)
                        : "memory");
                    __builtin_amdgcn_raw_buffer_store_b128(vp0, Sr, r0b + goff[0], 0, 2);
                    __builtin_amdgcn_raw_buffer_store_b128(vp1, Sr, r0b + goff[1], 0, 2);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (ntl > 0 && lane == 0)
                __hip_atomic_store(flags + ptile(ut0 + (ntl - 1) * ustep), epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        // the NU updater slabs folded by the last updater to finish (slot 0
        // of each updater is free now)
        double *U = &ust[uw][0][0][0];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            U[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = gacc[r];
            U[256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)] = sacc[r];
        }
        int arrived = 0;
        if (lane == 0) arrived = __hip_atomic_fetch_add(&upd_in, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        arrived = __shfl(arrived, 0, 64);
        if (arrived == NU - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            for (int e = lane; e < 512; e += 64) {
                double a = 0.0;
                for (int u = 0; u < NU; ++u) a += ust[u][0][0][e];
                // e < 256: G slab (at 2G; the consumers' when g0), else S2 (at G)
                if (!(g0 && e < 256)) part[(e < 256 ? 2 * G : G) * 256 + bid * 256 + (e & 255)] = a;
            }
        }
        return;
    }
    // -------------------------------------------------------------- consumers
    const int cw = w - NL - NU;
    {
        const int pr = (cw * 3) / NC;
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    }
    const int bytes = (int)(n * 128);
    // the gather source through a buffer resource: all of it below 2^24 rows,
    // else a window of kWinRows rows centred on the strip's own row (wb: the
    // window's first row; the plan proved every column inside it)
    const bool win = GEN && nx >= kWinRows;
    auto xwin = [&](int64_t s0, int64_t &wb) {
        const int64_t c = xoff + s0 - kWinRows / 2;
        wb = win ? (c > 0 ? c : 0) : 0;
        const int64_t rows = win ? (nx - wb < kWinRows ? nx - wb : kWinRows) : nx;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Vg + wb * 16), (short)0, (int)(rows * 128),
                                                 0x00020000);
    };
    int64_t wb0 = 0;
    auto xr = xwin(0, wb0);
    const auto yr = __builtin_amdgcn_make_buffer_rsrc(Yo, (short)0, bytes, 0x00020000);
    double *S0 = scr[cw];
    d4_t macc = {0.0, 0.0, 0.0, 0.0}, gcc = {0.0, 0.0, 0.0, 0.0};
    double v1[4] = {0.0, 0.0, 0.0, 0.0};  // the pending strip's own V_{j+1} rows (pair-swapped layout)
    int64_t s0p = -1;
    // S1 += V_{j+1}^T Y over the pending strip (Y parked in S0, swizzled)
    auto epilogue = [&]() {
        double ya[4], va[4];
        const bool ev = (lane & 1) == 0;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {  // to the accumulator layout (row 4r + g, column c)
            const double x = v1[2 * h2], y = v1[2 * h2 + 1];
            const double got = dpp_swap1(ev ? y : x);
            va[2 * h2] = ev ? x : got;
            va[2 * h2 + 1] = ev ? got : y;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) ya[r] = S0[fw_sw(4 * r + (lane >> 4), lane & 15)];
#pragma unroll
        for (int r = 0; r < 4; ++r) macc = mfma16(va[r], ya[r], macc);
        if (g0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) gcc = mfma16(va[r], va[r], gcc);
        }
    };
    for (int64_t i = 0; i < nt; ++i) {
        const int s = (int)(i % K);
        const int64_t r0 = tile_of(i) * TR;
        const int64_t s0 = r0 + 16 * cw;
        const int g = lane >> 3, p = lane & 7;
        const uint32_t lane_off = 16u * p;
        int64_t wb = 0;
        if (win) xr = xwin(s0, wb);
        long spin = 0;
        while (__hip_atomic_load(&ready[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)i &&
               ++spin < kWsSpin)
            __builtin_amdgcn_s_sleep(1);
        if (spin >= kWsSpin) { *err = 4; break; }
        asm volatile("" ::: "memory");
        typename C::Stage &S = st[s];
        const int64_t kA = S.rp[0];
        const int co = (int)(kA & (C::CPP - 1)), vo = (int)(kA & 1);
        const int nrow = (int)(n - r0 < TR ? n - r0 : TR);
        const int runlen = (int)(S.rp[nrow] - kA);
        const uint64_t pw = S.pr[cw];
        const int ra = (int)(pw >> (4 * g)) & 15, rb = (int)(pw >> (4 * (15 - g))) & 15;
        const int lra = 16 * cw + ra, lrb = 16 * cw + rb;
        const int o0 = lra < nrow ? (int)(S.rp[lra] - kA) : 0;
        const int len0 = lra < nrow ? (int)(S.rp[lra + 1] - kA) - o0 : 0;
        const int o1 = lrb < nrow ? (int)(S.rp[lrb] - kA) : 0;
        const int len1 = lrb < nrow ? (int)(S.rp[lrb + 1] - kA) - o1 : 0;
        const int cnt = len0 + len1;
        double y[4] = {0.0, 0.0, 0.0, 0.0};
        if (runlen <= CAP) {  // tile-uniform
            const CT *cp = S.col + co;
            // column -> window row: C16 columns are offsets from the strip's own
            // row (xoff + s0), 32-bit ones gather-source rows
            const uint32_t cb16 = C16 ? (uint32_t)(xoff + s0 - wb) : (uint32_t)(-wb);
            const double *vp = S.val + vo;
            auto slot = [&](int ff) {
                const int o = ff < len0 ? o0 + ff : o1 + (ff - len0);
                return ff < cnt ? o : o0;
            };
            auto issue = [&](int f, double2 *xs) {
                int32_t cc[8];
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) cc[tt] = cp[slot(f + tt)];
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) {
                    const uint32_t off = f + tt < cnt ? __umul24((unsigned)cc[tt] + cb16, 128u) + lane_off
                                                      : 0x80000000u;
                    const auto u4 = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, GA);
                    __builtin_memcpy(&xs[tt], &u4, 16);
                }
            };
            auto fmas = [&](int f, const double2 *xs) {
#pragma unroll
                for (int tt = 0; tt < 8; ++tt) {
                    const double v = vp[slot(f + tt)];
                    if (f + tt < len0) {
                        y[0] = fma(v, xs[tt].x, y[0]);
                        y[1] = fma(v, xs[tt].y, y[1]);
                    } else {  // masked entries: x == 0, v finite
                        y[2] = fma(v, xs[tt].x, y[2]);
                        y[3] = fma(v, xs[tt].y, y[3]);
                    }
                }
            };
            double2 xs[8];
            issue(0, xs);  // step 0 for every lane (masked past cnt)
            if (s0p >= 0) epilogue();
            fmas(0, xs);
            for (int f = 8; f < cnt; f += 8) {  // group-uniform
                issue(f, xs);
                fmas(f, xs);
            }
        } else {  // long run (rare): epilogue first, then gather from global
            if (s0p >= 0) epilogue();
            ws_gather<const int32_t *, const double *, GA>(col + kA, val + kA, o0, len0, o1, cnt, xr, lane_off,
                                                               y, (uint32_t)wb);
        }
        // the CSR stage is no longer read by this wave
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) atomicAdd(&done[s], 1);
        // Y rows out (16 B per lane per row; rows past n out of range), Y
        // parked for the S1 epilogue, the strip's own V_{j+1} rows loaded
        {
            const auto st0 = make_double2(y[0], y[1]), st1 = make_double2(y[2], y[3]);
            const uint32_t oa = (uint32_t)((s0 + ra) * 128) + lane_off, ob = (uint32_t)((s0 + rb) * 128) + lane_off;
            const uint32_t fa = s0 + ra < n ? oa : 0x80000000u, fb = s0 + rb < n ? ob : 0x80000000u;
            if (cpol & 4) {  // streaming (nt) Y stores
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&st0), yr, fa, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&st1), yr, fb, 0, 2);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&st0), yr, fa, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const v4u32_t *>(&st1), yr, fb, 0, 0);
            }
        }
        S0[fw_sw(ra, 2 * p)] = y[0];
        S0[fw_sw(ra, 2 * p + 1)] = y[1];
        S0[fw_sw(rb, 2 * p)] = y[2];
        S0[fw_sw(rb, 2 * p + 1)] = y[3];
        // two 16-B loads per lane (the pair swap in the epilogue makes the
        // accumulator layout): lane (g, c) loads row 8 h2 + g (c even) or
        // 8 h2 + 4 + g (c odd), columns c & ~1, (c & ~1) + 1
        // (four 8-B loads in the accumulator layout measured 0.4 % slower)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int c = lane & 15;
            const int64_t row = s0 + 8 * h2 + 4 * (c & 1) + (lane >> 4);
            const uint32_t off = row < n ? (uint32_t)((xoff + row - wb) * 128 + (c & ~1) * 8) : 0x80000000u;
            const auto u = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, GA);
            __builtin_memcpy(&v1[2 * h2], &u, 16);
        }
        s0p = s0;
        wave_lds_sync();
    }
    if (s0p >= 0) epilogue();
    // the block's NC consumer slabs folded into one at part[bid] (S1) by the
    // last consumer to finish, in a fixed order
    // (g0: consumer cw's G slab in updater strip slot 1 + cw / (3 NU), part
    // (cw / 3) mod NU, matrix cw mod 3)
    auto gslab = [&](int c) { return &ust[(c / 3) % NU][1 + c / (3 * NU)][c % 3][0]; };
#pragma unroll
    for (int r = 0; r < 4; ++r) S0[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = macc[r];
    if (g0) {
        double *Gs = gslab(cw);
#pragma unroll
        for (int r = 0; r < 4; ++r) Gs[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = gcc[r];
    }
    int arrived = 0;
    if (lane == 0) arrived = __hip_atomic_fetch_add(&cons_in, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    arrived = __shfl(arrived, 0, 64);
    if (arrived == NC - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        double *slab = part + bid * 256;
        for (int e = lane; e < 256; e += 64) {
            double a[4] = {0.0, 0.0, 0.0, 0.0};
            int sl = 0;
            for (; sl + 3 < NC; sl += 4) {
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] += scr[sl + q][e];
            }
            for (; sl < NC; ++sl) a[0] += scr[sl][e];
            slab[e] = (a[0] + a[1]) + (a[2] + a[3]);
        }
        if (g0) {
            double *gout = part + (2 * G + bid) * 256;
            for (int e = lane; e < 256; e += 64) {
                double a = 0.0;
                for (int c = 0; c < NC; ++c) a += gslab(c)[e];
                gout[e] = a;
            }
        }
    }
}

// The step shape wf_plan16 takes for rows of this density, read from the
// same knobs by wf_plan16 and wf_first_gram (one rule): 200 the
// wide shape (more than 10.2 entries per row), 111 the default one (1 loader
// + 11 consumers + 4 updaters), 0 a measurement shape LZ_WF_SHAPE = 10 / 11 /
// 12 (2 loaders, NC consumers, 14 - NC updaters; *nc = NC); *allowed = false
// when LZ_PASS_WF=0 selects the two-pass step or the rows reach 2^24.  Read
// per call.
static int wf_shape(int64_t n, int64_t nnz, int *nc, bool *allowed)
{
    const char *e = getenv("LZ_PASS_WF");  // "0": the two-pass step (A/B)
    const char *sh = getenv("LZ_WF_SHAPE");  // consumers per block (A/B)
    const int want = sh ? atoi(sh) : 111;
    const bool wide = (double)nnz > 10.2 * (double)n;
    const int var = wide ? 200 : (want == 10 || want == 11 || want == 12) ? 0 : 111;
    *nc = var == 200 ? 10 : var ? 11 : want;
    *allowed = !(e && e[0] == '0') && n < (1 << 24);
    return var;
}

// Whether wf_plan16 will most likely pick the default wavefront shape, whose
// first launch can sum beta_0's Gram (XO 1): the solve then skips the separate
// Gram (it would share the fabric with the plan).  (The plan may still refuse
// the rows -- too few, or columns out of reach -- and the solve then runs the
// Gram itself: correct, only not beside the plan.)
bool wf_first_gram(int64_t n, int64_t nnz)
{
    int nc = 0;
    bool allowed = false;
    return wf_shape(n, nnz, &nc, &allowed) == 111 && allowed;
}

int wf_plan16(lz_handle *h, int64_t n, int64_t nnz, const int64_t *rp, const int32_t *col, WfPlan *pl, int64_t nx,
              int64_t xoff)
{
    if (nx < 0) nx = n;
    pl->ok = false;
    pl->planned = false;
    pl->col16 = nullptr;
    // rows of about 11 entries or fewer on average: the tile's CSR run fits the
    // kWfCapPerRow-entry-per-row stage; up to kWfWideRow: the wide shape (longer
    // runs take a slow global-gather path)
    bool allowed = false;
    pl->var = wf_shape(n, nnz, &pl->nc, &allowed);
    pl->tr = 16 * pl->nc;
    // (a gather source of 2^24+ rows is read through per-strip windows: the
    // plan below checks that every column falls inside its strip's)
    if (!allowed || n < pl->tr || xoff < 0 || xoff + n > nx ||
        (double)nnz > kWfWideRow * (double)n)
        return LZ_OK;
    const int64_t T = ceil_div(n, (int64_t)pl->tr);
    if ((size_t)T + 64 > h->wf_cap) {
        LZ_HIP_TRY(hipStreamSynchronize(h->stream));
        (void)hipFree(h->wf_deps);
        (void)hipFree(h->wf_flags);
        h->wf_deps = nullptr;
        h->wf_flags = nullptr;
        h->wf_cap = 0;
        LZ_HIP_TRY(hipMalloc(&h->wf_deps, sizeof(int2) * (size_t)(T + 64)));
        LZ_HIP_TRY(hipMalloc(&h->wf_flags, sizeof(int) * (size_t)(T + 64)));
        h->wf_cap = (size_t)T + 64;
    }
    // pass 1's 16-bit columns in the same pass (col16_plan's buffer and encoding)
    const char *c = getenv("LZ_PASS1_C16");  // "0": 32-bit columns (A/B); read per call
    int16_t *c16 = nullptr;
    if (!(c && c[0] == '0') && nnz > 0) {
        const size_t bytes = (size_t)nnz * 2 + 16;  // + the dword the kernel's range may end in
        if (bytes > h->c16_cap) {
            LZ_HIP_TRY(hipStreamSynchronize(h->stream));
            (void)hipFree(h->c16buf);
            h->c16buf = nullptr;
            h->c16_cap = 0;
            LZ_HIP_TRY(hipMalloc(&h->c16buf, bytes));
            h->c16_cap = bytes;
        }
        c16 = static_cast<int16_t *>(h->c16buf);
    }
    int *spans = h->err_flag + 12;  // err_flag[0]: device error word; [8], [9]: other plans
    LZ_HIP_TRY(hipMemsetAsync(spans, 0, 4 * sizeof(int), h->stream));
    // (one tile per block measured slower: its per-block atomics contend)
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(T, (int64_t)h->n_cu * 8));
    hipLaunchKernelGGL(k_wf_deps, dim3(grid), dim3(256), 0, h->stream, n, pl->tr, rp, col,
                       static_cast<int2 *>(h->wf_deps), c16, spans, xoff, nx >= kWinRows ? 1 : 0);
    LZ_LAUNCH_CHECK();
    int sp[4] = {0, 0, 0, 1};
    LZ_HIP_TRY(hipMemcpyAsync(sp, spans, sizeof(sp), hipMemcpyDeviceToHost, h->stream));
    LZ_HIP_TRY(hipStreamSynchronize(h->stream));
    pl->planned = true;
    pl->hback = sp[0];
    pl->hfwd = sp[1];
    pl->ok = sp[2] <= kWfMaxSpan && !(sp[3] & 2);
    pl->xoff = xoff;
    if (c16 && !(sp[3] & 1)) pl->col16 = c16;
    return LZ_OK;
}

int wf_step16(lz_handle *h, int64_t n, const int64_t *rp, const int32_t *col, const int16_t *col16,
              const double *val, const uint64_t *pairs, const WfPlan &pl, const double *Yj, const double *Vprev,
              const double *Vj, double *Vout, const double *binv, const double *P1, const double *P2,
              const double *Vg, double *Yo, int epoch, int *nparts, int64_t nx, int64_t p1a, int64_t p1b,
              double *part, const int64_t *q, double *Vsave, bool qo)
{
    const int64_t T = ceil_div(n, (int64_t)pl.tr);
    const int64_t xoff = pl.xoff;
    if (nx < 0) nx = n;
    if (p1b < 0) p1b = T;
    if (!part) part = h->partials2;
    // pass-2 tiles [q0, q1) u [q2, q3) (default: all of them)
    const int64_t q0 = q ? q[0] : 0, q1 = q ? q[1] : T, q2 = q ? q[2] : T, q3 = q ? q[3] : T;
    LZ_ARG_CHECK(xoff >= 0 && xoff + n <= nx && 0 <= p1a && p1a <= p1b && p1b <= T, "wavefront step ranges");
    LZ_ARG_CHECK(0 <= q0 && q0 <= q1 && q1 <= q2 && q2 <= q3 && q3 <= T && (p1a == p1b || q2 == q3),
                 "wavefront step pass-2 ranges");
    LZ_ARG_CHECK(pl.ok && n < (1 << 24), "wavefront step: wf_plan16 first");
    LZ_ARG_CHECK(pairs != nullptr, "strip row orders (strip_pairs) missing");
    LZ_ARG_CHECK(P2 == nullptr || (Yj && Vj && Vout && binv && Vout == Vg + 16 * xoff), "wavefront step buffers");
    LZ_ARG_CHECK(qo || Vsave == nullptr || (P2 && pl.var != 0), "wavefront step: SW stores (the 111 / wide shapes)");
    LZ_ARG_CHECK(!qo || (P2 && Vsave && pl.var == 111 && p1a == p1b && xoff == 0 && (nx < 0 || nx == n) && !q),
                 "wavefront post-call state: a one-GPU pass-2-only launch of the default shape");
    static_assert(12 <= kPairPad, "row orders must cover the last tile's strips");
    // pass 2 covers its tile ranges when it runs; a pass-1-only launch its range
    const int64_t nq = (q1 - q0) + (q3 - q2);
    const int64_t work = P2 ? std::max(nq, p1b - p1a) : p1b - p1a;
    if (work <= 0) {
        *nparts = 0;
        return LZ_OK;
    }
    // (virtual ranks sharing the device: each rank's share, so every grid is
    // resident; LZ_GRID_CAP, read per call: a cap for measurement, e.g. one
    // virtual rank's share of the CUs run alone)
    const char *gc = getenv("LZ_GRID_CAP");
    const int cap = gc && atoi(gc) > 0 ? atoi(gc) : (h->grid_cap > 0 ? h->grid_cap : h->n_cu);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(work, std::min(cap, h->n_cu)));
    // dbg: timing diagnostics (results are wrong), only in a -DLZ_DIAG build
    // (LZ_WF_DBG): bit 0 skips the loaders' flag polls, bit 1 the updaters'
    // work, bit 2 the pass-1 tiles; bit 3 / bit 6 run the updaters at issue
    // priority 0 / 3 (default 2); bit 7 stores V_{j+1} plain instead of sc1
    // (rows another XCD gathers then read stale).  The shipped library always
    // passes 0.
#ifdef LZ_DIAG
    const char *dg = getenv("LZ_WF_DBG");
    const int dbg = dg ? atoi(dg) : 0;
#else
    constexpr int dbg = 0;
#endif
    if (P2 && nq == 0 && p1a == p1b) {  // nothing to do
        *nparts = 0;
        return LZ_OK;
    }
    // the updaters' pace (tiles ahead of the block's pass 1): at least the
    // tiles a pass-1 tile reaches ahead in the block's order, plus two
    const int KB = grid < 8 ? grid : grid / 8;
    const int lmin = (int)((pl.hback + pl.hfwd + KB - 1) / KB) + 2;
    // C3 (lmin 4): shape 111 best at lmin + 3 = 7 (5: 3.07 ms, 6: 1.90, 7: 1.82,
    // 8: 1.84, 10: 1.87); the 2-loader shapes at lmin + 4; the wide shape flat
    // from lmin to lmin + 16 (profiles/r04_wide_lead_ab.log)
#ifndef LZ_WF_LEAD_ADD  // (a measurement build may move the one-loader shapes' offset)
#define LZ_WF_LEAD_ADD 3
#endif
    const int lead = lmin + (pl.var ? LZ_WF_LEAD_ADD : 4);
    // streaming (nt) hints: bit 0 the updaters' reads, bit 1 the CSR stages,
    // bit 2 the Y stores, bit 3 the V_{j+1} stores.  7: every stream touched
    // once is nt, so the V_{j+1} rows stay in L2 for the gathers (C3: 1.74-1.81
    // -> 1.69-1.70 ms; 8, nt on V_{j+1} too, 1.84)
    constexpr int cpol = 7;
    // Liveness needs every block resident at once (their waits on each other's
    // flags).  The launch is checked: the occupancy of the instantiation at its
    // block size must admit the grid (one block per CU, grid <= CUs).  A block
    // that lands on a CU another kernel still holds starts when that kernel
    // ends; the bounded waits cover that, so no kernel that itself waits on
    // this launch may share the device (lz_hip.h).  (A cooperative launch was
    // measured and removed in round 5: 0.3-0.8 % slower at C3,
    // profiles/r04b_coop_ab.log; the runtime ran such launches one at a time,
    // so 8 virtual ranks' step launches serialised, 106 against 57.4 ms per C4
    // step; and the one process that used it ended in a segfault at exit,
    // DESIGN.md 5.)
    int rc = LZ_OK;
    // (the post-call state launch is not a step: no class of its own, as the
    // strip kernel it replaces had none)
    const int ev = qo ? -1 : prof_begin(h, PROF_SPMM_PASS);
    // (the block is 64 (NC + NL + NU) threads: the kernel refuses any other size)
    auto go = [&](auto kern, int waves) {
        // blocks per CU of this instantiation, cached per kernel (every
        // instantiation has the same function type, so a static in this lambda
        // would be one cache for all of them); per process: one device model
        int occ = -1;
        {
            static std::mutex mu;
            static std::unordered_map<const void *, int> occ_cache;
            std::lock_guard<std::mutex> lk(mu);
            const auto it = occ_cache.find(reinterpret_cast<const void *>(kern));
            if (it != occ_cache.end()) {
                occ = it->second;
            } else {
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64 * waves, 0) != hipSuccess) occ = 0;
                occ_cache.emplace(reinterpret_cast<const void *>(kern), occ);
            }
        }
        if ((int64_t)grid > (int64_t)occ * h->n_cu) {
            set_error("wavefront step: %d blocks of %d threads cannot all be resident (%d per CU x %d CUs)", grid,
                      64 * waves, occ, h->n_cu);
            rc = LZ_E_HIP;
            return;
        }
        const int2 *deps = static_cast<const int2 *>(h->wf_deps);
        int *flags = h->wf_flags, *err = h->err_flag;
        int64_t a_n = n, a_hb = pl.hback, a_nx = nx, a_p1a = p1a, a_p1b = p1b, a_T = T, a_xo = xoff, a_q0 = q0,
                a_q1 = q1, a_q2 = q2, a_q3 = q3;
        int a_ep = epoch, a_lead = lead, a_dbg = dbg, a_cp = cpol;
        double *a_sv = Vsave;
        const int64_t *a_rp = rp;
        const int32_t *a_col = col;
        const int16_t *a_c16 = col16;
        const double *a_val = val, *a_Yj = Yj, *a_Vp = Vprev, *a_Vj = Vj, *a_bi = binv, *a_P1 = P1, *a_P2 = P2,
                     *a_Vg = Vg;
        const uint64_t *a_pr = pairs;
        double *a_Vo = Vout, *a_Yo = Yo, *a_part = part;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 0, h->stream, a_n, a_rp, a_col, a_c16, a_val, a_pr,
                           a_Yj, a_Vp, a_Vj, a_Vo, a_bi, a_P1, a_P2, a_Vg, a_Yo, deps, flags, a_ep, a_hb, a_lead,
                           a_part, err, a_dbg, a_nx, a_p1a, a_p1b, a_T, a_cp, a_xo, a_q0, a_q1, a_q2, a_q3, a_sv);
    };
    // LDS (<= 160 KB): strip slots per updater DU + 1, fewer with 32-bit columns
    constexpr int cap12 = 12 * 16 * kWfCapPerRow, cap11 = 11 * 16 * kWfCapPerRow, cap10 = 10 * 16 * kWfCapPerRow;
    // (the instantiation must match pl.tr: the tile count above is the host's)
    const bool sw = Vsave != nullptr && !qo;
    // the one-GPU solve's launches (every pass-2 tile, whole source, no SW) take
    // the specialised form (GEN = false) of the default shapes
    const bool one = !sw && xoff == 0 && nx == n && q0 == 0 && q1 == T && q2 == T && q3 == T;
#ifdef LZ_WF_GEN_ONLY  // (measurement build: the general form everywhere)
    const bool spec = false;
    (void)one;
#else
    const bool spec = one;
#endif
    // (beta_0's Gram in a first launch: the default shape only, wf_first_gram)
    const bool g0 = !P2 && Vj != nullptr;
    if (g0 && pl.var != 111) {
        set_error("wavefront first launch with beta_0's Gram: the default shape only (internal)");
        rc = LZ_E_ARG;
    } else if (qo && col16) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true, false, false, 2>, 11 + 1 + 4);
    else if (qo) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false, false, false, 2>, 11 + 1 + 4);
    else if (g0 && col16 && spec) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true, false, false, 1>, 11 + 1 + 4);
    else if (g0 && col16) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true, false, true, 1>, 11 + 1 + 4);
    else if (g0 && spec) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false, false, false, 1>, 11 + 1 + 4);
    else if (g0) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false, false, true, 1>, 11 + 1 + 4);
    else if (pl.var == 200 && col16 && sw) go(k_wf16<10, kWfWideCap, 2, 1, 3, 1, true, true>, 10 + 1 + 3);
    else if (pl.var == 200 && col16 && spec) go(k_wf16<10, kWfWideCap, 2, 1, 3, 1, true, false, false>, 10 + 1 + 3);
    else if (pl.var == 200 && col16) go(k_wf16<10, kWfWideCap, 2, 1, 3, 1, true>, 10 + 1 + 3);
    else if (pl.var == 200 && sw) go(k_wf16<10, kWfWideCap, 2, 1, 2, 1, false, true>, 10 + 1 + 2);
    else if (pl.var == 200 && spec) go(k_wf16<10, kWfWideCap, 2, 1, 2, 1, false, false, false>, 10 + 1 + 2);
    else if (pl.var == 200) go(k_wf16<10, kWfWideCap, 2, 1, 2, 1, false>, 10 + 1 + 2);
    else if (pl.var == 111 && col16 && sw) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true, true>, 11 + 1 + 4);
    else if (pl.var == 111 && col16 && spec) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true, false, false>, 11 + 1 + 4);
    else if (pl.var == 111 && col16) go(k_wf16<11, cap11, kWfK, 1, 4, 1, true>, 11 + 1 + 4);
    else if (pl.var == 111 && sw) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false, true>, 11 + 1 + 4);
    else if (pl.var == 111 && spec) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false, false, false>, 11 + 1 + 4);
    else if (pl.var == 111) go(k_wf16<11, cap11, kWfK, 1, 4, 1, false>, 11 + 1 + 4);
    else if (col16) {
        if (pl.nc == 12) go(k_wf16<12, cap12, kWfK, kWfNL, 2, 3, true>, 12 + kWfNL + 2);
        else if (pl.nc == 11) go(k_wf16<11, cap11, kWfK, kWfNL, 3, 2, true>, 11 + kWfNL + 3);
        else go(k_wf16<10, cap10, kWfK, kWfNL, 4, 2, true>, 10 + kWfNL + 4);
    } else {
        if (pl.nc == 12) go(k_wf16<12, cap12, kWfK, kWfNL, 2, 2, false>, 12 + kWfNL + 2);
        else if (pl.nc == 11) go(k_wf16<11, cap11, kWfK, kWfNL, 3, 2, false>, 11 + kWfNL + 3);
        else go(k_wf16<10, cap10, kWfK, kWfNL, 4, 1, false>, 10 + kWfNL + 4);
    }
    prof_end(h, ev);
    LZ_TRY(rc);
    LZ_LAUNCH_CHECK();
    *nparts = grid;
    return LZ_OK;
}

// The wavefront step's three sums over the slab sets of one step's launches
// (one set single-GPU; a distributed step's pass-2 launches, its step launch
// and its boundary launches): set t holds [S1 | S2 | G] of sl.g[t] block slabs
// each, at sl.p[t]; out[256 m, 256 m + 256) = matrix m summed over every set,
// sets in order.  12 blocks, so that no CU pulls more than an eighth of a
// megabyte (one CU alone reads ~64 B per clock): block (m, r) sums entries
// [64 r, 64 r + 64) of matrix m; thread (q, i) adds slabs q, q + 16, ... with
// four independent accumulators, then the 16 partial sums are added in a
// fixed tree -- bitwise reproducible.
__global__ __launch_bounds__(1024) void k_wf_fold(WfSlabs sl, double *__restrict__ out)
{
    __shared__ double ps[16][64];
    const int m = blockIdx.x >> 2, q = threadIdx.x >> 6, i = (blockIdx.x & 3) * 64 + (threadIdx.x & 63);
    auto sum = [&](const double *p, int P) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int g = q;
        for (; g + 48 < P; g += 64) {
            a0 += p[(int64_t)g * 256 + i];
            a1 += p[(int64_t)(g + 16) * 256 + i];
            a2 += p[(int64_t)(g + 32) * 256 + i];
            a3 += p[(int64_t)(g + 48) * 256 + i];
        }
        for (; g < P; g += 16) a0 += p[(int64_t)g * 256 + i];
        return (a0 + a1) + (a2 + a3);
    };
    double s = 0.0;
    for (int t = 0; t < sl.k; ++t)
        if (sl.g[t] > 0) s = t == 0 ? sum(sl.p[t] + (int64_t)m * sl.g[t] * 256, sl.g[t])
                                    : s + sum(sl.p[t] + (int64_t)m * sl.g[t] * 256, sl.g[t]);
    ps[q][threadIdx.x & 63] = s;
    __syncthreads();
    if (q == 0) {
        const int l = threadIdx.x & 63;
        double t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = (ps[4 * k][l] + ps[4 * k + 1][l]) + (ps[4 * k + 2][l] + ps[4 * k + 3][l]);
        out[m * 256 + i] = (t[0] + t[1]) + (t[2] + t[3]);
    }
}

int wf_fold16(lz_handle *h, const WfSlabs &sl, double *out)
{
    LZ_ARG_CHECK(sl.k >= 1 && sl.k <= WfSlabs::kMax, "wavefront fold: 1..6 slab sets");
    const int ev = prof_begin(h, PROF_SMALL);
    hipLaunchKernelGGL(k_wf_fold, dim3(12), dim3(1024), 0, h->stream, sl, out);
    prof_end(h, ev);
    LZ_LAUNCH_CHECK();
    return LZ_OK;
}

int wf_reset16(lz_handle *h, int64_t n, const WfPlan &pl)
{
    const int64_t T = ceil_div(n, (int64_t)pl.tr);
    LZ_ARG_CHECK((size_t)T <= h->wf_cap, "wf_plan16 first");
    LZ_HIP_TRY(hipMemsetAsync(h->wf_flags, 0, sizeof(int) * (size_t)T, h->stream));
    return LZ_OK;
}

}  // namespace lz
