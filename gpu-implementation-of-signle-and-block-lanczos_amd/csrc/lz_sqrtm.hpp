// lz_sqrtm.hpp -- the wave-level pieces of the b x b symmetric square root
// (beta = sqrtm(G), beta^-1) that k_sqrtm_b (lz_dense.hip) runs after its slab
// reduction: any kernel that includes them gets k_sqrtm_b's bits.  The
// reference's sqrtm: kernels/my_sqrtm_cusolver.hpp (syevj, then V f(L) V^T).
// One wave (lanes tid < 64) runs each function; Am, Um are B x (B + 1) LDS
// matrices, cc / ss B-entry LDS vectors.
#pragma once

#include "lz_kernels.hpp"

namespace lz {

// Jacobi rotation for the pair (p, q): c, s with R[p][p] = R[q][q] = c,
// R[p][q] = -s, R[q][p] = s annihilating a_pq -- Numerical Recipes' angle
// (t = tan(theta) = sgn(d) a2 / (|d| + r), d = a_qq - a_pp, a2 = 2 a_pq,
// r = hypot(d, a2)) through the half-angle forms, which need no division and
// no square root: with cos(2 theta) = |d| / r, c^2 = u = (1 + |d| / r) / 2
// and s = sin(2 theta) / (2 c) = sgn(d) a2 / (2 r c).  Two reciprocal square
// roots (v_rsq_f64 and one Newton step each) replace the division, the sqrt
// and the rsq of the direct form, which head every round's dependent chain
// (C3: the sqrtm kernel 56.8 -> 51.4 us per step).
__device__ __forceinline__ void jacobi_rot(double app, double aqq, double apq, double &c, double &s)
{
#pragma clang fp contract(off)
    constexpr double kTol2 = 2.220446049250313e-16 * 2.220446049250313e-16;
    c = 1.0;
    s = 0.0;
    if (apq != 0.0 && apq * apq > kTol2 * (fabs(app) * fabs(aqq))) {
        const double d = aqq - app, a2 = 2.0 * apq;
        const double r2 = d * d + a2 * a2;
        double ir = __builtin_amdgcn_rsq(r2);
        ir = ir * (1.5 - 0.5 * r2 * ir * ir);  // 1 / r
        const double u = 0.5 + 0.5 * (fabs(d) * ir);
        double iu = __builtin_amdgcn_rsq(u);
        iu = iu * (1.5 - 0.5 * u * iu * iu);  // 1 / c
        c = u * iu;
        s = (0.5 * (d >= 0.0 ? a2 : -a2)) * (ir * iu);
    }
}

// A = the symmetric G (from its lower triangle, as syevj with
// CUBLAS_FILL_MODE_LOWER), U = I; lane t owns entries (t / B + (64 / B) k, t % B)
template <int B>
__device__ __forceinline__ void sqrtm_init(const double *g, double *Am, double *Um, int tid)
{
    constexpr int LD = B + 1, NE = B * B / 64, RS = 64 / B;
    const int j = tid % B, r0 = tid / B;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int i = r0 + RS * k;
        Am[i * LD + j] = (i < j) ? g[j * B + i] : g[i * B + j];
        Um[i * LD + j] = (i == j) ? 1.0 : 0.0;
    }
    wave_lds_sync();
}

// The round-robin (circle method) parallel cyclic Jacobi of k_sqrtm_b (see
// there), register-resident form for B = 16, 32: on return Am's diagonal
// holds the eigenvalues and Um = V^T (LDS copies in index order).  Returns
// the sweeps run.
template <int B>
__device__ int jacobi_rr(double *Am, double *Um, int tid)
{
#pragma clang fp contract(off)
    static_assert(B == 16 || B == 32, "register-resident Jacobi: B in {16, 32}");
    constexpr int LD = B + 1;
    constexpr double kTol2 = 2.220446049250313e-16 * 2.220446049250313e-16;
    int nsw = 0;
    // Register-resident form.  The NPB = B/2 pairs (p, B-1-p) cut A into
    // NPB x NPB 2x2 pair-blocks; lane L owns QS = NPB^2/64 of them: position
    // rows {P, B-1-P} x columns {Q_t, B-1-Q_t}, t < QS (P = L / LPP,
    // Q_t = (L % LPP) QS + t, LPP = NPB / QS lanes per row pair), and the
    // same rows x index columns of U.  Per round: the lanes holding a
    // diagonal block form that pair's rotation, every lane fetches its row
    // and column rotations by lane shuffles and updates its blocks in
    // registers (same products, same order as the LDS form, so A stays
    // bit-symmetric); the circle move is one scatter to the LDS copy (moved
    // positions) and one gather back -- no LDS round trip for the rotation
    // parameters and about half the LDS accesses of the LDS form.
    constexpr int NPB = B / 2, QS = NPB * NPB / 64, LPP = NPB / QS;
    const int P = tid / LPP, Q0 = (tid % LPP) * QS;
    auto owner = [](int p) { return p * LPP + p / QS; };  // lane holding pair p's diagonal block
    auto mv = [](int x) { return x == 0 ? 0 : (x == 1 ? B - 1 : x - 1); };
    const int X[2] = {P, B - 1 - P}, XM[2] = {mv(X[0]), mv(X[1])};
    int Y[QS][2], YM[QS][2];
#pragma unroll
    for (int t = 0; t < QS; ++t) {
        Y[t][0] = Q0 + t;
        Y[t][1] = B - 1 - (Q0 + t);
        YM[t][0] = mv(Y[t][0]);
        YM[t][1] = mv(Y[t][1]);
    }
    const bool has_diag = (tid % LPP) == P / QS;  // slot P % QS holds block (P, P)
    double a[QS][2][2], u[QS][2][2];
#pragma unroll
    for (int t = 0; t < QS; ++t)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                a[t][ii][jj] = Am[X[ii] * LD + Y[t][jj]];
                u[t][ii][jj] = Um[X[ii] * LD + Y[t][jj]];
            }
    for (int sweep = 0; sweep < 60; ++sweep) {
        nsw = sweep;
        bool need = false;  // the LDS copy holds this sweep's matrix in index order
#pragma unroll
        for (int t = 0; t < QS; ++t)
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const int x = X[ii], y = Y[t][jj];
                    const double aij = a[t][ii][jj];
                    if (x != y && aij != 0.0 &&
                        aij * aij > kTol2 * (fabs(Am[x * LD + x]) * fabs(Am[y * LD + y])))
                        need = true;
                }
        if (__ballot(need) == 0) break;  // wave-uniform
#pragma unroll 1
        for (int rnd = 0; rnd < B - 1; ++rnd) {
            double c = 1.0, sn = 0.0;
            if (has_diag) {
                double d00 = a[0][0][0], d11 = a[0][1][1], d01 = a[0][0][1];
#pragma unroll
                for (int t = 1; t < QS; ++t)
                    if (P % QS == t) {
                        d00 = a[t][0][0];
                        d11 = a[t][1][1];
                        d01 = a[t][0][1];
                    }
                jacobi_rot(d00, d11, d01, c, sn);
            }
            const double cP = __shfl(c, owner(P), 64), sP = __shfl(sn, owner(P), 64);
            // R[x0][x0] = R[x1][x1] = c, R[x0][x1] = -s, R[x1][x0] = s
            const double ci[2] = {cP, cP}, si[2] = {-sP, sP};
#pragma unroll
            for (int t = 0; t < QS; ++t) {
                const int Qt = Q0 + t;
                const double cQ = __shfl(c, owner(Qt), 64), sQ = __shfl(sn, owner(Qt), 64);
                const double cj[2] = {cQ, cQ}, sj[2] = {-sQ, sQ};
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        const double x1 = a[t][ii][jj] * (ci[ii] * cj[jj]);
                        const double x2 = a[t][ii][1 - jj] * (ci[ii] * sj[jj]);
                        const double x3 = a[t][1 - ii][jj] * (si[ii] * cj[jj]);
                        const double x4 = a[t][1 - ii][1 - jj] * (si[ii] * sj[jj]);
                        const bool ann = (P == Qt) && (ii != jj) && sP != 0.0;  // the annihilated pair
                        Am[XM[ii] * LD + YM[t][jj]] = ann ? 0.0 : (x1 + x4) + (x2 + x3);
                        Um[XM[ii] * LD + Y[t][jj]] = u[t][ii][jj] * ci[ii] + u[t][1 - ii][jj] * si[ii];
                    }
            }
            wave_lds_sync();
#pragma unroll
            for (int t = 0; t < QS; ++t)
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        a[t][ii][jj] = Am[X[ii] * LD + Y[t][jj]];
                        u[t][ii][jj] = Um[X[ii] * LD + Y[t][jj]];
                    }
            wave_lds_sync();
        }
    }
    return nsw;
}

// beta = V f(L) V^T (f = sqrt |.|) and beta^-1 (f = 1 / sqrt |.|) from the
// Jacobi result, V[i][k] = U[k][i], f(L) tabulated once in cc / ss; L != null:
// LB = L * beta (g, the Gram, is dead and parks beta).  wbi / wp1 (optional,
// LDS): beta^-1 and LB as the stored type rounds them.
template <typename T, int B>
__device__ void sqrtm_tail(const double *Am, const double *Um, double *cc, double *ss, double *g, T *beta, T *binv,
                           const T *L, T *LB, double *wbi, double *wp1, int tid)
{
#pragma clang fp contract(off)
    constexpr int LD = B + 1, NE = B * B / 64, RS = 64 / B;
    const int j = tid % B, r0 = tid / B;
    // beta = V f(L) V^T with V[i][k] = U[k][i]; f(L) tabulated once
    if (tid < B) {
        const double sq = sqrt(fabs(Am[tid * LD + tid]));
        cc[tid] = sq;
        ss[tid] = 1.0 / sq;
    }
    wave_lds_sync();
#pragma unroll 1
    for (int k = 0; k < NE; ++k) {
        const int i = r0 + RS * k;
        double s1 = 0.0, s2 = 0.0;
#pragma unroll 4
        for (int kk = 0; kk < B; ++kk) {
            const double vv = Um[kk * LD + i] * Um[kk * LD + j];
            s1 += vv * cc[kk];
            s2 += vv * ss[kk];
        }
        if (beta) beta[i * B + j] = (T)s1;
        if (binv) binv[i * B + j] = (T)s2;
        if (L) g[i * B + j] = s1;  // g (the Gram) is dead: park beta for LB
        if (wbi) wbi[i * B + j] = (double)(T)s2;
    }
    if (L) {  // LB = L * beta (the Q-free iteration's P1 = beta_{j-1}^-1 beta_j)
        wave_lds_sync();
#pragma unroll 1
        for (int k = 0; k < NE; ++k) {
            const int i = r0 + RS * k;
            double s = 0.0;
#pragma unroll 4
            for (int kk = 0; kk < B; ++kk) s = fma((double)L[i * B + kk], g[kk * B + j], s);
            LB[i * B + j] = (T)s;
            if (wp1) wp1[i * B + j] = (double)(T)s;
        }
    }
}

// Coupled Newton-Schulz square root for B = 16 on the f64 MFMA (one wave):
// A = G / |G|_F (G symmetrised from its lower triangle, as sqrtm_init),
// Y_0 = A, Z_0 = I, T = (3 I - Z_k Y_k) / 2, Y_{k+1} = Y_k T, Z_{k+1} = T Z_k,
// so Y -> A^{1/2} and Z -> A^{-1/2} (quadratically once the smallest
// eigenvalue of Z Y is near 1; about log(kappa(G)) / log(2.25) + 5
// iterations).  The same beta = G^{1/2}, beta^-1 = G^{-1/2} as the Jacobi
// route for a well-conditioned SPD G, in ~20 dependent 16 x 16 products
// instead of ~7 sweeps of 15 rotation rounds.  Returns false -- the caller
// then runs the Jacobi route, whose small eigenvalues keep high relative
// accuracy -- unless |Z Y - I|_max fell to the rounding floor within kNsMax
// iterations AND |Z|_F^2 <= kNsKappa, which bounds kappa(G) by 4e6 (kappa(G)
// up to 1e6: beta within ~4e-14 and beta^-1 within ~3e-12 of the Jacobi
// route's, scripts/probe/sqrtm_probe.hip), so an ill-conditioned or nearly
// rank-deficient G (Krylov breakdown) takes the reference's
// eigendecomposition path.
// Lane l = (c = l & 15, q = l >> 4) keeps rows/columns in the MFMA operand
// layouts: xa[k] = X[c][4q + k] (A operand, permuted contraction order),
// xb[k] = X[4q + k][c] (B operand); a product comes back as D[q + 4 r][c].
// S0, S1, S2: 16 x 17 LDS doubles of scratch each.  On success ya / yb / za /
// zb hold the converged Y and Z, and scale = |G|_F.
constexpr int kNsMax = 22;
constexpr double kNsKappa = 4e6;  // |Z|_F^2 bound: kappa(G) <= 4e6 (sqrtm_ns16)
__device__ __forceinline__ bool sqrtm_ns16(const double *g, double *S0, double *S1, double *S2, double ya[4],
                                           double yb[4], double za[4], double zb[4], double &scale, int tid)
{
    constexpr int LD = 17;
    const int c = tid & 15, q = tid >> 4;
    double f = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 4 * q + k;
        const double a = c < j ? g[j * 16 + c] : g[c * 16 + j];  // symmetric: A[c][j] = A[j][c]
        ya[k] = a;
        f = fma(a, a, f);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o, 64);
    if (!(f > 0.0) || !(f < 1e300)) return false;
    scale = sqrt(f);
    const double is = 1.0 / scale;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ya[k] *= is;
        yb[k] = ya[k];
        za[k] = zb[k] = (c == 4 * q + k) ? 1.0 : 0.0;
    }
    double prev = 1e300;
    for (int it = 0; it < kNsMax; ++it) {
        d4_t m = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; ++k) m = mfma16(za[k], yb[k], m);  // M = Z Y
        double e = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) e = fmax(e, fabs(m[r] - ((q + 4 * r == c) ? 1.0 : 0.0)));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) e = fmax(e, __shfl_xor(e, o, 64));
        if (!(e < 1e3)) return false;              // diverging, or NaN
        if (e <= 1.5e-14 || (e < 1e-10 && e >= 0.5 * prev)) {  // at the rounding floor
            // and only for kappa(G) <= kNsKappa: Z ~ A^{-1/2}, so |Z|_F^2 =
            // sum 1 / lambda_i(A) >= 1 / lambda_min(A) >= kappa(G) (lambda_max(A)
            // <= 1).  Past it the Newton-Schulz floor (beta^-1 off the Jacobi
            // route by ~6e-10 at kappa 1e8, profiles/r04v_sqrtm_probe.log) is
            // above the eigendecomposition route's, which then runs.
            double z2 = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) z2 = fma(za[k], za[k], z2);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) z2 += __shfl_xor(z2, o, 64);
            return z2 <= kNsKappa;
        }
        prev = e;
#pragma unroll
        for (int r = 0; r < 4; ++r) S0[(q + 4 * r) * LD + c] = ((q + 4 * r == c) ? 1.5 : 0.0) - 0.5 * m[r];
        wave_lds_sync();
        double ta[4], tb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ta[k] = S0[c * LD + 4 * q + k];
            tb[k] = S0[(4 * q + k) * LD + c];
        }
        d4_t y = {0.0, 0.0, 0.0, 0.0}, z = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            y = mfma16(ya[k], tb[k], y);  // Y T
            z = mfma16(ta[k], zb[k], z);  // T Z
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            S1[(q + 4 * r) * LD + c] = y[r];
            S2[(q + 4 * r) * LD + c] = z[r];
        }
        wave_lds_sync();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ya[k] = S1[c * LD + 4 * q + k];
            yb[k] = S1[(4 * q + k) * LD + c];
            za[k] = S2[c * LD + 4 * q + k];
            zb[k] = S2[(4 * q + k) * LD + c];
        }
        wave_lds_sync();  // S0..S2 rewritten next iteration
    }
    return false;
}

// beta = |G|_F^{1/2} Y and beta^-1 = Z / |G|_F^{1/2} (symmetrised) from
// sqrtm_ns16, stored as sqrtm_tail stores the Jacobi route's: beta / binv
// (global, T), g <- beta when L (LB = L beta), wbi / wp1 (LDS, optional).
template <typename T>
__device__ void sqrtm_ns16_tail(const double ya[4], const double yb[4], const double za[4], const double zb[4],
                                double scale, double *g, T *beta, T *binv, const T *L, T *LB, double *wbi,
                                double *wp1, int tid)
{
    const int c = tid & 15, q = tid >> 4;
    const double rs = sqrt(scale), irs = 1.0 / rs;
    wave_lds_sync();  // every lane's reads of g (the Gram) are done
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int e = c * 16 + 4 * q + k;
        const double b = (0.5 * (ya[k] + yb[k])) * rs, bi = (0.5 * (za[k] + zb[k])) * irs;
        if (beta) beta[e] = (T)b;
        if (binv) binv[e] = (T)bi;
        if (L) g[e] = b;
        if (wbi) wbi[e] = (double)(T)bi;
    }
    if (L) {
        wave_lds_sync();
        const int j = tid % 16, r0 = tid / 16;
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
            const int i = r0 + 4 * k;
            double s = 0.0;
#pragma unroll 4
            for (int kk = 0; kk < 16; ++kk) s = fma((double)L[i * 16 + kk], g[kk * 16 + j], s);
            LB[i * 16 + j] = (T)s;
            if (wp1) wp1[i * 16 + j] = (double)(T)s;
        }
    }
}

// Coupled Newton-Schulz square root for B = 32 (sqrtm_ns16's iteration and
// exits) on the f64 MFMA, by waves 0..3 of the workgroup: wave w owns block
// (I, J) = (w >> 1, w & 1) of every 32 x 32 product, C_IJ = sum_K A_IK B_KJ,
// 8 v_mfma_f64_16x16x4f64 per product (lane (c, q) supplies A[16I + c][16K +
// 4q + k] and B[16K + 4q + k][16J + c]; C comes back as C[16I + q + 4r][16J +
// c]).  Y, Z, T live in LDS (32 x 33 doubles each); one iteration is three
// products and three workgroup barriers.  EVERY thread of the workgroup calls
// this (the barriers); threads past 256 only keep the count.  red: 8 doubles
// of LDS.  On success Ys / Zs hold the converged Y and Z, scale = |G|_F.
// Replaces the one-wave Jacobi of the reference's syevjBatched route
// (utils/lib_utils.hpp:696-745) at b = 32 for kappa(G) <= kNsKappa.
__device__ __forceinline__ bool sqrtm_ns32(const double *g, double *Ys, double *Zs, double *Ts, double *red,
                                           double &scale, int tid)
{
    constexpr int LD = 33;
    const bool act = tid < 256;
    const int w = (tid >> 6) & 3, lane = tid & 63, c = lane & 15, q = lane >> 4;
    const int I = w >> 1, J = w & 1;
    // A = sym(G) / |G|_F (lower triangle read, as sqrtm_init), Z = I
    double f = 0.0;
    if (act) {
        for (int e = tid; e < 1024; e += 256) {
            const int i = e >> 5, j = e & 31;
            const double a = j < i ? g[i * 32 + j] : g[j * 32 + i];
            Ys[i * LD + j] = a;
            Zs[i * LD + j] = i == j ? 1.0 : 0.0;
            f = fma(a, a, f);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o, 64);
        if (lane == 0) red[w] = f;
    }
    __syncthreads();
    f = (red[0] + red[1]) + (red[2] + red[3]);
    if (!(f > 0.0) || !(f < 1e300)) return false;  // (uniform)
    scale = sqrt(f);
    const double is = 1.0 / scale;
    if (act)
        for (int e = tid; e < 1024; e += 256) Ys[(e >> 5) * LD + (e & 31)] *= is;
    __syncthreads();
    auto prod = [&](const double *A, const double *B) {
        d4_t m = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int K = 0; K < 2; ++K)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                m = mfma16(A[(16 * I + c) * LD + 16 * K + 4 * q + k], B[(16 * K + 4 * q + k) * LD + 16 * J + c], m);
        return m;
    };
    double prev = 1e300;
    for (int it = 0; it < kNsMax; ++it) {
        if (act) {
            const d4_t m = prod(Zs, Ys);  // M = Z Y
            double e = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool d = 16 * I + q + 4 * r == 16 * J + c;
                e = fmax(e, fabs(m[r] - (d ? 1.0 : 0.0)));
                Ts[(16 * I + q + 4 * r) * LD + 16 * J + c] = (d ? 1.5 : 0.0) - 0.5 * m[r];
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) e = fmax(e, __shfl_xor(e, o, 64));
            if (lane == 0) red[w] = e;
        }
        __syncthreads();
        const double e = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
        if (!(e < 1e3)) return false;  // diverging, or NaN (uniform)
        if (e <= 3e-14 || (e < 1e-10 && e >= 0.5 * prev)) {  // at the rounding floor
            // and only for kappa(G) <= kNsKappa (sqrtm_ns16: |Z|_F^2 >= kappa(G))
            double z2 = 0.0;
            if (act) {
                for (int x = tid; x < 1024; x += 256) {
                    const double z = Zs[(x >> 5) * LD + (x & 31)];
                    z2 = fma(z, z, z2);
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) z2 += __shfl_xor(z2, o, 64);
                if (lane == 0) red[4 + w] = z2;
            }
            __syncthreads();
            return (red[4] + red[5]) + (red[6] + red[7]) <= kNsKappa;
        }
        prev = e;
        d4_t y = {0.0, 0.0, 0.0, 0.0}, z = {0.0, 0.0, 0.0, 0.0};
        if (act) {
            y = prod(Ys, Ts);  // Y T
            z = prod(Ts, Zs);  // T Z
        }
        __syncthreads();  // every read of Y, Z, T done
        if (act) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                Ys[(16 * I + q + 4 * r) * LD + 16 * J + c] = y[r];
                Zs[(16 * I + q + 4 * r) * LD + 16 * J + c] = z[r];
            }
        }
        __syncthreads();
    }
    return false;
}

// beta = |G|_F^{1/2} sym(Y), beta^-1 = sym(Z) / |G|_F^{1/2} from sqrtm_ns32
// (every thread of the workgroup calls it), stored as sqrtm_tail stores the
// Jacobi route's: beta / binv (global, T), g <- beta when L (LB = L beta).
template <typename T>
__device__ void sqrtm_ns32_tail(const double *Ys, const double *Zs, double scale, double *g, T *beta, T *binv,
                                const T *L, T *LB, int tid)
{
    constexpr int LD = 33;
    const double rs = sqrt(scale), irs = 1.0 / rs;
    for (int e = tid; e < 1024; e += blockDim.x) {
        const int i = e >> 5, j = e & 31;
        const double b = (0.5 * (Ys[i * LD + j] + Ys[j * LD + i])) * rs;
        const double bi = (0.5 * (Zs[i * LD + j] + Zs[j * LD + i])) * irs;
        if (beta) beta[e] = (T)b;
        if (binv) binv[e] = (T)bi;
        if (L) g[e] = b;  // g (the Gram) is dead: park beta for LB
    }
    if (L) {
        __syncthreads();
        for (int e = tid; e < 1024; e += blockDim.x) {
            const int i = e >> 5, j = e & 31;
            double s = 0.0;
#pragma unroll 4
            for (int kk = 0; kk < 32; ++kk) s = fma((double)L[i * 32 + kk], g[kk * 32 + j], s);
            LB[e] = (T)s;
        }
    }
}

}  // namespace lz
