// lz_host.cpp -- liblz_host.so: host-side logic around the GPU hot path
// (include/lz_host.h).  No GPU calls.
#include "lz_host.h"

#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

// ----------------------------------------------------------------- RNG
inline uint64_t splitmix64(uint64_t &x)
{
    uint64_t z = (x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

struct RowRng {
    uint64_t s;
    RowRng(uint64_t seed, uint64_t row)
    {
        s = seed ^ (row * 0xD1B54A32D192ED03ULL);
        (void)splitmix64(s);
    }
    uint64_t next() { return splitmix64(s); }
    double unif() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    double sym() { return 2.0 * unif() - 1.0; }                                     // [-1,1)
};

// ------------------------------------------------ symmetric generator core
// A generator gives, for each row r, its strict-upper entries (col > r, sorted,
// distinct) and values; the CSR is that upper triangle mirrored plus a diagonal.
// Rows [r0, r1) of the global matrix (row_ptr local, columns global).  Lower
// entries of those rows come from source rows s in [s0, r1) (s0 = r0 minus the
// generator's reach), so a slab is generated without the rest of the matrix
// and is identical to the same rows of the whole.
template <typename Upper>
int64_t sym_count(int64_t r0, int64_t r1, int64_t s0, Upper &&upper, int64_t *rp)
{
    const int64_t nl = r1 - r0;
    std::vector<int64_t> cnt(nl, 1);  // diagonal
#pragma omp parallel
    {
        std::vector<int32_t> c;
        std::vector<double> v;
#pragma omp for schedule(dynamic, 4096)
        for (int64_t s = s0; s < r1; ++s) {
            upper(s, c, v);
            if (s >= r0) {
#pragma omp atomic
                cnt[s - r0] += (int64_t)c.size();
            }
            for (int32_t cc : c) {
                if (cc < r0 || cc >= r1) continue;
#pragma omp atomic
                cnt[cc - r0] += 1;
            }
        }
    }
    rp[0] = 0;
    for (int64_t r = 0; r < nl; ++r) rp[r + 1] = rp[r] + cnt[r];
    return rp[nl];
}

template <typename Upper>
void sym_fill(int64_t r0, int64_t r1, int64_t s0, Upper &&upper, uint64_t seed, const int64_t *rp,
              int32_t *col, double *v64, float *v32)
{
    const int64_t n = r1 - r0;  // local rows
    std::vector<std::atomic<int64_t>> lo_pos(n);
    for (int64_t r = 0; r < n; ++r) lo_pos[r].store(0, std::memory_order_relaxed);
    std::vector<int64_t> lo_cnt(n);
#pragma omp parallel
    {
        std::vector<int32_t> c;
        std::vector<double> v;
#pragma omp for schedule(dynamic, 4096)
        for (int64_t s = s0; s < r1; ++s) {
            upper(s, c, v);
            if (s >= r0) {
                const int64_t r = s - r0;
                const int64_t len = rp[r + 1] - rp[r];
                const int64_t lo = len - 1 - (int64_t)c.size();
                lo_cnt[r] = lo;
                RowRng dg(seed ^ 0xA5A5A5A5ULL, (uint64_t)s);
                const double d = dg.sym();
                const int64_t at = rp[r] + lo;
                col[at] = (int32_t)s;
                if (v64) v64[at] = d;
                if (v32) v32[at] = (float)d;
                for (size_t t = 0; t < c.size(); ++t) {
                    col[at + 1 + t] = c[t];
                    if (v64) v64[at + 1 + t] = v[t];
                    if (v32) v32[at + 1 + t] = (float)v[t];
                }
            }
            for (size_t t = 0; t < c.size(); ++t) {
                const int64_t cc = c[t];
                if (cc < r0 || cc >= r1) continue;
                const int64_t rl = cc - r0;
                const int64_t slot = lo_pos[rl].fetch_add(1, std::memory_order_relaxed);
                col[rp[rl] + slot] = (int32_t)s;
                if (v64) v64[rp[rl] + slot] = v[t];
                if (v32) v32[rp[rl] + slot] = (float)v[t];
            }
        }
        // lower segments were filled in arrival order: sort them by column
#pragma omp for schedule(dynamic, 4096)
        for (int64_t r = 0; r < n; ++r) {
            const int64_t lo = lo_cnt[r];
            if (lo < 2) continue;
            std::vector<std::pair<int32_t, double>> seg(lo);
            for (int64_t t = 0; t < lo; ++t)
                seg[t] = {col[rp[r] + t], v64 ? v64[rp[r] + t] : (double)v32[rp[r] + t]};
            std::sort(seg.begin(), seg.end(),
                      [](const auto &a, const auto &b) { return a.first < b.first; });
            for (int64_t t = 0; t < lo; ++t) {
                col[rp[r] + t] = seg[t].first;
                if (v64) v64[rp[r] + t] = seg[t].second;
                if (v32) v32[rp[r] + t] = (float)seg[t].second;
            }
        }
    }
}

// distinct sorted upper columns drawn by `draw`, with their values
template <typename Draw>
void draw_upper(RowRng &g, int64_t k, Draw &&draw, std::vector<int32_t> &c, std::vector<double> &v)
{
    std::vector<std::pair<int32_t, double>> e;
    e.reserve(k);
    int64_t tries = 0;
    while ((int64_t)e.size() < k && tries < 8 * k + 16) {
        ++tries;
        const int64_t cc = draw(g);
        if (cc < 0) continue;
        bool dup = false;
        if (k <= 64) {
            for (auto &x : e)
                if (x.first == cc) { dup = true; break; }
        }
        if (dup) { (void)g.next(); continue; }
        e.push_back({(int32_t)cc, g.sym()});
    }
    std::sort(e.begin(), e.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    if (k > 64)  // large rows: drop duplicates after the sort
        e.erase(std::unique(e.begin(), e.end(),
                            [](const auto &a, const auto &b) { return a.first == b.first; }),
                e.end());
    c.resize(e.size());
    v.resize(e.size());
    for (size_t t = 0; t < e.size(); ++t) {
        c[t] = e[t].first;
        v[t] = e[t].second;
    }
}

struct Banded {
    int64_t n, hw;
    double h;
    uint64_t seed;
    void operator()(int64_t r, std::vector<int32_t> &c, std::vector<double> &v) const
    {
        RowRng g(seed, (uint64_t)r);
        const double fl = std::floor(h);
        int64_t k = (int64_t)fl + (g.unif() < (h - fl) ? 1 : 0);
        const int64_t avail = std::min<int64_t>(hw, n - 1 - r);
        if (avail <= 0) { c.clear(); v.clear(); return; }
        if (k > avail) k = avail;
        const int64_t nn = n, hh = hw;
        draw_upper(g, k, [=](RowRng &gg) -> int64_t {
            const int64_t d = 1 + (int64_t)(gg.next() % (uint64_t)hh);
            const int64_t cc = r + d;
            return cc < nn ? cc : -1;
        }, c, v);
    }
};

struct PowerLaw {
    int64_t n, cap;
    double a, xmin;
    uint64_t seed;
    void operator()(int64_t r, std::vector<int32_t> &c, std::vector<double> &v) const
    {
        RowRng g(seed, (uint64_t)r);
        const double u = 1.0 - g.unif();  // (0,1]
        int64_t k = (int64_t)std::floor(xmin * std::pow(u, -1.0 / a));
        const int64_t avail = n - 1 - r;
        k = std::min<int64_t>(std::min<int64_t>(k, cap), avail);
        if (k <= 0) { c.clear(); v.clear(); return; }
        draw_upper(g, k, [=](RowRng &gg) -> int64_t {
            return r + 1 + (int64_t)(gg.next() % (uint64_t)avail);
        }, c, v);
    }
};

double powerlaw_xmin(double npr, double a) { return std::max(0.5, ((npr - 1.0) / 2.0 + 0.5) * (a - 1.0) / a); }

// ------------------------------------------------------ eigen (tred2/tql2)
// Householder tridiagonalisation followed by the implicit QL method (the
// EISPACK tred2/tql2 algorithms).  V row-major k x k.
// Attribution: a close restatement of the public-domain JAMA library's
// EigenvalueDecomposition (tred2 / tql2, MathWorks and NIST, 1998-2012), which
// follows the EISPACK routines of Smith et al. (1976) and Bowdler, Martin,
// Reinsch and Wilkinson (Handbook for Auto. Comp., Vol. II -- Linear Algebra);
// its local names (c2, c3, s2, el1, dl1, tst1) are kept.  Not from the
// reference repository, which calls cuSOLVER syevd here (lib_utils.hpp:542-590).
void tred2(int n, std::vector<double> &V, std::vector<double> &d, std::vector<double> &e)
{
    auto Vr = [&](int i, int j) -> double & { return V[(size_t)i * n + j]; };
    for (int j = 0; j < n; ++j) d[j] = Vr(n - 1, j);
    for (int i = n - 1; i > 0; --i) {
        double scale = 0.0, h = 0.0;
        for (int k = 0; k < i; ++k) scale += std::fabs(d[k]);
        if (scale == 0.0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; ++j) {
                d[j] = Vr(i - 1, j);
                Vr(i, j) = 0.0;
                Vr(j, i) = 0.0;
            }
        } else {
            for (int k = 0; k < i; ++k) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            double f = d[i - 1];
            double g = std::sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h -= f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; ++j) e[j] = 0.0;
            for (int j = 0; j < i; ++j) {
                f = d[j];
                Vr(j, i) = f;
                g = e[j] + Vr(j, j) * f;
                for (int k = j + 1; k <= i - 1; ++k) {
                    g += Vr(k, j) * d[k];
                    e[k] += Vr(k, j) * f;
                }
                e[j] = g;
            }
            f = 0.0;
            for (int j = 0; j < i; ++j) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            const double hh = f / (h + h);
            for (int j = 0; j < i; ++j) e[j] -= hh * d[j];
            for (int j = 0; j < i; ++j) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; ++k) Vr(k, j) -= (f * e[k] + g * d[k]);
                d[j] = Vr(i - 1, j);
                Vr(i, j) = 0.0;
            }
        }
        d[i] = h;
    }
    for (int i = 0; i < n - 1; ++i) {
        Vr(n - 1, i) = Vr(i, i);
        Vr(i, i) = 1.0;
        const double h = d[i + 1];
        if (h != 0.0) {
            for (int k = 0; k <= i; ++k) d[k] = Vr(k, i + 1) / h;
            for (int j = 0; j <= i; ++j) {
                double g = 0.0;
                for (int k = 0; k <= i; ++k) g += Vr(k, i + 1) * Vr(k, j);
                for (int k = 0; k <= i; ++k) Vr(k, j) -= g * d[k];
            }
        }
        for (int k = 0; k <= i; ++k) Vr(k, i + 1) = 0.0;
    }
    for (int j = 0; j < n; ++j) {
        d[j] = Vr(n - 1, j);
        Vr(n - 1, j) = 0.0;
    }
    Vr(n - 1, n - 1) = 1.0;
    e[0] = 0.0;
}

void tql2(int n, std::vector<double> &V, std::vector<double> &d, std::vector<double> &e)
{
    auto Vr = [&](int i, int j) -> double & { return V[(size_t)i * n + j]; };
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    double f = 0.0, tst1 = 0.0;
    const double eps = std::ldexp(1.0, -52);
    for (int l = 0; l < n; ++l) {
        tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
        int m = l;
        while (m < n) {
            if (std::fabs(e[m]) <= eps * tst1) break;
            ++m;
        }
        if (m > l) {
            int iter = 0;
            do {
                ++iter;
                double g = d[l];
                double p = (d[l + 1] - g) / (2.0 * e[l]);
                double r = std::hypot(p, 1.0);
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                const double dl1 = d[l + 1];
                double h = g - d[l];
                for (int i = l + 2; i < n; ++i) d[i] -= h;
                f += h;
                p = d[m];
                double c = 1.0, c2 = c, c3 = c;
                const double el1 = e[l + 1];
                double s = 0.0, s2 = 0.0;
                for (int i = m - 1; i >= l; --i) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = std::hypot(p, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    for (int k = 0; k < n; ++k) {
                        h = Vr(k, i + 1);
                        Vr(k, i + 1) = s * Vr(k, i) + c * h;
                        Vr(k, i) = c * Vr(k, i) - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::fabs(e[l]) > eps * tst1 && iter < 100);
        }
        d[l] += f;
        e[l] = 0.0;
    }
}

void assemble_T(int m, int b, const double *alpha, const double *beta, double *T)
{
    const int k = m * b;
    std::fill(T, T + (size_t)k * k, 0.0);
    for (int blk = 0; blk < m; ++blk) {
        const double *a = alpha + (size_t)blk * b * b;
        for (int r = 0; r < b; ++r)
            for (int c = 0; c < b; ++c) T[(size_t)(blk * b + r) * k + blk * b + c] = a[r * b + c];
        if (blk >= 1) {
            const double *bt = beta + (size_t)blk * b * b;
            for (int r = 0; r < b; ++r)
                for (int c = 0; c < b; ++c) {
                    T[(size_t)((blk - 1) * b + r) * k + blk * b + c] = bt[r * b + c];
                    T[(size_t)(blk * b + c) * k + (blk - 1) * b + r] = bt[r * b + c];
                }
        }
    }
}

// glibc random_r TYPE_3 (x^31 + x^3 + 1), srand(seed): r[i] = r[i-31] + r[i-3],
// outputs r[i] >> 1 for i >= 344.  Circular buffer of the last 34 states.
struct GlibcRand {
    uint32_t ring[34];
    int head = 0;  // ring[head] is the oldest state r[i-34]
    explicit GlibcRand(uint32_t seed)
    {
        std::vector<uint32_t> r(344);
        const int32_t s = seed == 0 ? 1 : (int32_t)seed;
        r[0] = (uint32_t)s;
        for (int i = 1; i < 31; ++i) {
            const int64_t v = (16807LL * (int64_t)(int32_t)r[i - 1]) % 2147483647LL;
            r[i] = (uint32_t)(v < 0 ? v + 2147483647LL : v);
        }
        for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
        for (int i = 34; i < 344; ++i) r[i] = r[i - 31] + r[i - 3];
        for (int t = 0; t < 34; ++t) ring[t] = r[344 - 34 + t];
    }
    int32_t next()
    {
        // oldest = r[i-34]; r[i-31] at head+3, r[i-3] at head+31
        const uint32_t v = ring[(head + 3) % 34] + ring[(head + 31) % 34];
        ring[head] = v;
        head = (head + 1) % 34;
        return (int32_t)(v >> 1);
    }
};

}  // namespace

extern "C" {

int lzh_num_threads(void) { return omp_get_max_threads(); }

int64_t lzh_gen_banded_count(int64_t n, double npr, int64_t hw, uint64_t seed, int64_t *rp)
{
    return lzh_gen_banded_local_count(n, npr, hw, seed, 0, n, rp);
}

int lzh_gen_banded_fill(int64_t n, double npr, int64_t hw, uint64_t seed, const int64_t *rp,
                        int32_t *col, double *v64, float *v32)
{
    return lzh_gen_banded_local_fill(n, npr, hw, seed, 0, n, rp, col, v64, v32);
}

int64_t lzh_gen_banded_local_count(int64_t n, double npr, int64_t hw, uint64_t seed, int64_t r0,
                                   int64_t r1, int64_t *rp)
{
    if (n <= 0 || !rp || npr < 1.0 || hw < 1 || n > 2147483647LL) return -1;
    if (r0 < 0 || r1 > n || r0 >= r1) return -1;
    return sym_count(r0, r1, std::max<int64_t>(0, r0 - hw), Banded{n, hw, (npr - 1.0) / 2.0, seed}, rp);
}

int lzh_gen_banded_local_fill(int64_t n, double npr, int64_t hw, uint64_t seed, int64_t r0,
                              int64_t r1, const int64_t *rp, int32_t *col, double *v64, float *v32)
{
    if (n <= 0 || !rp || !col || r0 < 0 || r1 > n || r0 >= r1) return -1;
    sym_fill(r0, r1, std::max<int64_t>(0, r0 - hw), Banded{n, hw, (npr - 1.0) / 2.0, seed}, seed,
             rp, col, v64, v32);
    return 0;
}

int64_t lzh_gen_powerlaw_count(int64_t n, double npr, double a, int64_t cap, uint64_t seed,
                               int64_t *rp)
{
    if (n <= 0 || !rp || npr < 1.0 || a <= 1.0 || cap < 1 || n > 2147483647LL) return -1;
    return sym_count(0, n, 0, PowerLaw{n, cap, a, powerlaw_xmin(npr, a), seed}, rp);
}

int lzh_gen_powerlaw_fill(int64_t n, double npr, double a, int64_t cap, uint64_t seed,
                          const int64_t *rp, int32_t *col, double *v64, float *v32)
{
    if (n <= 0 || !rp || !col) return -1;
    sym_fill(0, n, 0, PowerLaw{n, cap, a, powerlaw_xmin(npr, a), seed}, seed, rp, col, v64, v32);
    return 0;
}

int64_t lzh_ell_to_csr_count(int64_t n, int64_t w, const double *data, const uint32_t *idx,
                             int keep_zeros, int64_t *rp)
{
    (void)idx;
    if (n < 0 || w < 0 || !rp) return -1;
    rp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t c = 0;
        for (int64_t s = 0; s < w; ++s) c += (keep_zeros || data[r + s * n] != 0.0);
        rp[r + 1] = rp[r] + c;
    }
    return rp[n];
}

int lzh_ell_to_csr_fill(int64_t n, int64_t w, const double *data, const uint32_t *idx,
                        int keep_zeros, const int64_t *rp, int32_t *col, double *val)
{
    if (n < 0 || !rp || !col || !val) return -1;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
        std::vector<std::pair<int32_t, double>> e;
        for (int64_t s = 0; s < w; ++s) {
            const double v = data[r + s * n];
            if (keep_zeros || v != 0.0) e.push_back({(int32_t)idx[r + s * n], v});
        }
        std::stable_sort(e.begin(), e.end(),
                         [](const auto &a, const auto &b) { return a.first < b.first; });
        for (size_t t = 0; t < e.size(); ++t) {
            col[rp[r] + t] = e[t].first;
            val[rp[r] + t] = e[t].second;
        }
    }
    return 0;
}

int lzh_rand_B(int64_t n, int b, uint32_t seed, int64_t skip, int row_major, double *out)
{
    if (n <= 0 || b <= 0 || !out) return -1;
    GlibcRand g(seed);
    for (int64_t s = 0; s < skip; ++s) (void)g.next();
    const int64_t total = n * b;
    for (int64_t i = 0; i < total; ++i) {
        const double v = ((double)g.next() / (double)2147483647) + 1.0;  // rand()/RAND_MAX + 1
        if (row_major) out[(i % n) * b + i / n] = v;
        else out[i] = v;
    }
    return 0;
}

int64_t lzh_rand_lc(uint32_t seed)
{
    GlibcRand g(seed);
    return 1 + (g.next() % 100);
}

int lzh_uniform_B(int64_t n, int b, uint64_t seed, double *o64, float *o32)
{
    return lzh_uniform_B_rows(0, n, b, seed, o64, o32);
}

int lzh_uniform_B_rows(int64_t r0, int64_t n, int b, uint64_t seed, double *o64, float *o32)
{
    if (n <= 0 || b <= 0 || r0 < 0) return -1;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t r = r0 + i;
        RowRng g(seed ^ 0x5bd1e995ULL, (uint64_t)r);
        for (int c = 0; c < b; ++c) {
            const double v = 1.0 + g.unif();
            if (o64) o64[i * b + c] = v;
            if (o32) o32[i * b + c] = (float)v;
        }
    }
    return 0;
}

int lzh_sym_eig(int k, const double *A, double *eval, double *evec)
{
    if (k <= 0 || !A || !eval) return -1;
    std::vector<double> V((size_t)k * k), d(k), e(k);
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j)  // lower triangle, mirrored
            V[(size_t)i * k + j] = (i >= j) ? A[(size_t)i * k + j] : A[(size_t)j * k + i];
    tred2(k, V, d, e);
    tql2(k, V, d, e);
    std::vector<int> order(k);
    for (int i = 0; i < k; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return d[a] < d[b]; });
    for (int i = 0; i < k; ++i) eval[i] = d[order[i]];
    if (evec)
        for (int r = 0; r < k; ++r)
            for (int i = 0; i < k; ++i) evec[(size_t)r * k + i] = V[(size_t)r * k + order[i]];
    return 0;
}

int lzh_assemble_T(int m, int b, const double *alpha, const double *beta, double *T)
{
    if (m <= 0 || b <= 0 || !alpha || !beta || !T) return -1;
    assemble_T(m, b, alpha, beta, T);
    return 0;
}

int lzh_ritz_values(int m, int b, const double *alpha, const double *beta, double *ritz)
{
    const int k = m * b;
    std::vector<double> T((size_t)k * k);
    if (lzh_assemble_T(m, b, alpha, beta, T.data())) return -1;
    return lzh_sym_eig(k, T.data(), ritz, nullptr);
}

int lzh_block_solution(int m, int b, double T_end, const double *alpha, const double *beta,
                       const double *q, double *solution)
{
    const int k = m * b;
    std::vector<double> T((size_t)k * k), V((size_t)k * k), ev(k), F((size_t)k * b);
    if (lzh_assemble_T(m, b, alpha, beta, T.data())) return -1;
    for (auto &x : T) x *= T_end;
    lzh_sym_eig(k, T.data(), ev.data(), V.data());
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < b; ++c) {
            double s = 0.0;
            for (int i = 0; i < k; ++i)
                s += V[(size_t)r * k + i] * std::exp(ev[i]) * V[(size_t)c * k + i];
            F[(size_t)r * b + c] = s;
        }
    for (int c = 0; c < b; ++c) {
        double s = 0.0;
        for (int r = 0; r < k; ++r) {
            double f = 0.0;
            for (int i = 0; i < b; ++i) f += F[(size_t)r * b + i] * beta[i * b + c];
            s += f * q[r];
        }
        solution[c] = s;
    }
    return 0;
}

int lzh_partition_rows(int64_t n, const int64_t *rp, int parts, int64_t *bounds)
{
    if (n < 0 || parts < 1 || !rp || !bounds) return -1;
    const int64_t nnz = rp[n];
    bounds[0] = 0;
    for (int p = 1; p < parts; ++p) {
        const int64_t target = (int64_t)((double)nnz * p / parts);
        int64_t r = std::lower_bound(rp, rp + n + 1, target) - rp;
        r = std::max(r, bounds[p - 1]);
        bounds[p] = std::min(r, n);
    }
    bounds[parts] = n;
    return 0;
}

int lzh_remap_cols_padded(int64_t nnz, const int32_t *col, int parts, const int64_t *bounds,
                          int64_t n_pad, int32_t *out)
{
    if (nnz < 0 || !col || !out || !bounds || parts < 1) return -1;
    if ((double)n_pad * parts > 2147483647.0) return -2;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t j = col[k];
        const int p = (int)(std::upper_bound(bounds, bounds + parts + 1, j) - bounds) - 1;
        out[k] = (int32_t)(p * n_pad + (j - bounds[p]));
    }
    return 0;
}

// Halo plan (SURVEY.md 8e "halo exchange of only the referenced columns"):
// the distinct off-rank columns of the local CSR, sorted ascending (so grouped
// by owner in rank order), and the columns rewritten into the compact
// numbering [0, n_local) = own rows, n_local + i = i-th halo row.
int64_t lzh_halo_plan(int64_t nnz, const int32_t *col, int parts, const int64_t *bounds, int rank,
                      int32_t *col_out, int64_t *recv_counts, int32_t *halo_rows)
{
    if (nnz < 0 || !col || !col_out || !bounds || !recv_counts || !halo_rows || parts < 1 ||
        rank < 0 || rank >= parts)
        return -1;
    const int64_t r0 = bounds[rank], r1 = bounds[rank + 1], nl = r1 - r0;
    std::vector<int32_t> off;
    off.reserve(1024);
    for (int64_t k = 0; k < nnz; ++k)
        if (col[k] < r0 || col[k] >= r1) off.push_back(col[k]);
    std::sort(off.begin(), off.end());
    off.erase(std::unique(off.begin(), off.end()), off.end());
    const int64_t nh = (int64_t)off.size();
    if ((double)nl + (double)nh > 2147483647.0) return -2;
    if (nh && (off.front() < 0 || off.back() >= bounds[parts])) return -3;
    std::copy(off.begin(), off.end(), halo_rows);
    for (int p = 0; p < parts; ++p)
        recv_counts[p] = std::lower_bound(off.begin(), off.end(), (int32_t)bounds[p + 1]) -
                         std::lower_bound(off.begin(), off.end(), (int32_t)bounds[p]);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) {
        const int32_t j = col[k];
        col_out[k] = (j >= r0 && j < r1)
                         ? (int32_t)(j - r0)
                         : (int32_t)(nl + (std::lower_bound(off.begin(), off.end(), j) - off.begin()));
    }
    return nh;
}

static const char kMagic[8] = {'L', 'Z', 'C', 'S', 'R', '0', '0', '1'};

int lzh_csr_write(const char *path, int64_t n, int64_t nc, int64_t nnz, const int64_t *rp,
                  const int32_t *col, const void *val, int dtype)
{
    FILE *f = std::fopen(path, "wb");
    if (!f) return -1;
    const int32_t dt = dtype, z = 0;
    const size_t vs = dtype == 0 ? 8 : 4;
    bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(&n, 8, 1, f) == 1 &&
              std::fwrite(&nc, 8, 1, f) == 1 && std::fwrite(&nnz, 8, 1, f) == 1 &&
              std::fwrite(&dt, 4, 1, f) == 1 && std::fwrite(&z, 4, 1, f) == 1 &&
              std::fwrite(rp, 8, n + 1, f) == (size_t)(n + 1) &&
              std::fwrite(col, 4, nnz, f) == (size_t)nnz &&
              std::fwrite(val, vs, nnz, f) == (size_t)nnz;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? 0 : -2;
}

int lzh_csr_read_header(const char *path, int64_t *n, int64_t *nc, int64_t *nnz, int *dtype)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) return -1;
    char mg[8];
    int32_t dt = 0, z = 0;
    const bool ok = std::fread(mg, 1, 8, f) == 8 && std::memcmp(mg, kMagic, 8) == 0 &&
                    std::fread(n, 8, 1, f) == 1 && std::fread(nc, 8, 1, f) == 1 &&
                    std::fread(nnz, 8, 1, f) == 1 && std::fread(&dt, 4, 1, f) == 1 &&
                    std::fread(&z, 4, 1, f) == 1;
    std::fclose(f);
    *dtype = dt;
    return ok ? 0 : -2;
}

int lzh_csr_read(const char *path, int64_t *rp, int32_t *col, void *val)
{
    int64_t n, nc, nnz;
    int dt;
    if (lzh_csr_read_header(path, &n, &nc, &nnz, &dt)) return -1;
    FILE *f = std::fopen(path, "rb");
    if (!f) return -1;
    std::fseek(f, 40, SEEK_SET);
    const size_t vs = dt == 0 ? 8 : 4;
    const bool ok = std::fread(rp, 8, n + 1, f) == (size_t)(n + 1) &&
                    std::fread(col, 4, nnz, f) == (size_t)nnz &&
                    std::fread(val, vs, nnz, f) == (size_t)nnz;
    std::fclose(f);
    return ok ? 0 : -2;
}

// matrix_a restatement: see lz_matrix_a.cpp
}  // extern "C"
