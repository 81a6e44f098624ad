// Sweep count / cycle probe of k_sqrtm_b (build: scripts/probe/Makefile).
// Compiled under a private namespace so its kernels cannot alias liblz_hip.so's.
#define LZ_SQRTM_PROBE 1
#define lz lzprobe
#include "../../gpu-implementation-of-signle-and-block-lanczos_amd/csrc/lz_dense.hip"
#include <cstdarg>
namespace lzprobe {
void set_error(const char *, ...) {}
int prof_begin(lz_handle *, int) { return -1; }
void prof_end(lz_handle *, int) {}
int ensure_partials(lz_handle *, size_t) { return 0; }
}  // namespace lzprobe
#include <cmath>
#include <random>
#include <vector>

template <int B>
static void run(double cond)
{
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd;
    // G = Q diag(ev) Q^T with Q from Gram-Schmidt of a Gaussian matrix
    std::vector<double> Q(B * B), G(B * B, 0.0);
    for (auto &x : Q) x = nd(rng);
    for (int c = 0; c < B; ++c) {
        for (int k = 0; k < c; ++k) {
            double d = 0;
            for (int r = 0; r < B; ++r) d += Q[r * B + c] * Q[r * B + k];
            for (int r = 0; r < B; ++r) Q[r * B + c] -= d * Q[r * B + k];
        }
        double nn = 0;
        for (int r = 0; r < B; ++r) nn += Q[r * B + c] * Q[r * B + c];
        nn = std::sqrt(nn);
        for (int r = 0; r < B; ++r) Q[r * B + c] /= nn;
    }
    for (int k = 0; k < B; ++k) {
        const double ev = std::pow(cond, -double(k) / (B - 1));
        for (int i = 0; i < B; ++i)
            for (int j = 0; j < B; ++j) G[i * B + j] += Q[i * B + k] * ev * Q[j * B + k];
    }
    double *dG, *db, *dbi;
    hipMalloc(&dG, B * B * 8); hipMalloc(&db, B * B * 8); hipMalloc(&dbi, B * B * 8);
    hipMemcpy(dG, G.data(), B * B * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, dG, nullptr, 0, db, dbi, nullptr, nullptr, nullptr, lzprobe::WfAlpha{}, 0);
    hipEventRecord(e0);
    const int R = 20;
    for (int r = 0; r < R; ++r)
        hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, dG, nullptr, 0, db, dbi, nullptr, nullptr, nullptr, lzprobe::WfAlpha{}, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long pr[2];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(lzprobe::lz_sqrtm_probe), sizeof(pr));
    std::printf("B=%d cond=%.0e  %.2f us/launch  sweeps=%lld  jacobi_cycles=%lld (%.1f per round)\n", B, cond,
                ms * 1e3 / R, pr[0], pr[1], double(pr[1]) / ((pr[0] + 1) * (B - 1)));
    hipFree(dG); hipFree(db); hipFree(dbi);
}

// The wavefront step's call (B = 16): G, S1 and S2 from P slabs each, then the
// alpha products; against the same G from 1 slab and from the matrix itself.
static void run_wf(int P, bool alpha, int ns)
{
    constexpr int B = 16;
    std::mt19937_64 rng(2);
    std::normal_distribution<double> nd;
    std::vector<double> part(3 * (size_t)P * 256), X(B * B);
    for (auto &x : X) x = nd(rng);
    for (int p = 0; p < P; ++p)
        for (int i = 0; i < B; ++i)
            for (int j = 0; j < B; ++j) {
                double g = 0;
                for (int k = 0; k < B; ++k) g += X[i * B + k] * X[j * B + k];
                part[(2 * (size_t)P + p) * 256 + i * B + j] = (g + (i == j ? 1.0 : 0.0)) / P;
                part[(size_t)p * 256 + i * B + j] = nd(rng) / P;
                part[((size_t)P + p) * 256 + i * B + j] = nd(rng) / P;
            }
    double *dp, *db, *dbi, *dL, *dLB, *da, *dP2, *dV, *dq;
    hipMalloc(&dp, part.size() * 8);
    hipMalloc(&db, 2048); hipMalloc(&dbi, 2048); hipMalloc(&dL, 2048); hipMalloc(&dLB, 2048);
    hipMalloc(&da, 2048); hipMalloc(&dP2, 2048); hipMalloc(&dV, 16 * 128); hipMalloc(&dq, 128);
    hipMemcpy(dp, part.data(), part.size() * 8, hipMemcpyHostToDevice);
    hipMemset(dL, 0, 2048); hipMemset(dV, 0, 16 * 128);
    lzprobe::WfAlpha wa{};
    if (alpha) {
        wa.part = dp; wa.P = P; wa.alpha = da; wa.P2 = dP2; wa.V = dV; wa.lc = 3; wa.qrow = dq;
    }
    auto go = [&]() {
        hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, nullptr,
                           dp + 2 * (size_t)P * 256, P, db, dbi, nullptr, dL, dLB, wa, ns);
    };
    go();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    const int R = 20;
    for (int r = 0; r < R; ++r) go();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long pr[2];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(lzprobe::lz_sqrtm_probe), sizeof(pr));
    std::printf("wf B=16 P=%d alpha=%d ns=%d  %.2f us/launch  sweeps=%lld  jacobi_cycles=%lld\n", P, (int)alpha,
                ns, ms * 1e3 / R, pr[0], pr[1]);
    hipFree(dp);
}

// Newton-Schulz (ns = 1) against the Jacobi route (ns = 0) on the same G of
// condition number cond: time per launch and the largest relative difference
// of beta and beta^-1 (a fallback to Jacobi shows as a difference of 0).
static void run_ns(double cond)
{
    constexpr int B = 16;
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    std::vector<double> Q(B * B), G(B * B, 0.0);
    for (auto &x : Q) x = nd(rng);
    for (int c = 0; c < B; ++c) {
        for (int k = 0; k < c; ++k) {
            double d = 0;
            for (int r = 0; r < B; ++r) d += Q[r * B + c] * Q[r * B + k];
            for (int r = 0; r < B; ++r) Q[r * B + c] -= d * Q[r * B + k];
        }
        double nn = 0;
        for (int r = 0; r < B; ++r) nn += Q[r * B + c] * Q[r * B + c];
        nn = std::sqrt(nn);
        for (int r = 0; r < B; ++r) Q[r * B + c] /= nn;
    }
    for (int k = 0; k < B; ++k) {
        const double ev = 3.7 * std::pow(cond, -double(k) / (B - 1));
        for (int i = 0; i < B; ++i)
            for (int j = 0; j < B; ++j) G[i * B + j] += Q[i * B + k] * ev * Q[j * B + k];
    }
    double *dG, *db, *dbi;
    hipMalloc(&dG, B * B * 8); hipMalloc(&db, B * B * 8); hipMalloc(&dbi, B * B * 8);
    hipMemcpy(dG, G.data(), B * B * 8, hipMemcpyHostToDevice);
    std::vector<double> b[2], bi[2];
    float us[2];
    for (int ns = 0; ns < 2; ++ns) {
        auto go = [&]() {
            hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, dG, nullptr, 0, db, dbi,
                               nullptr, nullptr, nullptr, lzprobe::WfAlpha{}, ns);
        };
        go();
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) go();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        us[ns] = ms * 1e3f / 20;
        b[ns].resize(B * B); bi[ns].resize(B * B);
        hipMemcpy(b[ns].data(), db, B * B * 8, hipMemcpyDeviceToHost);
        hipMemcpy(bi[ns].data(), dbi, B * B * 8, hipMemcpyDeviceToHost);
    }
    double nb = 0, nbi = 0, db_ = 0, dbi_ = 0;
    for (int e = 0; e < B * B; ++e) {
        nb = std::fmax(nb, std::fabs(b[0][e]));
        nbi = std::fmax(nbi, std::fabs(bi[0][e]));
        db_ = std::fmax(db_, std::fabs(b[1][e] - b[0][e]));
        dbi_ = std::fmax(dbi_, std::fabs(bi[1][e] - bi[0][e]));
    }
    std::printf("NS vs Jacobi  cond(G)=%.0e  jacobi %.2f us  ns %.2f us  max|dbeta|/max|beta| %.2e  "
                "max|dbinv|/max|binv| %.2e\n", cond, us[0], us[1], db_ / nb, dbi_ / nbi);
    hipFree(dG); hipFree(db); hipFree(dbi);
}

int main()
{
    for (double c : {1.0, 1e2, 1e4, 1e6, 1e8, 1e10, 1e12, 1e16}) run_ns(c);
    for (int P : {1, 256}) { run_wf(P, false, 0); run_wf(P, true, 0); run_wf(P, true, 1); }
    for (double c : {1e2, 1e12}) { run<8>(c); run<16>(c); run<32>(c); }
    // empty-ish launch floor
    return 0;
}
