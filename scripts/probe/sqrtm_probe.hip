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
    hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, dG, nullptr, 0, db, dbi, nullptr, nullptr, nullptr);
    hipEventRecord(e0);
    const int R = 20;
    for (int r = 0; r < R; ++r)
        hipLaunchKernelGGL((lzprobe::k_sqrtm_b<double, B>), dim3(1), dim3(1024), 0, 0, dG, nullptr, 0, db, dbi, nullptr, nullptr, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long pr[2];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(lzprobe::lz_sqrtm_probe), sizeof(pr));
    std::printf("B=%d cond=%.0e  %.2f us/launch  sweeps=%lld  jacobi_cycles=%lld (%.1f per round)\n", B, cond,
                ms * 1e3 / R, pr[0], pr[1], double(pr[1]) / ((pr[0] + 1) * (B - 1)));
    hipFree(dG); hipFree(db); hipFree(dbi);
}

int main()
{
    for (double c : {1e2, 1e12}) { run<8>(c); run<16>(c); run<32>(c); }
    // empty-ish launch floor
    return 0;
}
