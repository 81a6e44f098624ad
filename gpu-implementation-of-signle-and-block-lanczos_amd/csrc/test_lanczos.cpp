// test_lanczos.cpp -- the reference driver (test_lanczos.cu:131-362) rebuilt on
// the C++ drop-in layer include/lz_methods.hpp (the reference's methods/ API
// over the C ABI): same CLI (-N grid, -m iterations) and output lines, plus
// options for the block width, the operator and the validation run.
//
//   test_lanczos [-N 10] [-m 5] [--block 4] [--vector [--fp32]] [--unfused]
//                [--matrix matrix_a|banded|powerlaw|file:PATH] [--n ROWS]
//                [--nnz-per-row 10] [--halfwidth 4096] [--bug-compat-change-order]
//                [--fdtd-steps STEPS] [--T-end 1] [--lc ROW] [--device 0] [--row-major-B]
//
// Defaults reproduce the reference run: block Lanczos, b = 4 (N_COL), fp64, on
// the Yee operator of grid N with B from the glibc rand() stream and
// lc = 1 + rand() % 100 drawn first; B is stored as the reference stores it,
// column-major with its rows padded to a multiple of 768 (or 768 x #CU,
// test_lanczos.cu:174-187), and handed to block_lanczos_blas that way; the
// validation run is the reference's: 10^6 forward-Euler steps for the block
// path (:325,336), 10^5 for the single-vector one (:118).  --fdtd-steps 0
// skips it.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lz_methods.hpp"

#define CHECK(x)                                                                        \
    do {                                                                                \
        int rc_ = (x);                                                                  \
        if (rc_ != 0) {                                                                 \
            std::fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, lz_last_error());     \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)
struct Csr {
    int64_t n = 0, nnz = 0;
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    std::vector<double> val;
};

static Csr matrix_a(int N, bool bug)
{
    int64_t n, slots;
    CHECK(lzh_matrix_a_shape(N, &n, &slots));
    std::vector<double> d(slots);
    std::vector<uint32_t> ix(slots);
    CHECK(lzh_matrix_a_ell(N, bug ? 1 : 0, d.data(), ix.data()));
    Csr A;
    A.n = n;
    A.rp.resize(n + 1);
    A.nnz = lzh_ell_to_csr_count(n, 4, d.data(), ix.data(), 0, A.rp.data());
    A.col.resize(A.nnz);
    A.val.resize(A.nnz);
    CHECK(lzh_ell_to_csr_fill(n, 4, d.data(), ix.data(), 0, A.rp.data(), A.col.data(),
                              A.val.data()));
    return A;
}

int main(int argc, char **argv)
{
    int N = 10, m = 5, b = 4, device = 0;
    bool vector = false, unfused = false, bug = false, fp32 = false;
    std::string matrix = "matrix_a";
    int64_t nrows = 1000000, halfwidth = 4096, fdtd_steps = -1, lc = -1;
    bool row_major_B = false;
    double npr = 10.0, T_end = 1.0;
    for (int i = 1; i < argc; ++i) {
        std::string o = argv[i];
        auto nxt = [&]() -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", o.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (o == "-N") N = (int)std::stod(nxt());
        else if (o == "-m") m = (int)std::stod(nxt());
        else if (o == "--block") b = std::atoi(nxt());
        else if (o == "--vector") vector = true;
        else if (o == "--unfused") unfused = true;
        else if (o == "--fp32") fp32 = true;  // --vector: test_VectorLanczos<float> (test_lanczos.cu:355)
        else if (o == "--matrix") matrix = nxt();
        else if (o == "--n") nrows = (int64_t)std::stod(nxt());
        else if (o == "--nnz-per-row") npr = std::stod(nxt());
        else if (o == "--halfwidth") halfwidth = (int64_t)std::stod(nxt());
        else if (o == "--bug-compat-change-order") bug = true;
        else if (o == "--fdtd-steps") fdtd_steps = (int64_t)std::stod(nxt());
        else if (o == "--T-end") T_end = std::stod(nxt());
        else if (o == "--lc") lc = (int64_t)std::stod(nxt());
        else if (o == "--device") device = std::atoi(nxt());
        else if (o == "--row-major-B") row_major_B = true;  // B as an n x b row-major block instead
        else { std::fprintf(stderr, "unknown option %s\n", o.c_str()); return 2; }
    }
    if (vector) b = 1;
    if (fdtd_steps < 0) fdtd_steps = vector ? 100000 : 1000000;  // test_lanczos.cu:118 / :325,336
    if (fp32 && !vector) { std::fprintf(stderr, "--fp32 applies to --vector\n"); return 2; }
    if (lc < 0) lc = lzh_rand_lc(1);  // 1 + rand() % 100, test_lanczos.cu:326

    Csr A;
    if (matrix == "matrix_a") {
        A = matrix_a(N, bug);
    } else if (matrix == "banded" || matrix == "powerlaw") {
        A.n = nrows;
        A.rp.resize(nrows + 1);
        A.nnz = matrix == "banded"
                    ? lzh_gen_banded_count(nrows, npr, halfwidth, 20261015ULL, A.rp.data())
                    : lzh_gen_powerlaw_count(nrows, npr, 2.1, 100000, 20261015ULL, A.rp.data());
        A.col.resize(A.nnz);
        A.val.resize(A.nnz);
        if (matrix == "banded")
            CHECK(lzh_gen_banded_fill(nrows, npr, halfwidth, 20261015ULL, A.rp.data(),
                                      A.col.data(), A.val.data(), nullptr));
        else
            CHECK(lzh_gen_powerlaw_fill(nrows, npr, 2.1, 100000, 20261015ULL, A.rp.data(),
                                        A.col.data(), A.val.data(), nullptr));
    } else if (matrix.rfind("file:", 0) == 0) {
        const std::string path = matrix.substr(5);
        int64_t nc;
        int dt;
        CHECK(lzh_csr_read_header(path.c_str(), &A.n, &nc, &A.nnz, &dt));
        if (dt != 0) { std::fprintf(stderr, "file must hold fp64 values\n"); return 2; }
        A.rp.resize(A.n + 1);
        A.col.resize(A.nnz);
        A.val.resize(A.nnz);
        CHECK(lzh_csr_read(path.c_str(), A.rp.data(), A.col.data(), A.val.data()));
    } else {
        std::fprintf(stderr, "unknown --matrix %s\n", matrix.c_str());
        return 2;
    }
    const int64_t n = A.n;
    if (lc >= n) lc = n - 1;
    std::printf(" the size of the problem is \n%lld\n", (long long)n);

    // B: glibc rand() stream after the lc draw (random_matrix_B), row-major n x b
    std::vector<double> B((size_t)n * b);
    CHECK(lzh_rand_B(n, b, 1, 1, 1, B.data()));

    // the reference driver's objects (test_lanczos.cu:190-236) as lz_methods.hpp containers
    lz::Context ctx(device);
    lz::Csr_matrix<double> Ad(n, n, A.rp, A.col, A.val);
    lz::Vector<double> q((int64_t)m * b);
    std::vector<double> alpha, beta;  // host copies, m * b * b and (m + 1) * b * b
    std::vector<double> sol;
    std::vector<double> qh;
    if (vector && fp32) {
        std::vector<float> bvec(n), vf(A.val.begin(), A.val.end());
        for (int64_t r = 0; r < n; ++r) bvec[r] = (float)B[r];
        lz::Csr_matrix<float> Af(n, n, A.rp, A.col, vf);
        lz::Vector<float> bv(bvec), q0(n), q1(n), w(n), qf(m);
        std::vector<float> al(m), be(m);
        std::printf(" start Lanczos \n");
        auto t0 = std::chrono::steady_clock::now();
        lz::vector_lanczos(Af, bv, m, lc, qf, al.data(), be.data(), q0, q1, w, ctx);
        auto t1 = std::chrono::steady_clock::now();
        std::printf(" end Lanczos \n");
        std::printf("elapsed time: %11.6f\n", std::chrono::duration<double>(t1 - t0).count());
        alpha.assign(al.begin(), al.end());
        beta.assign(be.begin(), be.end());
        beta.push_back(0.0);
        const std::vector<float> qv = qf.copy_to_host();
        qh.assign(qv.begin(), qv.end());
    } else if (vector) {
        std::vector<double> bvec(n);
        for (int64_t r = 0; r < n; ++r) bvec[r] = B[r];
        lz::Vector<double> bv(bvec), q0(n), q1(n), w(n);
        std::vector<double> al(m), be(m);
        std::printf(" start Lanczos \n");
        auto t0 = std::chrono::steady_clock::now();
        lz::vector_lanczos(Ad, bv, m, lc, q, al.data(), be.data(), q0, q1, w, ctx);
        auto t1 = std::chrono::steady_clock::now();
        std::printf(" end Lanczos \n");
        std::printf("elapsed time: %11.6f\n", std::chrono::duration<double>(t1 - t0).count());
        // scalar recurrence: beta[0] = ||b||; T off-diagonal = beta[1..]
        alpha = al;
        beta = be;
        beta.push_back(0.0);
    } else {
        // the reference's padding of B (test_lanczos.cu:174-187): rows up to a
        // multiple of 768 (6 warps x 4 x 32), or of 768 x #CU for large n
        int ncu = 0;
        lz::hip_check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device), "CU count");
        const int64_t pads = n < 768LL * ncu ? 768 : 768LL * ncu;
        const int64_t ld = (n + pads - 1) / pads * pads;
        std::vector<double> Bcm((size_t)ld * b, 0.0);
        for (int64_t r = 0; r < n; ++r)
            for (int c = 0; c < b; ++c) Bcm[(size_t)c * ld + r] = B[(size_t)r * b + c];
        lz::Dense_matrix<double> Bm = row_major_B ? lz::Dense_matrix<double>(n, b, B)
                                                  : lz::Dense_matrix<double>(ld, b, Bcm, LZ_COL_MAJOR, ld);
        lz::Dense_matrix<double> Q0(ld, b, LZ_COL_MAJOR, ld), Q1(ld, b, LZ_COL_MAJOR, ld), W(ld, b, LZ_COL_MAJOR, ld);
        std::vector<lz::Dense_matrix<double>> al, be;
        for (int j = 0; j < m; ++j) al.emplace_back(b, b);
        for (int j = 0; j <= m; ++j) be.emplace_back(b, b);
        std::printf(" start Lanczos \n");
        auto t0 = std::chrono::steady_clock::now();
        if (unfused)
            lz::block_lanczos_blas_reference_order(Ad, Bm, m, lc, q, al.data(), be.data(), Q0, Q1, W, ctx);
        else
            lz::block_lanczos_blas(Ad, Bm, m, lc, q, al.data(), be.data(), Q0, Q1, W, ctx);
        auto t1 = std::chrono::steady_clock::now();
        std::printf(" end Lanczos \n");
        std::printf("elapsed time: %11.6f\n", std::chrono::duration<double>(t1 - t0).count());
        if (ctx.device_error()) {
            std::fprintf(stderr, "device error word set: results invalid\n");
            return 1;
        }
        for (auto &x : al) {
            const auto v = x.copy_to_host();
            alpha.insert(alpha.end(), v.begin(), v.end());
        }
        for (auto &x : be) {
            const auto v = x.copy_to_host();
            beta.insert(beta.end(), v.begin(), v.end());
        }
    }
    if (!(vector && fp32)) qh = q.copy_to_host();
    const std::vector<double> ritz = lz::ritz_values(m, b, alpha, beta);
    sol = lz::block_solution(m, b, T_end, alpha, beta, qh);
    std::printf("Ritz values (%d):", m * b);
    for (double r : ritz) std::printf(" %.15e", r);
    if (vector) {  // test_lanczos.cu:111-112
        std::printf("\nThe solution for vector_lanczos \n%.15e\n", sol[0]);
    } else {       // test_lanczos.cu:288-289
        std::printf("\nSolution for block lanczos\n");
        for (double s : sol) std::printf("%.15e\n", s);
    }

    if (fdtd_steps > 0) {
        lz::Dense_matrix<double> U0(n, b, B);
        if (vector) {  // fdtd_vector(A, b, 1e5, 1, lc), test_lanczos.cu:118-123
            const std::vector<double> fd = lz::ftdt_block(Ad, U0, (unsigned)fdtd_steps, T_end, lc, ctx);
            std::printf("Solution from fdtd %.15e\n", fd[0]);
            std::printf("Relative error for block lanczos is %.6e\n", std::fabs(sol[0] - fd[0]) / std::fabs(fd[0]));
            return 0;
        }
        std::printf(" start fdtd \n");  // ftdt_block(A, B, fdtd_steps, T_end, lc), test_lanczos.cu:292-301
        const std::vector<double> fd = lz::ftdt_block(Ad, U0, (unsigned)fdtd_steps, T_end, lc, ctx);
        std::printf("Solution from fdtd\n");
        double num = 0, den = 0;
        for (int c = 0; c < b; ++c) {
            std::printf("%.15e\n", fd[c]);
            num += (sol[c] - fd[c]) * (sol[c] - fd[c]);
            den += fd[c] * fd[c];
        }
        std::printf("Relative error for block lanczos is %.6e\n", std::sqrt(num / den));
    }
    return 0;
}
