// oracle/ref_export.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A thin extern "C" shim that compiles the reference's own *host* code in place
// (headers under /root/reference/source, built with -DDISABLE_CUDA) so that the
// golden-vector script and the oracle self-checks can call the reference
// directly.  Nothing here is copied from the reference: every function below
// only calls the reference's own routines:
//
//   ref_matrix_a_*   -> Matrix_A<double>(N,N,N)            matrix_a/build_A_ell.hpp:8-255
//                       Ell_matrix::mult_diagonal           objects/ell_matrix.hpp:340-361
//                       Ell_matrix::change_order(4)         objects/ell_matrix.hpp:362-403 (buggy host path, :389)
//   ref_random_B     -> random_matrix_B<double>(n_rows)     matrix_a/build_ell_utils.hpp:271-280
//                       (after the one rand() draw main() spends on lc, test_lanczos.cu:326)
//   ref_ell_spmm     -> Ell_matrix::spmm host loop          objects/ell_matrix.hpp:287-300
//   ref_lc           -> 1 + rand()%100                      test_lanczos.cu:326
//
// Built by oracle/Makefile into oracle/_ref/libref_N{4,16}.so (N_COL is a
// compile-time constant in the reference, so one library per block width).
#include "utils/common.hpp"
#include "objects/ell_matrix.hpp"
#include "methods/copy_functions.hpp"
#include "matrix_a/build_A_ell.hpp"

#include <cstdlib>
#include <cstring>

#define REF_CAT2(a, b) a##b
#define REF_CAT(a, b) REF_CAT2(a, b)
#define REF_SYM(name) REF_CAT(REF_CAT(name, _N), N_COL)

namespace {
// Build A = D*W for the Yee grid of size N and return it (host ELL).
Ell_matrix<double> build_A(unsigned N, int change_order)
{
    auto info = Matrix_A<double>(N, N, N);
    Ell_matrix<double> D = info.first;
    Ell_matrix<double> W = info.second;
    D.mult_diagonal(W);
    if (change_order) D.change_order(4);
    return D;
}
}  // namespace

extern "C" {

// n_rows, total ELL slots, width of A for grid size N.
int REF_SYM(ref_matrix_a_shape)(unsigned N, unsigned long long *n_rows,
                                unsigned long long *size, unsigned long long *width)
{
    Ell_matrix<double> A = build_A(N, 0);
    *n_rows = A.n_rows();
    *size = A.size();
    *width = A.width();
    return 0;
}

// Copies the ELL data/idx arrays.  change_order=0: column-major slots
// (slot s of row r at r + s*n_rows); change_order=1: the as-run layout after the
// reference's host change_order(4) (row-major, stride 4).
int REF_SYM(ref_matrix_a)(unsigned N, int change_order, double *data, unsigned *idx)
{
    Ell_matrix<double> A = build_A(N, change_order);
    for (std::size_t i = 0; i < A.size(); ++i) {
        data[i] = A(i);
        idx[i] = A[i];
    }
    return 0;
}

// B exactly as the block driver builds it: srand() untouched (glibc seed 1),
// one draw for lc, then random_matrix_B (column-major n_rows x N_COL).
int REF_SYM(ref_random_B)(unsigned n_rows, double *out)
{
    srand(1);
    (void)rand();  // lc draw, test_lanczos.cu:326
    Dense_matrix<double> B = random_matrix_B<double>(n_rows);
    for (std::size_t i = 0; i < (std::size_t)n_rows * N_COL; ++i) out[i] = B(i);
    return 0;
}

unsigned REF_SYM(ref_lc)(void)
{
    srand(1);
    return 1 + (rand() % 100);
}

// Host ELL SpMM of the reference: Y = A*X with X, Y column-major n_rows x N_COL.
int REF_SYM(ref_ell_spmm)(unsigned long long n_rows, unsigned long long size,
                          const double *data, const unsigned *idx,
                          const double *X, double *Y)
{
    Ell_matrix<double> A(n_rows, size, n_rows, MemorySpace::Host);
    for (std::size_t i = 0; i < size; ++i) {
        A(i) = data[i];
        A[i] = idx[i];
    }
    Dense_matrix<double> Xm(n_rows, N_COL, MemorySpace::Host);
    Dense_matrix<double> Ym(n_rows, N_COL, MemorySpace::Host);
    for (std::size_t i = 0; i < n_rows * N_COL; ++i) Xm(i) = X[i];
    A.spmm(Xm, Ym);
    for (std::size_t i = 0; i < n_rows * N_COL; ++i) Y[i] = Ym(i);
    return 0;
}

}  // extern "C"
