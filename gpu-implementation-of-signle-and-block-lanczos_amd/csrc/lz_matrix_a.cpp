// lz_matrix_a.cpp -- restatement of the reference's problem generator: the
// Yee-grid Maxwell operator A = D*W (matrix_a/build_A_ell.hpp:8-255 with the
// helpers of matrix_a/build_ell_utils.hpp and Ell_matrix::mult_diagonal,
// objects/ell_matrix.hpp:340-361), reproducing the reference's floating-point
// operation order so the values are bit-identical (checked against the
// reference's own host code compiled in place: tests/test_host.py and
// tests/test_oracle.py against oracle/_ref).
//
// Storage: "ELL, column-major slots" like the reference before change_order:
// slot s of row r at r + s*n_rows, uint32 column index, explicit zeros kept.
#include <cstdint>
#include <vector>

#include "lz_host.h"

namespace {

struct Ell {
    int64_t rows = 0, cols = 0, width = 0;
    std::vector<double> d;
    std::vector<uint32_t> ix;
    Ell() = default;
    // Ell_matrix(n_rows, size, n_cols): zero data / zero indices, width = size/rows
    Ell(int64_t r, int64_t size, int64_t c) : rows(r), cols(c), width(size / r), d(size, 0.0), ix(size, 0) {}
    int64_t size() const { return (int64_t)d.size(); }
};

struct Dense {  // column-major
    int64_t rows = 0, cols = 0;
    std::vector<double> a;
    Dense(int64_t r, int64_t c) : rows(r), cols(c), a(r * c, 0.0) {}
    double &at(int64_t i, int64_t j) { return a[i + rows * j]; }
};

std::vector<double> linspace(double xl, double xr, int64_t N)  // build_ell_utils.hpp:94-106
{
    const double h = (xr - xl) / (N - 1);
    std::vector<double> g(N);
    for (int64_t i = 0; i < N; ++i) g[i] = xl + i * h;
    return g;
}

std::vector<double> diff(const std::vector<double> &v)  // :83-92
{
    std::vector<double> o(v.size() - 1);
    for (size_t i = 0; i < o.size(); ++i) o[i] = v[i + 1] - v[i];
    return o;
}

Dense diag_of(const std::vector<double> &v)  // Dense_matrix(const Vector&), dense_matrix.hpp:107-131
{
    Dense D((int64_t)v.size(), (int64_t)v.size());
    for (size_t i = 0; i < v.size(); ++i) D.at(i, i) = v[i];
    return D;
}

Dense diag_inv(Dense D)  // :168-179
{
    for (int64_t i = 0; i < D.rows; ++i) D.at(i, i) = 1. / D.at(i, i);
    return D;
}

Dense bidiagonal(int64_t N, double dg, double up)  // :122-138
{
    Dense R(N, N + 1);
    for (int64_t i = 0; i < N; ++i) {
        R.a[i + N * i] = dg;
        R.a[i + N * (i + 1)] = up;
    }
    return R;
}

Dense transpose(const Dense &M)  // Dense_matrix::tra, dense_matrix.hpp:324-334
{
    Dense T(M.cols, M.rows);
    for (int64_t c = 0; c < M.cols; ++c)
        for (int64_t r = 0; r < M.rows; ++r) T.a[c + M.cols * r] = M.a[r + M.rows * c];
    return T;
}

// this = my*this + other*A*B on a zero-initialised this (Dense_matrix::mm, :299-323)
Dense mm(const Dense &A, const Dense &B, int64_t rows, int64_t cols)
{
    Dense R(rows, cols);
    for (int64_t c = 0; c < cols; ++c)
        for (int64_t r = 0; r < rows; ++r) {
            double sum = 0;
            for (int64_t el = 0; el < A.cols; ++el) sum += A.a[r + rows * el] * B.a[el + A.cols * c];
            R.a[r + rows * c] = 0. * R.a[r + rows * c] + 1. * sum;
        }
    return R;
}

void dense_scale(Dense &M, double s)  // mult_scalar -> sadd(s, 0, *this), :336-371
{
    for (auto &x : M.a) x = s * x + 0. * x;
}

Ell dense_to_ell(const Dense &M, int64_t width)  // build_ell_utils.hpp:141-166
{
    Ell e(M.rows, width * M.rows, M.cols);
    for (int64_t i = 0; i < M.rows; ++i) {
        int64_t ind = 0;
        for (int64_t j = 0; j < M.cols; ++j) {
            const double v = M.a[i + j * M.rows];
            if (v != 0) {
                e.d[i + ind * M.rows] = v;
                e.ix[i + ind * M.rows] = (uint32_t)j;
                ++ind;
            }
        }
    }
    return e;
}

Ell ell_diag(int64_t N, double s)  // diag, build_ell_utils.hpp:108-119
{
    Ell I(N, N, N);
    for (int64_t i = 0; i < N; ++i) {
        I.d[i] = s;
        I.ix[i] = (uint32_t)i;
    }
    return I;
}

Ell kronI(const Ell &X, const Ell &I)  // build_ell_utils.hpp:37-58
{
    const int64_t Ir = I.rows, Xr = X.rows, Xs = X.size(), Xc = X.cols;
    Ell R(Ir * Xr, Ir * Xs, Ir * Xc);
    for (int64_t j = 0; j < Ir; ++j)
        for (int64_t i = 0; i < Xs; ++i) {
            R.d[i * Ir + j] = X.d[i] * I.d[j];
            R.ix[i * Ir + j] = (uint32_t)(X.ix[i] * Ir + j);
        }
    return R;
}

Ell Ikron(const Ell &I, const Ell &X)  // build_ell_utils.hpp:8-33
{
    const int64_t Ir = I.rows, Xw = X.width, Xr = X.rows, Xs = X.size(), Xc = X.cols;
    Ell R(Ir * Xr, Ir * Xs, Ir * Xc);
    for (int64_t j = 0; j < Xw; ++j)
        for (int64_t i = 0; i < Xr * Ir; ++i) {
            R.d[i + j * (Xr * Ir)] = X.d[i % Xr + j * Xr];
            R.ix[i + j * (Xr * Ir)] = (uint32_t)(X.ix[i % Xr + j * Xr] + Xc * (i / Xr));
        }
    return R;
}

void insert(Ell &D, const Ell &d, int64_t r_loc, int64_t c_loc, int64_t c_shift)  // :61-81
{
    const int64_t dc = d.width, dr = d.rows, Dr = D.rows;
    const int64_t start = r_loc + c_loc * Dr;
    for (int64_t j = 0; j < dc; ++j)
        for (int64_t i = 0; i < dr; ++i) {
            D.d[start + i + j * Dr] = d.d[i + j * dr];
            D.ix[start + i + j * Dr] = (uint32_t)(d.ix[i + j * dr] + c_shift);
        }
}

void ell_scale(Ell &E, double s)  // Ell_matrix::mult_scalar, ell_matrix.hpp:253-266
{
    for (auto &x : E.d) x = x * s;
}

Ell build_A(int64_t N)
{
    const int64_t Nx = N, Ny = N, Nz = N;
    const double xl = 0., xr = 1., yl = 0., yr = 1., zl = 0., zr = 1.;
    const int64_t Nxp = Nx + 2, Nyp = Ny + 2, Nzp = Nz + 2;
    const double hx = (xr - xl) / (Nxp - 1), hy = (yr - yl) / (Nyp - 1), hz = (zr - zl) / (Nzp - 1);
    auto shift = [](std::vector<double> v, double s) {  // Vector::add_scalar = sadd(1,1,vec)
        for (auto &x : v) x = 1. * x + 1. * s;
        return v;
    };
    auto x_p = linspace(xl, xr, Nxp), x_d = shift(linspace(xl, xr - hx, Nxp - 1), hx / 2);
    auto y_p = linspace(yl, yr, Nyp), y_d = shift(linspace(yl, yr - hy, Nyp - 1), hy / 2);
    auto z_p = linspace(zl, zr, Nzp), z_d = shift(linspace(zl, zr - hz, Nzp - 1), hz / 2);
    auto dxp = diff(x_p), dxd = diff(x_d), dyp = diff(y_p), dyd = diff(y_d), dzp = diff(z_p),
         dzd = diff(z_d);
    Dense Wx_ = diag_of(dxp), Wxh_ = diag_of(dxd), Wy_ = diag_of(dyp), Wyh_ = diag_of(dyd),
          Wz_ = diag_of(dzp), Wzh_ = diag_of(dzd);
    Dense Wxi = diag_inv(Wx_), Wxhi = diag_inv(Wxh_), Wyi = diag_inv(Wy_), Wyhi = diag_inv(Wyh_),
          Wzi = diag_inv(Wz_), Wzhi = diag_inv(Wzh_);
    Dense bx = bidiagonal(Nx, 1., -1.), bxT = transpose(bx);
    Dense by = bidiagonal(Ny, 1., -1.), byT = transpose(by);
    Dense bz = bidiagonal(Nz, 1., -1.), bzT = transpose(bz);
    Dense X_ = mm(Wxi, bxT, Nx + 1, Nx), Y_ = mm(Wyi, byT, Ny + 1, Ny), Z_ = mm(Wzi, bzT, Nz + 1, Nz);
    Dense Xh_ = mm(Wxhi, bx, Nx, Nx + 1), Yh_ = mm(Wyhi, by, Ny, Ny + 1),
          Zh_ = mm(Wzhi, bz, Nz, Nz + 1);
    dense_scale(Xh_, -1.);
    dense_scale(Yh_, -1.);
    dense_scale(Zh_, -1.);
    Ell X = dense_to_ell(X_, 2), Y = dense_to_ell(Y_, 2), Z = dense_to_ell(Z_, 2);
    Ell Xh = dense_to_ell(Xh_, 2), Yh = dense_to_ell(Yh_, 2), Zh = dense_to_ell(Zh_, 2);
    Ell W_x = dense_to_ell(Wx_, 1), W_y = dense_to_ell(Wy_, 1), W_z = dense_to_ell(Wz_, 1);
    Ell W_xh = dense_to_ell(Wxh_, 1), W_yh = dense_to_ell(Wyh_, 1), W_zh = dense_to_ell(Wzh_, 1);
    Ell Ix = ell_diag(Nx, 1.), Iy = ell_diag(Ny, 1.), Iz = ell_diag(Nz, 1.);
    Ell Ixp = ell_diag(Nx + 1, 1.), Iyp = ell_diag(Ny + 1, 1.), Izp = ell_diag(Nz + 1, 1.);

    Ell De_12 = kronI(Z, kronI(Iyp, Ix));
    Ell De_13 = Ikron(Izp, kronI(Y, Ix));
    Ell De_21 = kronI(Z, Ikron(Iy, Ixp));
    Ell De_23 = Ikron(Izp, Ikron(Iy, X));
    Ell De_31 = Ikron(Iz, kronI(Y, Ixp));
    Ell De_32 = Ikron(Iz, Ikron(Iyp, X));
    ell_scale(De_12, -1.);
    ell_scale(De_23, -1.);
    ell_scale(De_31, -1.);
    Ell Dh_12 = kronI(Zh, Ikron(Iy, Ixp));
    Ell Dh_13 = Ikron(Iz, kronI(Yh, Ixp));
    Ell Dh_21 = kronI(Zh, Ikron(Iyp, Ix));
    Ell Dh_23 = Ikron(Iz, Ikron(Iyp, Xh));
    Ell Dh_31 = Ikron(Izp, kronI(Yh, Ix));
    Ell Dh_32 = Ikron(Izp, Ikron(Iy, Xh));
    ell_scale(Dh_13, -1.);
    ell_scale(Dh_21, -1.);
    ell_scale(Dh_32, -1.);

    const int64_t De_rows = De_12.rows + De_21.rows + De_31.rows;
    const int64_t De_size = De_12.size() + De_21.size() + De_31.size() + De_13.size() +
                            De_23.size() + De_32.size();
    const int64_t Dh_rows = Dh_12.rows + Dh_21.rows + Dh_31.rows;
    const int64_t Dh_size = Dh_12.size() + Dh_21.size() + Dh_31.size() + Dh_13.size() +
                            Dh_23.size() + Dh_32.size();
    Ell De(De_rows, De_size, Dh_rows), Dh(Dh_rows, Dh_size, De_rows);
    Ell D(De_rows + Dh_rows, De_size + Dh_size, De_rows + Dh_rows);
    int64_t s1 = Dh_12.rows, s2 = Dh_21.rows;
    insert(De, De_12, 0, 0, s1);
    insert(De, De_13, 0, De_12.width, s1 + s2);
    insert(De, De_21, De_12.rows, 0, 0);
    insert(De, De_23, De_12.rows, De_12.width, s1 + s2);
    insert(De, De_31, De_12.rows + De_21.rows, 0, 0);
    insert(De, De_32, De_12.rows + De_21.rows, De_12.width, s1);
    s1 = De_12.rows;
    s2 = De_21.rows;
    insert(Dh, Dh_12, 0, 0, s1);
    insert(Dh, Dh_13, 0, Dh_12.width, s1 + s2);
    insert(Dh, Dh_21, Dh_12.rows, 0, 0);
    insert(Dh, Dh_23, Dh_12.rows, Dh_12.width, s1 + s2);
    insert(Dh, Dh_31, Dh_12.rows + Dh_21.rows, 0, 0);
    insert(Dh, Dh_32, Dh_12.rows + Dh_21.rows, Dh_12.width, s1);
    insert(D, Dh, 0, 0, Dh_12.rows + Dh_21.rows + Dh_31.rows);
    insert(D, De, Dh.rows, 0, 0);

    Ell We_11 = kronI(W_zh, kronI(W_yh, W_x));
    Ell We_22 = kronI(W_zh, kronI(W_y, W_xh));
    Ell We_33 = kronI(W_z, kronI(W_yh, W_xh));
    Ell Wh_11 = kronI(W_z, kronI(W_y, W_xh));
    Ell Wh_22 = kronI(W_z, kronI(W_yh, W_x));
    Ell Wh_33 = kronI(W_zh, kronI(W_y, W_x));
    const int64_t We_rows = We_11.rows + We_22.rows + We_33.rows;
    const int64_t We_size = We_11.size() + We_22.size() + We_33.size();
    const int64_t Wh_rows = Wh_11.rows + Wh_22.rows + Wh_33.rows;
    const int64_t Wh_size = Wh_11.size() + Wh_22.size() + Wh_33.size();
    Ell We(We_rows, We_size, We_rows), Wh(Wh_rows, Wh_size, Wh_rows);
    insert(We, We_11, 0, 0, 0);
    insert(We, We_22, We_11.rows, 0, We_11.rows);
    insert(We, We_33, We_11.rows + We_22.rows, 0, We_11.rows + We_22.rows);
    insert(Wh, Wh_11, 0, 0, 0);
    insert(Wh, Wh_22, Wh_11.rows, 0, Wh_11.rows);
    insert(Wh, Wh_33, Wh_11.rows + Wh_22.rows, 0, Wh_11.rows + Wh_22.rows);
    ell_scale(Wh, -1.);
    Ell W(We.rows + Wh.rows, We.size() + Wh.size(), We.rows + Wh.rows);
    insert(W, We, 0, 0, 0);
    insert(W, Wh, We.rows, 0, We.rows);

    // A = D*W  (Ell_matrix::mult_diagonal)
    for (int64_t i = 0; i < D.size(); ++i) D.d[i] = D.d[i] * W.d[D.ix[i]];
    return D;
}

}  // namespace

extern "C" {

int lzh_matrix_a_shape(int N, int64_t *n_rows, int64_t *slots)
{
    if (N < 1 || !n_rows || !slots) return -1;
    const int64_t n = 3LL * N * (N + 1) * (2LL * N + 1);
    *n_rows = n;
    *slots = 4 * n;
    return 0;
}

int lzh_matrix_a_ell(int N, int bug_compat, double *data, uint32_t *idx)
{
    if (N < 1 || !data || !idx) return -1;
    Ell A = build_A(N);
    if (A.width != 4) return -2;
    const int64_t n = A.rows;
    for (int64_t i = 0; i < A.size(); ++i) {
        // change_order(4) as it runs (objects/ell_matrix.hpp:389): only slot 0 survives
        const bool keep = !bug_compat || i < n;
        data[i] = keep ? A.d[i] : 0.0;
        idx[i] = keep ? A.ix[i] : 0u;
    }
    return 0;
}

}  // extern "C"
