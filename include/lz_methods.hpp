/* include/lz_methods.hpp -- header-only C++ drop-in for the reference's
 * methods/ and kernels/ operator API on MI355X (gfx950), built on the C ABI of
 * liblz_hip.so (lz_hip.h) and liblz_host.so (lz_host.h).
 *
 * A reference caller (ibrohimmn1994/GPU-implementation-of-signle-and-block-Lanczos,
 * paths relative to source/) keeps its call sites and argument order:
 *
 *   reference                                                   here
 *   block_lanczos_blas<T>(A, B, m, lc, q, alpha, beta,          lz::block_lanczos_blas<T>(A, B, m, lc, q,
 *       Q0, Q1, W, args, eigen_val, cublasH, n_blocks, n_loads)     alpha, beta, Q0, Q1, W, ctx, eigen_val,
 *       (methods/block_lanczos.hpp:88-103)                          n_blocks, n_loads)
 *   vector_lanczos<T>(A, b, m, lc, q, alpha, beta, q0, q1, w)   lz::vector_lanczos<T>(...same..., ctx)
 *       (methods/vector_lanczos.hpp:8-18)
 *   spmm(Ell_matrix&, Dense_matrix& X, Dense_matrix& Y)         lz::spmm(A, X, Y[, ctx])
 *       (kernels/spmv_spmm.hpp:262,299)
 *   spmv(Ell_matrix&, Vector& x, Vector& y) (:209,235)          lz::spmv(A, x, y[, ctx])
 *   ftdt_block<T>(A, U0, Nsteps, T_end, lc) (methods/fdtd.hpp:33-56)
 *                                                               lz::ftdt_block<T>(A, U0, Nsteps, T_end, lc[, ctx])
 *   Assemble_T + expm_cusolver + solution (test_lanczos.cu:242-289)
 *                                                               lz::ritz_values / lz::block_solution
 *
 * Types: lz::Csr_matrix<T> stands where Ell_matrix<T> stood (CSR on the device;
 * lz::Csr_matrix<double>::from_ell converts the reference's ELL-4 arrays),
 * lz::Dense_matrix<T> where Dense_matrix<T> stood (device n x b block, ROW-major
 * by default -- one gathered row is one 128-B line at b = 16 fp64 -- or
 * column-major with a leading dimension, the reference's layout,
 * objects/dense_matrix.hpp:9), lz::Vector<T> where Vector<T> stood.  They own
 * their device memory (RAII, hipMalloc/hipFree) and are move-only (the
 * reference's deep-copying assignment, dense_matrix.hpp:147-165, is what the
 * Krylov rotation no longer needs).  lz::Context (one lz_handle, one stream)
 * replaces cublasHandle_t + cusolver_args; the overloads without a context use
 * a per-thread default context on device 0, like the reference's implicit one.
 *
 * Errors: a failing call throws std::runtime_error carrying lz_last_error()
 * (the reference aborts on CUDA errors and throws on cuBLAS/cuSOLVER ones,
 * utils/common.hpp:83-112).  Everything runs on the context's stream; the
 * method calls return with the work enqueued (results are read with
 * copy_to_host, which synchronises).
 */
#ifndef LZ_METHODS_HPP
#define LZ_METHODS_HPP

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "lz_hip.h"
#include "lz_host.h"

namespace lz {

inline void check(int rc, const char *what)
{
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + lz_last_error());
}
inline void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
constexpr lz_dtype dtype_of()
{
    static_assert(std::is_same<T, double>::value || std::is_same<T, float>::value, "fp64 or fp32");
    return std::is_same<T, double>::value ? LZ_F64 : LZ_F32;
}

// ------------------------------------------------------------------ context
class Context {
public:
    explicit Context(int device = 0, hipStream_t stream = nullptr)
    {
        check(lz_init(device, &h_), "lz_init");
        if (stream) check(lz_set_stream(h_, stream), "lz_set_stream");
        stream_ = stream;
    }
    ~Context() { lz_finalize(h_); }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    lz_handle *get() const { return h_; }
    hipStream_t stream() const { return stream_; }
    void synchronize() const { hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }
    // nonzero if a persistent kernel abandoned a bounded spin (results invalid)
    int device_error() const
    {
        int c = 0;
        check(lz_device_error(h_, &c), "lz_device_error");
        return c;
    }

private:
    lz_handle *h_ = nullptr;
    hipStream_t stream_ = nullptr;
};

inline Context &default_context()
{
    thread_local std::unique_ptr<Context> ctx;
    if (!ctx) ctx.reset(new Context(0));
    return *ctx;
}

// ------------------------------------------------------------- device buffer
template <typename T>
class DeviceArray {
public:
    DeviceArray() = default;
    explicit DeviceArray(size_t n) : n_(n)
    {
        if (n) hip_check(hipMalloc(&p_, sizeof(T) * n), "hipMalloc");
    }
    // The containers' transfers are blocking, as the reference's are: the copy
    // or fill has landed when the call returns, and a read-back sees every
    // stream's earlier work (a context may run on a non-blocking stream, which
    // the null-stream hipMemcpy / hipMemset would not order against).
    DeviceArray(const T *host, size_t n) : DeviceArray(n)
    {
        if (n) {
            hip_check(hipMemcpy(p_, host, sizeof(T) * n, hipMemcpyHostToDevice), "hipMemcpy H2D");
            hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        }
    }
    ~DeviceArray() { (void)hipFree(p_); }
    DeviceArray(DeviceArray &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    DeviceArray &operator=(DeviceArray &&o) noexcept
    {
        std::swap(p_, o.p_);
        std::swap(n_, o.n_);
        return *this;
    }
    DeviceArray(const DeviceArray &) = delete;
    DeviceArray &operator=(const DeviceArray &) = delete;
    T *data() { return p_; }
    const T *data() const { return p_; }
    size_t size() const { return n_; }
    std::vector<T> copy_to_host() const
    {
        std::vector<T> h(n_);
        if (n_) {
            hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
            hip_check(hipMemcpy(h.data(), p_, sizeof(T) * n_, hipMemcpyDeviceToHost), "hipMemcpy D2H");
        }
        return h;
    }
    void fill_zero()
    {
        if (n_) {
            hip_check(hipMemset(p_, 0, sizeof(T) * n_), "hipMemset");
            hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        }
    }

private:
    T *p_ = nullptr;
    size_t n_ = 0;
};

// ------------------------------------------------------------------ containers
// Vector<T> (objects/vector.hpp:17-376): n values on the device.
template <typename T>
class Vector {
public:
    Vector() = default;
    explicit Vector(int64_t n) : a_((size_t)n) { a_.fill_zero(); }
    explicit Vector(const std::vector<T> &h) : a_(h.data(), h.size()) {}
    int64_t size() const { return (int64_t)a_.size(); }
    T *data() { return a_.data(); }
    const T *data() const { return a_.data(); }
    std::vector<T> copy_to_host() const { return a_.copy_to_host(); }

private:
    DeviceArray<T> a_;
};

// Dense_matrix<T> (objects/dense_matrix.hpp:10-506): n_rows x n_cols block.
// Row-major (ld = n_cols) by default; LZ_COL_MAJOR with ld >= n_rows is the
// reference's storage (its ld = rows padded to a multiple of 768,
// test_lanczos.cu:174-187).
template <typename T>
class Dense_matrix {
public:
    Dense_matrix() = default;
    Dense_matrix(int64_t rows, int cols, lz_layout layout = LZ_ROW_MAJOR, int64_t ld = 0)
        : rows_(rows), cols_(cols), layout_(layout),
          ld_(ld ? ld : (layout == LZ_ROW_MAJOR ? cols : rows)),
          a_((size_t)(layout == LZ_ROW_MAJOR ? rows * ld_ : (int64_t)cols * ld_))
    {
        a_.fill_zero();
    }
    // from a host array in the same layout
    Dense_matrix(int64_t rows, int cols, const std::vector<T> &h, lz_layout layout = LZ_ROW_MAJOR, int64_t ld = 0)
        : rows_(rows), cols_(cols), layout_(layout), ld_(ld ? ld : (layout == LZ_ROW_MAJOR ? cols : rows)),
          a_(h.data(), h.size())
    {
    }
    int64_t n_rows() const { return rows_; }
    int n_cols() const { return cols_; }
    int64_t ld() const { return ld_; }
    lz_layout layout() const { return layout_; }
    T *data() { return a_.data(); }
    const T *data() const { return a_.data(); }
    std::vector<T> copy_to_host() const { return a_.copy_to_host(); }

private:
    int64_t rows_ = 0;
    int cols_ = 0;
    lz_layout layout_ = LZ_ROW_MAJOR;
    int64_t ld_ = 0;
    DeviceArray<T> a_;
};

// Csr_matrix<T>: the sparse operator (where the reference has Ell_matrix<T>,
// objects/ell_matrix.hpp:10-544): int64 row_ptr, int32 col, T val on the device.
template <typename T>
class Csr_matrix {
public:
    Csr_matrix() = default;
    Csr_matrix(int64_t n_rows, int64_t n_cols, const std::vector<int64_t> &rp, const std::vector<int32_t> &col,
               const std::vector<T> &val)
        : n_(n_rows), nc_(n_cols), nnz_((int64_t)col.size()), rp_(rp.data(), rp.size()),
          col_(col.data(), col.size()), val_(val.data(), val.size())
    {
        if ((int64_t)rp.size() != n_rows + 1 || val.size() != col.size())
            throw std::runtime_error("Csr_matrix: inconsistent sizes");
    }
    // the reference's ELL storage (width slots per row, column-major slots:
    // data[s * n + r], as Ell_matrix after its build, ell_matrix.hpp:46);
    // explicit zeros dropped unless keep_zeros
    static Csr_matrix from_ell(int64_t n, int64_t width, const std::vector<double> &data,
                               const std::vector<uint32_t> &idx, bool keep_zeros = false)
    {
        std::vector<int64_t> rp(n + 1);
        const int64_t nnz = lzh_ell_to_csr_count(n, width, data.data(), idx.data(), keep_zeros, rp.data());
        if (nnz < 0) throw std::runtime_error("lzh_ell_to_csr_count failed");
        std::vector<int32_t> col(nnz);
        std::vector<double> v(nnz);
        check(lzh_ell_to_csr_fill(n, width, data.data(), idx.data(), keep_zeros, rp.data(), col.data(), v.data()),
              "lzh_ell_to_csr_fill");
        std::vector<T> vt(v.begin(), v.end());
        return Csr_matrix(n, n, rp, col, vt);
    }
    int64_t n_rows() const { return n_; }
    int64_t n_cols() const { return nc_; }
    int64_t nnz() const { return nnz_; }
    const int64_t *row_ptr() const { return rp_.data(); }
    const int32_t *col() const { return col_.data(); }
    const T *val() const { return val_.data(); }

private:
    int64_t n_ = 0, nc_ = 0, nnz_ = 0;
    DeviceArray<int64_t> rp_;
    DeviceArray<int32_t> col_;
    DeviceArray<T> val_;
};

// --------------------------------------------------------------- operators
// Y = A X (kernels/spmv_spmm.hpp:262-333), any layout X / Y share
template <typename T>
void spmm(const Csr_matrix<T> &A, const Dense_matrix<T> &X, Dense_matrix<T> &Y, Context &ctx = default_context())
{
    if (X.layout() != Y.layout() || X.n_cols() != Y.n_cols() || X.n_rows() != A.n_cols() ||
        Y.n_rows() != A.n_rows())
        throw std::runtime_error("spmm: shape or layout mismatch");
    check(lz_csr_spmm(ctx.get(), A.n_rows(), A.n_cols(), A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(),
                      X.n_cols(), X.data(), X.ld(), X.layout(), Y.data(), Y.ld()),
          "spmm");
}

// y = A x (spmv_spmm.hpp:209-260)
template <typename T>
void spmv(const Csr_matrix<T> &A, const Vector<T> &x, Vector<T> &y, Context &ctx = default_context())
{
    check(lz_csr_spmv(ctx.get(), A.n_rows(), A.n_cols(), A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(),
                      x.data(), y.data()),
          "spmv");
}

// ------------------------------------------------------------------ methods
// The iteration's start block as n x b row-major (ld = b): B itself when it is
// stored that way, else its first n rows transposed once on the device into
// `tmp` -- the reference's B is column-major with its rows padded to a multiple
// of 768 (objects/dense_matrix.hpp:9, test_lanczos.cu:174-187).
template <typename T>
const T *row_major_block(const Dense_matrix<T> &B, int64_t n, DeviceArray<T> &tmp, Context &ctx, const char *who)
{
    const int b = B.n_cols();
    if (B.n_rows() < n) throw std::runtime_error(std::string(who) + ": B has fewer rows than A");
    if (B.layout() == LZ_ROW_MAJOR) {
        if (B.ld() != b) throw std::runtime_error(std::string(who) + ": a row-major B needs ld = b");
        return B.data();
    }
    tmp = DeviceArray<T>((size_t)n * b);
    check(lz_to_row_major(ctx.get(), n, b, dtype_of<T>(), B.data(), B.ld(), tmp.data()), who);
    return tmp.data();
}

// workspace blocks may come in either layout (the reference allocates Q0, Q1, W
// like B): their input content is ignored; on return they hold what the
// reference leaves in them (Q0 = Q1 = Q_{m-1}, W = the last residual), in
// their own layout
template <typename T>
void check_workspace(const Dense_matrix<T> &X, int64_t n, int b, const char *who)
{
    if (X.n_cols() != b || X.n_rows() < n || X.ld() < (X.layout() == LZ_ROW_MAJOR ? (int64_t)b : X.n_rows()))
        throw std::runtime_error(std::string(who) + ": workspace block is not n x b");
}

// the iteration writes row-major n x b blocks (ld = b): a caller block in that
// exact layout is used in place, any other gets a row-major temporary
template <typename T>
bool row_major_dense(const Dense_matrix<T> &X)
{
    return X.layout() == LZ_ROW_MAJOR && X.ld() == X.n_cols();
}

// the final n x b row-major block `src` into the caller's block X
template <typename T>
void store_block(Dense_matrix<T> &X, const T *src, int64_t n, int b, Context &ctx, const char *who)
{
    if (X.layout() == LZ_COL_MAJOR) {
        check(lz_to_col_major(ctx.get(), n, b, dtype_of<T>(), src, X.data(), X.ld()), who);
        return;
    }
    hip_check(hipMemcpy2DAsync(X.data(), sizeof(T) * X.ld(), src, sizeof(T) * b, sizeof(T) * b, n,
                               hipMemcpyDeviceToDevice, ctx.stream()),
              who);
}

// run `call(Q0, Q1, W)` on row-major n x b blocks and leave its final blocks in
// the caller's (m == 1: the reference does not write Q1)
template <typename T, typename F>
void with_final_blocks(Dense_matrix<T> &Q0, Dense_matrix<T> &Q1, Dense_matrix<T> &W, int64_t n, int b, unsigned m,
                       Context &ctx, const char *who, F call)
{
    for (Dense_matrix<T> *X : {&Q0, &Q1, &W}) check_workspace(*X, n, b, who);
    if (row_major_dense(Q0) && row_major_dense(Q1) && row_major_dense(W)) {
        call(Q0.data(), Q1.data(), W.data());
        return;
    }
    DeviceArray<T> t0((size_t)n * b), t1((size_t)n * b), t2((size_t)n * b);
    call(t0.data(), t1.data(), t2.data());
    store_block(Q0, t0.data(), n, b, ctx, who);
    if (m >= 2) store_block(Q1, t1.data(), n, b, ctx, who);
    store_block(W, t2.data(), n, b, ctx, who);
    ctx.synchronize();  // t0..t2 are released on return
}

// block_lanczos_blas (methods/block_lanczos.hpp:88-167).  alpha: array of m
// b x b matrices, beta: array of m + 1 (beta[m] = the last inverse square root,
// as the reference's).  B: the start block, row-major (ld = b) or the
// reference's column-major layout with a padded leading dimension (rows past
// A.n_rows() are padding, as in the reference).  Q0, Q1, W: workspace, either
// layout.  eigen_val, n_blocks, n_loads are accepted for call-site
// compatibility: the eigenvalues of each Gram are not needed by the caller, and
// launch shapes are chosen per operator.
template <typename T>
void block_lanczos_blas(const Csr_matrix<T> &A, const Dense_matrix<T> &B, unsigned m, unsigned lc, Vector<T> &q,
                        Dense_matrix<T> *alpha, Dense_matrix<T> *beta, Dense_matrix<T> &Q0, Dense_matrix<T> &Q1,
                        Dense_matrix<T> &W, Context &ctx, Vector<T> * /*eigen_val*/ = nullptr,
                        unsigned /*n_blocks*/ = 0, unsigned /*n_loads*/ = 0)
{
    const int b = B.n_cols();
    const int64_t n = A.n_rows(), bb = (int64_t)b * b;
    if (q.size() < (int64_t)m * b) throw std::runtime_error("block_lanczos_blas: q needs m*b entries");
    DeviceArray<T> Bt;
    const T *Bp = row_major_block(B, n, Bt, ctx, "block_lanczos_blas");
    DeviceArray<T> al((size_t)m * bb), be((size_t)(m + 1) * bb);
    with_final_blocks(Q0, Q1, W, n, b, m, ctx, "block_lanczos_blas", [&](T *q0, T *q1, T *w) {
        check(lz_block_lanczos(ctx.get(), n, A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(), b, (int)m, lc,
                               Bp, q.data(), al.data(), be.data(), q0, q1, w),
              "block_lanczos_blas");
    });
    // scatter into the caller's per-step matrices (device to device, on the stream)
    for (unsigned j = 0; j < m; ++j)
        hip_check(hipMemcpyAsync(alpha[j].data(), al.data() + j * bb, sizeof(T) * bb, hipMemcpyDeviceToDevice,
                                 ctx.stream()), "alpha copy");
    for (unsigned j = 0; j <= m; ++j)
        hip_check(hipMemcpyAsync(beta[j].data(), be.data() + j * bb, sizeof(T) * bb, hipMemcpyDeviceToDevice,
                                 ctx.stream()), "beta copy");
    ctx.synchronize();  // al / be are released on return
}

// The same iteration with one kernel (pair) per reference call, in the
// reference's op order (methods/block_lanczos.hpp:104-166): a second GPU path
// for parity and A/B measurement.
template <typename T>
void block_lanczos_blas_reference_order(const Csr_matrix<T> &A, const Dense_matrix<T> &B, unsigned m, unsigned lc,
                                        Vector<T> &q, Dense_matrix<T> *alpha, Dense_matrix<T> *beta,
                                        Dense_matrix<T> &Q0, Dense_matrix<T> &Q1, Dense_matrix<T> &W, Context &ctx)
{
    const int b = B.n_cols();
    const int64_t n = A.n_rows(), bb = (int64_t)b * b;
    DeviceArray<T> Bt;
    const T *Bp = row_major_block(B, n, Bt, ctx, "block_lanczos_blas_reference_order");
    DeviceArray<T> al((size_t)m * bb), be((size_t)(m + 1) * bb);
    with_final_blocks(Q0, Q1, W, n, b, m, ctx, "block_lanczos_blas_reference_order", [&](T *q0, T *q1, T *w) {
        check(lz_block_lanczos_unfused(ctx.get(), n, A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(), b,
                                       (int)m, lc, Bp, q.data(), al.data(), be.data(), q0, q1, w),
              "block_lanczos_blas_reference_order");
    });
    for (unsigned j = 0; j < m; ++j)
        hip_check(hipMemcpyAsync(alpha[j].data(), al.data() + j * bb, sizeof(T) * bb, hipMemcpyDeviceToDevice,
                                 ctx.stream()), "alpha copy");
    for (unsigned j = 0; j <= m; ++j)
        hip_check(hipMemcpyAsync(beta[j].data(), be.data() + j * bb, sizeof(T) * bb, hipMemcpyDeviceToDevice,
                                 ctx.stream()), "beta copy");
    ctx.synchronize();
}

// vector_lanczos (methods/vector_lanczos.hpp:8-67): alpha, beta are HOST arrays
// of m, as the reference's (beta[0] = ||b||).
template <typename T>
void vector_lanczos(const Csr_matrix<T> &A, const Vector<T> &b, unsigned m, unsigned lc, Vector<T> &q, T *alpha,
                    T *beta, Vector<T> &q0, Vector<T> &q1, Vector<T> &w, Context &ctx = default_context())
{
    DeviceArray<T> al(m), be(m);
    check(lz_vector_lanczos(ctx.get(), b.size(), A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(), (int)m, lc,
                            b.data(), q.data(), al.data(), be.data(), q0.data(), q1.data(), w.data()),
          "vector_lanczos");
    ctx.synchronize();
    const std::vector<T> ha = al.copy_to_host(), hb = be.copy_to_host();
    for (unsigned j = 0; j < m; ++j) {
        alpha[j] = ha[j];
        beta[j] = hb[j];
    }
}

// ftdt_block (methods/fdtd.hpp:33-56): Nsteps forward-Euler steps of U' = A U
// from U0 (n x b, row-major or the reference's padded column-major layout),
// returns row lc of the final state.
template <typename T>
std::vector<T> ftdt_block(const Csr_matrix<T> &A, const Dense_matrix<T> &U0, unsigned Nsteps, double T_end, unsigned lc,
                          Context &ctx = default_context())
{
    const int b = U0.n_cols();
    const int64_t n = A.n_rows();
    DeviceArray<T> Ut;
    const T *U0p = row_major_block(U0, n, Ut, ctx, "ftdt_block");
    Dense_matrix<T> U(n, b), D(n, b);
    DeviceArray<T> out(b);
    check(lz_fdtd_block(ctx.get(), n, A.nnz(), A.row_ptr(), A.col(), A.val(), dtype_of<T>(), b, U0p, Nsteps, T_end,
                        lc, U.data(), D.data(), out.data()),
          "ftdt_block");
    ctx.synchronize();
    return out.copy_to_host();
}

// -------------------------------------------------------- post-processing
// Ritz values = ascending eigenvalues of Assemble_T(m, alpha, beta)
// (objects/tridiagonal_matrix.hpp:90-156, utils/lib_utils.hpp:547-577); host
// arrays alpha[m*b*b], beta[(m+1)*b*b]
inline std::vector<double> ritz_values(int m, int b, const std::vector<double> &alpha, const std::vector<double> &beta)
{
    std::vector<double> r((size_t)m * b);
    check(lzh_ritz_values(m, b, alpha.data(), beta.data(), r.data()), "ritz_values");
    return r;
}

// solution = (expm(T_end T)[:, :b] beta_0)^T q  (test_lanczos.cu:272-289)
inline std::vector<double> block_solution(int m, int b, double T_end, const std::vector<double> &alpha,
                                          const std::vector<double> &beta, const std::vector<double> &q)
{
    std::vector<double> s(b);
    check(lzh_block_solution(m, b, T_end, alpha.data(), beta.data(), q.data(), s.data()), "block_solution");
    return s;
}

}  // namespace lz

#endif
