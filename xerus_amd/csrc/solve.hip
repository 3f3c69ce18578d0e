// Dense linear solves (blasWrapper::solve / solve_least_squares, blasLapackWrapper.cpp:540-721) and the
// blocked Cholesky they use for symmetric positive definite systems of any size.
//
// Dispatch as the reference's (mldivide order, :547-640): m != n -> least squares; not symmetric ->
// general solve; symmetric with a positive diagonal -> Cholesky, and if that fails the general path.
// The reference's LU (dgesv), LDL^T (dsysv) and dgelsd all return the solution of a nonsingular system
// (dgelsd: the minimum-norm least-squares solution, singular values <= EPSILON sigma_max dropped); here
// the general and least-squares paths are one SVD solve x = V S^+ U^T b with that same cut (min(m, n)
// <= 512; above: a shifted-CholeskyQR3 QR / LQ solve, full rank only), and the Cholesky path is a right-looking blocked factorisation: 256-column diagonal blocks by
// the register-resident potrf + explicit triangular inverse, panels and trailing updates as MFMA GEMMs
// (n unbounded). Triangular solves use the diagonal-block inverses, so both sweeps are GEMMs too.
#include <cmath>
#include <cstdio>
#include <vector>

#include "smallla.hpp"

namespace xrs {
namespace {

constexpr double kEps = 2.220446049250313e-16;
constexpr int kCholBlock = 256;

// dst (rows x cols, ld ldd) = alpha * src (ld lds)
__global__ void __launch_bounds__(256) k_copy2d(double* __restrict__ dst, size_t ldd, const double* __restrict__ src, size_t lds,
                                                size_t rows, size_t cols, double alpha) {
    const size_t total = rows * cols;
    for (size_t e = size_t(blockIdx.x) * 256 + threadIdx.x; e < total; e += size_t(gridDim.x) * 256) {
        const size_t r = e / cols, c = e - r * cols;
        dst[r * ldd + c] = alpha * src[r * lds + c];
    }
}

void copy2d(xrs_handle_t h, double* dst, size_t ldd, const double* src, size_t lds, size_t rows, size_t cols, double alpha = 1.0) {
    if (!rows || !cols) return;
    const size_t blocks = std::min<size_t>((rows * cols + 255) / 256, 4096);
    hipLaunchKernelGGL(k_copy2d, dim3(unsigned(blocks)), dim3(256), 0, h->stream, dst, ldd, src, lds, rows, cols, alpha);
    check_launch("k_copy2d");
}

// per-block partial maxima of A (signed values, as the reference's is_symmetric, :501-505)
__global__ void __launch_bounds__(256) k_max_partial(const double* __restrict__ A, size_t total, double* __restrict__ part) {
    double m = 0.0;
    for (size_t e = size_t(blockIdx.x) * 256 + threadIdx.x; e < total; e += size_t(gridDim.x) * 256) m = fmax(m, A[e]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// flags[0] = 1 if some |A_ij - A_ji| >= 4 max eps (not symmetric, :507-513); flags[1] = 1 if the
// diagonal is not positive definite-looking (A_00 > 0 and A_ii >= eps, :519-528)
__global__ void __launch_bounds__(256) k_sym_flags(const double* __restrict__ A, size_t n, const double* __restrict__ part, int nparts,
                                                   int* __restrict__ flags) {
    double mx = 0.0;
    for (int i = 0; i < nparts; ++i) mx = fmax(mx, part[i]);
    const double thr = 4.0 * mx * kEps;
    bool asym = false, baddiag = false;
    for (size_t e = size_t(blockIdx.x) * 256 + threadIdx.x; e < n * n; e += size_t(gridDim.x) * 256) {
        const size_t i = e / n, j = e - i * n;
        if (j > i && fabs(A[i * n + j] - A[j * n + i]) >= thr) asym = true;
        if (i == j && (i == 0 ? !(A[0] > 0.0) : A[e] < kEps)) baddiag = true;
    }
    if (asym) __hip_atomic_fetch_or(&flags[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (baddiag) __hip_atomic_fetch_or(&flags[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sinv[i] = 1 / S[i] for S[i] > rcond * S[0], else 0 (dgelsd's rank cut)
__global__ void k_inv_cut(const double* __restrict__ S, int k, double rcond, double* __restrict__ sinv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) sinv[i] = (S[i] > rcond * S[0]) ? 1.0 / S[i] : 0.0;
}

}  // namespace

// A = L L^T for symmetric positive definite A (n x n); L lower (n x n, upper part zero), Z the explicit
// inverses of the diagonal blocks (kCholBlock x kCholBlock each, packed). Returns false if a diagonal
// block is not positive definite (synchronises once).
bool chol_blocked(xrs_handle_t h, const double* A, size_t n, double* L, std::vector<DevBuf>& Z) {
    const size_t nblk = (n + kCholBlock - 1) / kCholBlock;
    DevBuf W(h, n * n * 8), st(h, nblk * 4), D(h, size_t(kCholBlock) * kCholBlock * 8), Dinv(h, dinv_elems(kCholBlock) * 8);
    DevBuf P(h, n * kCholBlock * 8), T(h, n * n * 8);
    XRS_HIP(hipMemcpyAsync(W.d(), A, n * n * 8, hipMemcpyDeviceToDevice, h->stream));
    XRS_HIP(hipMemsetAsync(L, 0, n * n * 8, h->stream));
    Z.clear();
    for (size_t jb = 0; jb < nblk; ++jb) {
        const size_t j0 = jb * kCholBlock, b = std::min<size_t>(kCholBlock, n - j0), rest = n - j0 - b;
        copy2d(h, D.d(), b, W.d() + j0 * n + j0, n, b, b);
        potrf(h, D.d(), int(b), 0.0, Dinv.d(), st.as<int>() + jb);
        Z.emplace_back(h, b * b * 8);
        TrinvBatch tb{};
        tb.L[0] = D.d();
        tb.Dinv[0] = Dinv.d();
        tb.X[0] = Z.back().d();
        tb.n[0] = int(b);
        trinv_batched(h, tb, 1);
        copy2d(h, L + j0 * n + j0, n, D.d(), b, b, b);
        if (!rest) break;
        // panel L_ij = W_ij Z_jj^T, trailing W -= L_ij L_ij^T
        gemm(h, P.d(), rest, b, 1.0, W.d() + (j0 + b) * n + j0, n, false, b, Z.back().d(), b, true);
        copy2d(h, L + (j0 + b) * n + j0, n, P.d(), b, rest, b);
        gemm_sym(h, T.d(), rest, 1.0, P.d(), b, false, b, P.d(), b, true);
        const size_t od[2] = {n, n}, id[2] = {rest, rest}, off[2] = {j0 + b, j0 + b};
        offset_add(h, W.d(), od, T.d(), id, 2, off, -1.0);
    }
    std::vector<int> s(nblk);
    read_status(h, st.as<int>(), int(nblk), s.data());
    for (int v : s)
        if (v != 0) return false;
    return true;
}

namespace {
// W[i][i] += rel * trace(W) (one workgroup; the shifted factorisations of the certificates)
__global__ void __launch_bounds__(256) k_shift_diag(double* __restrict__ W, size_t n, double rel) {
    __shared__ double red[4];
    double tr = 0.0;
    for (size_t i = threadIdx.x; i < n; i += 256) tr += W[i * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = tr;
    __syncthreads();
    const double s = rel * ((red[0] + red[1]) + (red[2] + red[3]));
    for (size_t i = threadIdx.x; i < n; i += 256) W[i * n + i] += s;
}
}  // namespace

int chol_full_blocks(size_t n) { return int((n + kCholBlock - 1) / kCholBlock); }

// Cholesky of A + shift_rel tr(A) I of any order, enqueued only: status[b] = potrf status of diagonal
// block b (chol_full_blocks(n) slots, all zero on success); L (n x n lower, upper zero) and the full
// inverse Z = L^{-1} (block forward substitution: Z_ii = L_ii^{-1}, Z_ij = -Z_ii L_i,<i Z_<i,j) when
// the pointers are given. The TT drivers use it for ranks above the batched kernels' 512.
void chol_full(xrs_handle_t h, const double* A, size_t n, double shift_rel, double* L, double* Z, int* status) {
    const size_t nblk = size_t(chol_full_blocks(n));
    DevBuf W(h, n * n * 8), Lown(h, L ? 8 : n * n * 8), D(h, size_t(kCholBlock) * kCholBlock * 8),
        Dinv(h, dinv_elems(kCholBlock) * 8), P(h, n * kCholBlock * 8), T(h, n * n * 8);
    double* Lm = L ? L : Lown.d();
    XRS_HIP(hipMemcpyAsync(W.d(), A, n * n * 8, hipMemcpyDeviceToDevice, h->stream));
    if (shift_rel != 0.0) {
        hipLaunchKernelGGL(k_shift_diag, dim3(1), dim3(256), 0, h->stream, W.d(), n, shift_rel);
        check_launch("k_shift_diag");
    }
    XRS_HIP(hipMemsetAsync(Lm, 0, n * n * 8, h->stream));
    if (Z) XRS_HIP(hipMemsetAsync(Z, 0, n * n * 8, h->stream));
    DevBuf Zb(h, size_t(kCholBlock) * kCholBlock * 8);
    for (size_t jb = 0; jb < nblk; ++jb) {
        const size_t j0 = jb * kCholBlock, b = std::min<size_t>(kCholBlock, n - j0), rest = n - j0 - b;
        copy2d(h, D.d(), b, W.d() + j0 * n + j0, n, b, b);
        potrf(h, D.d(), int(b), 0.0, Dinv.d(), status + jb);
        TrinvBatch tb{};
        tb.L[0] = D.d();
        tb.Dinv[0] = Dinv.d();
        tb.X[0] = Zb.d();
        tb.n[0] = int(b);
        trinv_batched(h, tb, 1);
        copy2d(h, Lm + j0 * n + j0, n, D.d(), b, b, b);
        if (Z) {
            copy2d(h, Z + j0 * n + j0, n, Zb.d(), b, b, b);
            if (j0) {   // Z[j, :j0] = -Z_jj (L[j, :j0] Z[:j0, :j0])
                gemm(h, T.d(), b, j0, 1.0, Lm + j0 * n, n, false, j0, Z, n, false);
                gemm(h, P.d(), b, j0, -1.0, Zb.d(), b, false, b, T.d(), j0, false);
                copy2d(h, Z + j0 * n, n, P.d(), j0, b, j0);
            }
        }
        if (!rest) break;
        gemm(h, P.d(), rest, b, 1.0, W.d() + (j0 + b) * n + j0, n, false, b, Zb.d(), b, true);   // L_ij = W_ij Z_jj^T
        copy2d(h, Lm + (j0 + b) * n + j0, n, P.d(), b, rest, b);
        gemm_sym(h, T.d(), rest, 1.0, P.d(), b, false, b, P.d(), b, true);
        const size_t od[2] = {n, n}, id[2] = {rest, rest}, off[2] = {j0 + b, j0 + b};
        offset_add(h, W.d(), od, T.d(), id, 2, off, -1.0);
    }
}

// X (n x p) = (L L^T)^{-1} B with the factors of chol_blocked
void chol_solve(xrs_handle_t h, const double* L, const std::vector<DevBuf>& Z, size_t n, const double* B, size_t p, double* X) {
    const size_t nblk = Z.size();
    DevBuf Y(h, n * p * 8), R(h, size_t(kCholBlock) * p * 8), T(h, size_t(kCholBlock) * p * 8);
    for (size_t jb = 0; jb < nblk; ++jb) {   // L Y = B
        const size_t j0 = jb * kCholBlock, b = std::min<size_t>(kCholBlock, n - j0);
        XRS_HIP(hipMemcpyAsync(R.d(), B + j0 * p, b * p * 8, hipMemcpyDeviceToDevice, h->stream));
        if (j0) {
            gemm(h, T.d(), b, p, 1.0, L + j0 * n, n, false, j0, Y.d(), p, false);
            axpy(h, R.d(), -1.0, T.d(), b * p);
        }
        gemm(h, Y.d() + j0 * p, b, p, 1.0, Z[jb].d(), b, false, b, R.d(), p, false);
    }
    for (size_t jb = nblk; jb-- > 0;) {   // L^T X = Y
        const size_t j0 = jb * kCholBlock, b = std::min<size_t>(kCholBlock, n - j0), rest = n - j0 - b;
        XRS_HIP(hipMemcpyAsync(R.d(), Y.d() + j0 * p, b * p * 8, hipMemcpyDeviceToDevice, h->stream));
        if (rest) {
            gemm(h, T.d(), b, p, 1.0, L + (j0 + b) * n + j0, n, true, rest, X + (j0 + b) * p, p, false);
            axpy(h, R.d(), -1.0, T.d(), b * p);
        }
        gemm(h, X + j0 * p, b, p, 1.0, Z[jb].d(), b, true, b, R.d(), p, false);
    }
}

// min(m, n) > 512 (no single-workgroup SVD there): shifted CholeskyQR3 (Fukaya et al. 2020) of A with the
// explicit inverses of its three Cholesky factors, so the triangular solves are GEMMs:
//   m >= n: A = Q R, R = L3^T L2^T L1^T       -> X = R^{-1} Q^T B = Z1^T Z2^T Z3^T (Q^T B)
//   m <  n: A = L Q, L = L1 L2 L3             -> X = Q^T L^{-1} B = Q^T Z3 Z2 Z1 B (the minimum-norm solution)
// Same solution as the reference's dgesv / dgelsd for a matrix of full rank min(m, n) with kappa < 1/u; a
// numerically rank-deficient system of that size is rejected (XRS_ENUMERIC) instead of getting dgelsd's
// truncated minimum-norm solution.
static void qr_solve_big(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p) {
    const bool wide = m < n;
    const size_t N = wide ? m : n, M = wide ? n : m;
    const int nb = chol_full_blocks(N);
    DevBuf G(h, N * N * 8), Z1(h, N * N * 8), Z2(h, N * N * 8), Z3(h, N * N * 8), Q1(h, m * n * 8), Q2(h, m * n * 8),
        st(h, size_t(3 * nb) * 4 + 64), Y(h, std::max(M, N) * p * 8), Y2(h, std::max(M, N) * p * 8);
    XRS_HIP(hipMemsetAsync(st.d(), 0, size_t(3 * nb) * 4, h->stream));
    auto gram = [&](const double* Xm) {
        if (wide) gemm_sym(h, G.d(), N, 1.0, Xm, n, false, M, Xm, n, true);   // X X^T
        else gemm_sym(h, G.d(), N, 1.0, Xm, n, true, M, Xm, n, false);        // X^T X
    };
    auto apply = [&](const double* Z, const double* Xm, double* out) {       // tall: X Z^T, wide: Z X
        if (wide) gemm(h, out, N, n, 1.0, Z, N, false, N, Xm, n, false);
        else gemm(h, out, m, N, 1.0, Xm, n, false, N, Z, N, true);
    };
    const double s_rel = 11.0 * (double(M) * N + double(N) * (N + 1)) * 1.1102230246251565e-16;
    gram(A);
    chol_full(h, G.d(), N, s_rel, nullptr, Z1.d(), st.as<int>());
    apply(Z1.d(), A, Q1.d());
    gram(Q1.d());
    chol_full(h, G.d(), N, 0.0, nullptr, Z2.d(), st.as<int>() + nb);
    apply(Z2.d(), Q1.d(), Q2.d());
    gram(Q2.d());
    chol_full(h, G.d(), N, 0.0, nullptr, Z3.d(), st.as<int>() + 2 * nb);
    double* Q = Q1.d();   // (Q1 no longer needed)
    apply(Z3.d(), Q2.d(), Q);
    std::vector<int> sts(size_t(3 * nb));
    read_status(h, st.as<int>(), 3 * nb, sts.data());
    for (int v : sts)
        if (v != 0) throw Error{XRS_ENUMERIC, "solve: a numerically rank-deficient system with min(m, n) > 512 is not supported"};
    if (!wide) {
        gemm(h, Y.d(), n, p, 1.0, Q, n, true, m, B, p, false);          // Q^T B
        gemm(h, Y2.d(), n, p, 1.0, Z3.d(), n, true, n, Y.d(), p, false);  // Z3^T
        gemm(h, Y.d(), n, p, 1.0, Z2.d(), n, true, n, Y2.d(), p, false);  // Z2^T
        gemm(h, X, n, p, 1.0, Z1.d(), n, true, n, Y.d(), p, false);       // Z1^T
    } else {
        gemm(h, Y.d(), m, p, 1.0, Z1.d(), m, false, m, B, p, false);
        gemm(h, Y2.d(), m, p, 1.0, Z2.d(), m, false, m, Y.d(), p, false);
        gemm(h, Y.d(), m, p, 1.0, Z3.d(), m, false, m, Y2.d(), p, false);
        gemm(h, X, n, p, 1.0, Q, n, true, m, Y.d(), p, false);            // Q^T (L^{-1} B)
    }
}

// Pseudo-inverse solution X = V S^+ U^T B (singular values below 8 eps sigma_0 cut, dgelsd's rule) plus two
// steps of iterative refinement x <- x - A^+ (A x - b) reusing the factors: the reference's dgesv / dsysv /
// dgelsd residuals on ill-conditioned systems (fullTensor_solve.cxx "solve vs least squares", kappa ~ 1e6:
// without refinement 4.2e-10 against LAPACK's 2.2e-12 for the indefinite system, 3.7e-10 against 4.4e-11 for
// least squares).
void svd_solve(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p) {
    const size_t k = std::min(m, n);
    if (k > size_t(kSmallMax)) {
        qr_solve_big(h, X, A, m, n, B, p);
        return;
    }
    DevBuf U(h, m * k * 8), S(h, k * 8), Vt(h, k * n * 8), Si(h, k * 8), T(h, k * p * 8), R(h, m * p * 8), D(h, n * p * 8);
    svd(h, A, m, n, U.d(), S.d(), Vt.d());
    hipLaunchKernelGGL(k_inv_cut, dim3(unsigned((k + 255) / 256)), dim3(256), 0, h->stream, S.d(), int(k), 8.0 * kEps, Si.d());
    check_launch("k_inv_cut");
    auto apply_pinv = [&](const double* rhs, double* out) {   // out = V S^+ U^T rhs
        gemm(h, T.d(), k, p, 1.0, U.d(), k, true, m, rhs, p, false);
        scale_rows(h, T.d(), Si.d(), k, p);
        gemm(h, out, n, p, 1.0, Vt.d(), n, true, k, T.d(), p, false);
    };
    apply_pinv(B, X);
    for (int it = 0; it < 2; ++it) {
        gemm(h, R.d(), m, p, 1.0, A, n, false, n, X, p, false);   // A x
        axpy(h, R.d(), -1.0, B, m * p);                            // A x - b
        apply_pinv(R.d(), D.d());
        axpy(h, X, -1.0, D.d(), n * p);
    }
}

void solve_dense(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p) {
    if (m != n) {
        svd_solve(h, X, A, m, n, B, p);
        return;
    }
    const size_t total = n * n;
    const int nparts = int(std::min<size_t>((total + 255) / 256, 1024));
    DevBuf part(h, size_t(nparts) * 8), flags(h, 64);
    XRS_HIP(hipMemsetAsync(flags.d(), 0, 64, h->stream));
    hipLaunchKernelGGL(k_max_partial, dim3(unsigned(nparts)), dim3(256), 0, h->stream, A, total, part.d());
    check_launch("k_max_partial");
    hipLaunchKernelGGL(k_sym_flags, dim3(unsigned(nparts)), dim3(256), 0, h->stream, A, n, part.d(), nparts, flags.as<int>());
    check_launch("k_sym_flags");
    int fl[2] = {0, 0};
    read_status(h, flags.as<int>(), 2, fl);
    if (!fl[0] && !fl[1]) {
        DevBuf L(h, n * n * 8);
        std::vector<DevBuf> Z;
        if (chol_blocked(h, A, n, L.d(), Z)) {
            chol_solve(h, L.d(), Z, n, B, p, X);
            return;
        }
    }
    svd_solve(h, X, A, m, n, B, p);
}

}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_solve(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p) {
    return guarded([&] {
        XRS_REQUIRE(h && X && A && B, "null argument");
        XRS_REQUIRE(m > 0 && n > 0 && p > 0, "solve: empty system");
        fence_readers(h);
        solve_dense(h, X, A, m, n, B, p);
    });
}

int xrs_solve_least_squares(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p) {
    return guarded([&] {
        XRS_REQUIRE(h && X && A && B, "null argument");
        XRS_REQUIRE(m > 0 && n > 0 && p > 0, "solve_least_squares: empty system");
        fence_readers(h);
        svd_solve(h, X, A, m, n, B, p);
    });
}

}  // extern "C"
