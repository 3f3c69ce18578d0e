// Factorisation drivers with the reference's semantics (blasLapackWrapper.cpp:201-498) on top of the
// GEMM / Cholesky / TRSM / QRCP / Jacobi kernels, plus their C-ABI entry points.
//
// Orthogonalisation (the hot path of TT rounding) is CholeskyQR2 on fp64 MFMA GEMMs:
//   G = A^T A, L1 = chol(G - tau I), Q1 = A L1^{-T}, G2 = Q1^T Q1, L2 = chol(G2), Q = Q1 L2^{-T}, R = (L1 L2)^T.
// The first Cholesky is shifted DOWN by tau = 4 (m + 2n) u ||A||_F^2: if it succeeds, the rounding errors
// of forming G and of the factorisation are covered and sigma_min(A) >= sqrt(tau/2) is *proven*
// (certified). A certified A has full numerical rank for the reference's QC rule (|R_kk| >= 16 u R_00) and
// no singular value below eps*sigma_0 for eps < sqrt(tau/2)/||A||_F, so rank decisions need no pivoting
// and no SVD. If certification fails, shifted CholeskyQR3 (Fukaya et al., SIAM J. Sci. Comput. 2020)
// still yields an orthonormal Q for any A with kappa < 1/u; exact rank semantics then come from the
// single-workgroup dgeqp3 emulation applied to the small n x n triangular factor, with the sign of
// dgeqp3's R_00 taken from A itself (it is -sign(A[0][p]) for the first max-norm column p).
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "smallla.hpp"

namespace xrs {

constexpr double kU = 1.1102230246251565e-16;       // unit roundoff 2^-53
constexpr double kDblEps = 2.220446049250313e-16;   // std::numeric_limits<double>::epsilon()

void transpose(xrs_handle_t h, double* out, const double* in, size_t rows, size_t cols) {
    const size_t dims[2] = {rows, cols};
    const size_t shuf[2] = {1, 0};
    permute(h, out, in, 2, dims, shuf);
}

int read_status(xrs_handle_t h, const int* status_dev, int count, int* host_out) {
    int* hs = static_cast<int*>(h->host_scratch);
    XRS_HIP(hipMemcpyAsync(hs, status_dev, size_t(count) * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    XRS_HIP(hipStreamSynchronize(h->stream));
    int any = 0;
    for (int i = 0; i < count; ++i) {
        host_out[i] = hs[i];
        any |= hs[i];
    }
    return any;
}

__global__ void __launch_bounds__(256) k_dev_identity(const double* __restrict__ G, int n, double* __restrict__ out) {
    __shared__ double red[4];
    double mx = 0.0;
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const double d = fabs(G[e] - ((e / n) == (e % n) ? 1.0 : 0.0));
        mx = (d > mx || d != d) ? d : mx;   // NaN propagates
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(mx, o, 64);
        mx = (t > mx || t != t) ? t : mx;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = red[0];
        for (int i = 1; i < 4; ++i) m = (red[i] > m || red[i] != red[i]) ? red[i] : m;
        out[0] = m;
    }
}

// First-order second CholeskyQR pass: G2 = I + E with ||E|| tiny -> L2 = I + Elow + O(E^2),
// Elow = strict_lower(E) + diag(E)/2. Writes L2 (lower) and Linv2 = I - Elow (lower) and max|E|.
__global__ void __launch_bounds__(256) k_first_order(const double* __restrict__ G2, int n, double* __restrict__ L2,
                                                     double* __restrict__ Li2, double* __restrict__ emax) {
    __shared__ double red[4];
    double mx = 0.0;
    for (int e = threadIdx.x + blockIdx.x * 256; e < n * n; e += 256 * gridDim.x) {
        const int i = e / n, j = e % n;
        const double eij = G2[e] - (i == j ? 1.0 : 0.0);
        const double d = fabs(eij);
        mx = (d > mx || d != d) ? d : mx;
        const double el = (i > j) ? eij : ((i == j) ? 0.5 * eij : 0.0);
        L2[e] = (i == j ? 1.0 : 0.0) + el;
        Li2[e] = (i == j ? 1.0 : 0.0) - el;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(mx, o, 64);
        mx = (t > mx || t != t) ? t : mx;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = red[0];
        for (int i = 1; i < 4; ++i) m = (red[i] > m || red[i] != red[i]) ? red[i] : m;
        emax[blockIdx.x] = m;
    }
}

static double max_abs_dev_identity(xrs_handle_t h, const double* G, size_t n) {
    double* out = static_cast<double*>(h->dev_scratch) + 32;
    hipLaunchKernelGGL(k_dev_identity, dim3(1), dim3(256), 0, h->stream, G, int(n), out);
    check_launch("k_dev_identity");
    double* hs = static_cast<double*>(h->host_scratch) + 32;
    XRS_HIP(hipMemcpyAsync(hs, out, 8, hipMemcpyDeviceToHost, h->stream));
    XRS_HIP(hipStreamSynchronize(h->stream));
    const double v = hs[0];
    return (v == v) ? v : 1e300;
}

// ------------------------------------------------------------------------------------------------
// The same CholeskyQR2 (certifying downward shift) / shifted CholeskyQR3 for Gram orders above the
// batched kernels' 512, on the blocked factorisation with explicit inverses (solve.hip chol_full): the
// triangular solves become GEMMs with L^{-1}. No Householder last resort at this size: a matrix that
// fails the verified shifted CholeskyQR3 (kappa >= 1/u) is rejected.
static OrthResult orthogonalize_big(xrs_handle_t h, const double* A, size_t m, size_t n, bool wide, double* Q, double* RL) {
    const size_t N = wide ? m : n, M = wide ? n : m;
    OrthResult res{false, 0.0, false};
    const int nb = chol_full_blocks(N);
    DevBuf G(h, N * N * 8), L1(h, N * N * 8), Z1(h, N * N * 8), L2(h, N * N * 8), Z2(h, N * N * 8), L3(h, N * N * 8),
        Z3(h, N * N * 8), T(h, N * N * 8), Q1(h, m * n * 8), Q2(h, m * n * 8), st(h, size_t(3 * nb) * 4 + 64);
    auto gram = [&](double* out, const double* X) {
        if (wide) gemm_sym(h, out, N, 1.0, X, n, false, M, X, n, true);   // X X^T
        else gemm_sym(h, out, N, 1.0, X, n, true, M, X, n, false);        // X^T X
    };
    auto apply = [&](const double* Z, const double* X, double* out) {   // tall: X Z^T, wide: Z X
        if (wide) gemm(h, out, N, n, 1.0, Z, N, false, N, X, n, false);
        else gemm(h, out, m, N, 1.0, X, n, false, N, Z, N, true);
    };
    auto all_zero = [&](int count) {
        std::vector<int> s(static_cast<size_t>(count));
        read_status(h, st.as<int>(), count, s.data());
        for (int v : s)
            if (v != 0) return false;
        return true;
    };
    const double tau_rel = 4.0 * double(M + 2 * N) * kU;
    gram(G.d(), A);
    chol_full(h, G.d(), N, -tau_rel, L1.d(), Z1.d(), st.as<int>());
    apply(Z1.d(), A, Q1.d());
    gram(G.d(), Q1.d());
    chol_full(h, G.d(), N, 0.0, L2.d(), Z2.d(), st.as<int>() + nb);
    apply(Z2.d(), Q1.d(), Q);
    if (wide) gemm(h, RL, N, N, 1.0, L1.d(), N, false, N, L2.d(), N, false);   // L = L1 L2
    else gemm(h, RL, N, N, 1.0, L2.d(), N, true, N, L1.d(), N, true);         // R = L2^T L1^T
    if (all_zero(2 * nb)) {
        res.certified = true;
        res.cert_ratio = std::sqrt(0.5 * tau_rel);
        return res;
    }
    res.robust = true;
    const double s_rel = 11.0 * (double(M) * N + double(N) * (N + 1)) * kU;
    gram(G.d(), A);
    chol_full(h, G.d(), N, s_rel, L1.d(), Z1.d(), st.as<int>());
    apply(Z1.d(), A, Q1.d());
    gram(G.d(), Q1.d());
    chol_full(h, G.d(), N, 0.0, L2.d(), Z2.d(), st.as<int>() + nb);
    apply(Z2.d(), Q1.d(), Q2.d());
    gram(G.d(), Q2.d());
    chol_full(h, G.d(), N, 0.0, L3.d(), Z3.d(), st.as<int>() + 2 * nb);
    apply(Z3.d(), Q2.d(), Q);
    if (wide) {   // L = L1 L2 L3
        gemm(h, T.d(), N, N, 1.0, L1.d(), N, false, N, L2.d(), N, false);
        gemm(h, RL, N, N, 1.0, T.d(), N, false, N, L3.d(), N, false);
    } else {      // R = L3^T L2^T L1^T
        gemm(h, T.d(), N, N, 1.0, L3.d(), N, true, N, L2.d(), N, true);
        gemm(h, RL, N, N, 1.0, T.d(), N, false, N, L1.d(), N, true);
    }
    if (all_zero(3 * nb)) {
        gram(T.d(), Q);
        if (max_abs_dev_identity(h, T.d(), N) <= 64.0 * double(N) * kU) return res;
    }
    // (qc / cq / qr / rq catch this and run the exact Householder emulation on the matrix itself)
    throw Error{XRS_ENUMERIC, "orthogonalize: a numerically rank-deficient matrix above 512 (shifted CholeskyQR3 failed)"};
}

// ------------------------------------------------------------------------------------------------
// CholeskyQR2 / shifted CholeskyQR3. Tall: A (m x n) = Q R. Wide: A (m x n) = L Q.
OrthResult orthogonalize(xrs_handle_t h, const double* A, size_t m, size_t n, bool wide, double* Q, double* RL) {
    const size_t N = wide ? m : n;   // Gram size
    const size_t M = wide ? n : m;   // long dimension
    XRS_REQUIRE(N >= 1 && M >= N, "orthogonalize: need a tall (or, wide=true, a wide) matrix");
    OrthResult res{false, 0.0, false};
    if (N > size_t(kSmallMax)) return orthogonalize_big(h, A, m, n, wide, Q, RL);
    const int Ni = int(N), nvec = int(M);
    DevBuf G(h, N * N * 8), Dv(h, (N + 32) * 32 * 8), L1(h, N * N * 8), Q1(h, m * n * 8), st(h, 64);
    auto gram = [&](double* out, const double* X) {
        if (wide) gemm(h, out, N, N, 1.0, X, n, false, M, X, n, true);   // X X^T
        else gemm(h, out, N, N, 1.0, X, n, true, M, X, n, false);        // X^T X
    };
    auto solve = [&](const double* L, const double* Y, double* X) {
        trsm(h, wide, L, Dv.d(), Ni, Y, n, X, n, nvec);
    };
    // ---- CholeskyQR2 with a certifying downward shift on the first factorisation
    const double tau_rel = 4.0 * double(M + 2 * N) * kU;
    int* stv = st.as<int>();
    gram(G.d(), A);
    potrf(h, G.d(), Ni, -tau_rel, Dv.d(), stv + 0);
    solve(G.d(), A, Q1.d());
    gram(L1.d(), Q1.d());
    {
        // second pass: first-order correction when Q1 is already orthonormal to ~1e-8 (then the
        // neglected O(E^2) term is below u), else a full second Cholesky + TRSM
        DevBuf L2(h, N * N * 8), Li2(h, N * N * 8);
        double* emax_dev = static_cast<double*>(h->dev_scratch) + 40;
        const unsigned nb = 8;
        hipLaunchKernelGGL(k_first_order, dim3(nb), dim3(256), 0, h->stream, L1.d(), Ni, L2.d(), Li2.d(), emax_dev);
        check_launch("k_first_order");
        int* hs = static_cast<int*>(h->host_scratch);
        double* hd = static_cast<double*>(h->host_scratch) + 8;
        XRS_HIP(hipMemcpyAsync(hs, stv, 8, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipMemcpyAsync(hd, emax_dev, nb * 8, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipStreamSynchronize(h->stream));
        double em = 0.0;
        for (unsigned i = 0; i < nb; ++i) em = (hd[i] > em || hd[i] != hd[i]) ? hd[i] : em;
        if (hs[0] == 0 && em <= 1e-8) {
            if (wide) {
                gemm(h, Q, N, n, 1.0, Li2.d(), N, false, N, Q1.d(), n, false);      // Q = (I - Elow) Q1
                gemm(h, RL, N, N, 1.0, G.d(), N, false, N, L2.d(), N, false);      // L = L1 L2
            } else {
                gemm(h, Q, m, N, 1.0, Q1.d(), n, false, N, Li2.d(), N, true);      // Q = Q1 (I - Elow)^T
                gemm(h, RL, N, N, 1.0, L2.d(), N, true, N, G.d(), N, true);        // R = L2^T L1^T
            }
            res.certified = true;
            res.cert_ratio = std::sqrt(0.5 * tau_rel);
            return res;
        }
    }
    potrf(h, L1.d(), Ni, 0.0, Dv.d(), stv + 1);
    solve(L1.d(), Q1.d(), Q);
    if (wide) gemm(h, RL, N, N, 1.0, G.d(), N, false, N, L1.d(), N, false);   // L = L1 L2
    else gemm(h, RL, N, N, 1.0, L1.d(), N, true, N, G.d(), N, true);          // R = L2^T L1^T
    int sts[3] = {0, 0, 0};
    if (read_status(h, stv, 2, sts) == 0) {
        res.certified = true;
        res.cert_ratio = std::sqrt(0.5 * tau_rel);
        return res;
    }
    // ---- shifted CholeskyQR3: valid for any kappa(A) < 1/u
    res.robust = true;
    const double s_rel = 11.0 * (double(M) * N + double(N) * (N + 1)) * kU;
    DevBuf Q2(h, m * n * 8), L2(h, N * N * 8), T(h, N * N * 8);
    gram(G.d(), A);
    potrf(h, G.d(), Ni, s_rel, Dv.d(), stv + 0);
    solve(G.d(), A, Q1.d());
    gram(L1.d(), Q1.d());
    potrf(h, L1.d(), Ni, 0.0, Dv.d(), stv + 1);
    solve(L1.d(), Q1.d(), Q2.d());
    gram(L2.d(), Q2.d());
    potrf(h, L2.d(), Ni, 0.0, Dv.d(), stv + 2);
    solve(L2.d(), Q2.d(), Q);
    if (wide) {  // L = L1 L2 L3
        gemm(h, T.d(), N, N, 1.0, G.d(), N, false, N, L1.d(), N, false);
        gemm(h, RL, N, N, 1.0, T.d(), N, false, N, L2.d(), N, false);
    } else {     // R = L3^T L2^T L1^T
        gemm(h, T.d(), N, N, 1.0, L2.d(), N, true, N, L1.d(), N, true);
        gemm(h, RL, N, N, 1.0, T.d(), N, false, N, G.d(), N, true);
    }
    if (read_status(h, stv, 3, sts) == 0) {
        // Cholesky-based passes can "succeed" on an exactly singular Gram with meaningless factors:
        // accept only a verified orthonormal Q (||Q^T Q - I||_max <= 64 n u), else fall through.
        gram(T.d(), Q);
        if (max_abs_dev_identity(h, T.d(), N) <= 64.0 * double(N) * kU) return res;
    }
    // ---- last resort: unpivoted Householder (exact dgeqrf + dorgqr emulation, one workgroup)
    if (!wide) {
        qrcp(h, A, m, n, Q, RL, false, false, false);
    } else {
        DevBuf At(h, m * n * 8), Qt(h, m * n * 8), Rt(h, m * m * 8);
        transpose(h, At.d(), A, m, n);                     // n x m
        qrcp(h, At.d(), n, m, Qt.d(), Rt.d(), false, false, false);   // A^T = Qt Rt
        transpose(h, Q, Qt.d(), n, m);                     // Q = Qt^T (m x n)
        transpose(h, RL, Rt.d(), m, m);                    // L = Rt^T
    }
    return res;
}

// ------------------------------------------------------------------------------------------------
// QC with the reference's rank rule (blasLapackWrapper.cpp:243-305).
static bool small_problem(size_t m, size_t n) { return m * n <= 4096 || std::min(m, n) <= 8; }

static void compact_cols(xrs_handle_t h, double* dst, size_t ldd, const double* src, size_t lds, size_t rows, size_t cols) {
    if (ldd == lds && dst == src) return;
    XRS_HIP(hipMemcpy2DAsync(dst, ldd * 8, src, lds * 8, cols * 8, rows, hipMemcpyDeviceToDevice, h->stream));
}

size_t qc(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* C) {
    XRS_REQUIRE(m > 0 && n > 0, "Dimension m and n must be larger than zero");
    const size_t k = std::min(m, n);
    auto exact = [&] {   // the dgeqp3 emulation on A itself
        DevBuf Qf(h, m * k * 8);
        const size_t r = qrcp(h, A, m, n, Qf.d(), C, true, false, true);
        compact_cols(h, Q, r, Qf.d(), k, m, r);
        return r;
    };
    if (m < n || small_problem(m, n)) return exact();
    OrthResult o;
    try {
        o = orthogonalize(h, A, m, n, false, Q, C);
    } catch (const Error& e) {   // above 512: numerically rank-deficient beyond shifted CholeskyQR3
        if (e.code != XRS_ENUMERIC) throw;
        return exact();
    }
    // certified: sigma_min >= cert*||A||_F > 16 u R_00 (R_00 <= ||A||_F) -> rank n
    if (o.certified && o.cert_ratio > 64.0 * kDblEps) return n;
    // not certified: (numerically) rank-deficient or nearly so. A Gram-based factor of such an A is accurate only
    // to ~kappa u in its near-null directions (an entrywise-product TT moved to core 0 measured 5e-12 relative
    // error through the former pivoted QR of the CholeskyQR factor), so the dgeqp3 emulation runs on A itself
    return exact();
}

// CQ: the reference runs col-major dgeqp3 on A^T (blasLapackWrapper.cpp:317-371), i.e. QC of A^T.
size_t cq(xrs_handle_t h, const double* A, size_t m, size_t n, double* C, double* Q) {
    XRS_REQUIRE(m > 0 && n > 0, "Dimension m and n must be larger than zero");
    const size_t k = std::min(m, n);
    auto exact = [&] {
        DevBuf At(h, m * n * 8), Qt(h, n * k * 8), Ct(h, k * m * 8);
        transpose(h, At.d(), A, m, n);                           // n x m
        const size_t r = qrcp(h, At.d(), n, m, Qt.d(), Ct.d(), true, false, true);   // A^T = Qt Ct
        DevBuf Qc(h, n * r * 8 + 8);
        compact_cols(h, Qc.d(), r, Qt.d(), k, n, r);
        transpose(h, Q, Qc.d(), n, r);                            // Q = Qt^T  (r x n)
        transpose(h, C, Ct.d(), r, m);                            // C = Ct^T  (m x r)
        return r;
    };
    if (n < m || small_problem(m, n)) return exact();
    OrthResult o;
    try {
        o = orthogonalize(h, A, m, n, true, Q, C);               // A = L Q, C := L (m x m)
    } catch (const Error& e) {
        if (e.code != XRS_ENUMERIC) throw;
        return exact();
    }
    if (o.certified && o.cert_ratio > 64.0 * kDblEps) return m;
    return exact();   // (see qc)
}

void qr(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* R) {
    XRS_REQUIRE(m > 0 && n > 0, "Dimension m and n must be larger than zero");
    if (m >= n && !small_problem(m, n)) {
        try {
            orthogonalize(h, A, m, n, false, Q, R);
            return;
        } catch (const Error& e) {   // rank-deficient above 512: the exact dgeqrf emulation
            if (e.code != XRS_ENUMERIC) throw;
        }
    }
    qrcp(h, A, m, n, Q, R, false, false, false);
}

void rq(xrs_handle_t h, const double* A, size_t m, size_t n, double* R, double* Q) {
    XRS_REQUIRE(m > 0 && n > 0, "Dimension m and n must be larger than zero");
    if (m <= n && !small_problem(m, n)) {
        try {
            orthogonalize(h, A, m, n, true, Q, R);
            return;
        } catch (const Error& e) {
            if (e.code != XRS_ENUMERIC) throw;
        }
    }
    const size_t k = std::min(m, n);
    DevBuf At(h, m * n * 8), Qt(h, n * k * 8), Rt(h, k * m * 8);
    transpose(h, At.d(), A, m, n);
    qrcp(h, At.d(), n, m, Qt.d(), Rt.d(), false, false, false);   // A^T = Qt Rt
    transpose(h, Q, Qt.d(), n, k);
    transpose(h, R, Rt.d(), k, m);
}

// U[:, j] *= 1 / S[j] (0 for S[j] == 0): U = R V S^{-1}
__global__ void k_div_cols(double* __restrict__ U, const double* __restrict__ S, size_t m, size_t k) {
    for (size_t e = size_t(blockIdx.x) * blockDim.x + threadIdx.x; e < m * k; e += size_t(gridDim.x) * blockDim.x) {
        const double s = S[e % k];
        U[e] = s > 0.0 ? U[e] / s : 0.0;
    }
}

// 512 < min(m, n) <= 1024: tall A = Q R (shifted CholeskyQR3), the right singular vectors of R by the
// multi-workgroup block Jacobi on its rows (accurate to u for every singular value), U = Q R V S^{-1}
// re-orthonormalised by CholeskyQR (its columns of tiny singular values carry u sigma_0 / sigma_j;
// the re-orthonormalisation keeps U S Vt = A to u ||A||). Wide A through A^T.
static void svd_big(xrs_handle_t h, const double* A, size_t m, size_t n, double* U, double* S, double* Vt) {
    if (m < n) {
        DevBuf At(h, m * n * 8), U2(h, n * m * 8), V2(h, m * m * 8);
        transpose(h, At.d(), A, m, n);                 // n x m, tall
        svd_big(h, At.d(), n, m, U2.d(), S, V2.d());   // A^T = U2 S V2t
        transpose(h, U, V2.d(), m, m);                  // U = V2t^T (m x m)
        transpose(h, Vt, U2.d(), n, m);                 // Vt = U2^T (m x n)
        return;
    }
    XRS_REQUIRE(n <= 1024, "svd: min(m, n) > 1024 not supported");
    DevBuf Q(h, m * n * 8), R(h, n * n * 8), Ur(h, n * n * 8), Uq(h, m * n * 8), Rn(h, n * n * 8), st(h, 64);
    orthogonalize(h, A, m, n, false, Q.d(), R.d());
    XRS_HIP(hipMemsetAsync(st.d(), 0, 64, h->stream));
    jacobi_vt(h, R.d(), int(n), false, int(n), int(n), S, Vt, int(n), st.as<int>(), 60);
    jacobi_settle(h, st.as<int>(), int(n), int(n), [&](int kernel) {   // (-2: recomputed, see jacobi_settle)
        jacobi_vt(h, R.d(), int(n), false, int(n), int(n), S, Vt, int(n), st.as<int>(), 60, kernel);
    });
    gemm(h, Ur.d(), n, n, 1.0, R.d(), n, false, n, Vt, n, true);   // R V = U_R S
    hipLaunchKernelGGL(k_div_cols, dim3(unsigned(std::min<size_t>((n * n + 255) / 256, 4096))), dim3(256), 0, h->stream, Ur.d(), S, n, n);
    check_launch("k_div_cols");
    gemm(h, Uq.d(), m, n, 1.0, Q.d(), n, false, n, Ur.d(), n, false);   // Q U_R
    orthogonalize(h, Uq.d(), m, n, false, U, Rn.d());
}

__global__ void __launch_bounds__(1024) k_amax(const double* __restrict__ x, size_t n, double* __restrict__ out) {
    __shared__ double red[16];
    double mx = 0.0;
    for (size_t e = threadIdx.x; e < n; e += 1024) {
        const double d = fabs(x[e]);
        mx = (d > mx || d != d) ? d : mx;   // NaN propagates
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(mx, o, 64);
        mx = (t > mx || t != t) ? t : mx;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double v = red[0];
        for (int i = 1; i < 16; ++i) v = (red[i] > v || red[i] != red[i]) ? red[i] : v;
        out[0] = v;
    }
}

static void svd_core(xrs_handle_t h, const double* A, size_t m, size_t n, double* U, double* S, double* Vt);

// the bidiagonal route (syev.hip svd_bidiag) on a square n x n A; false: run the Jacobi route (XRS_SVD_BIDIAG=2:
// a failed check throws instead)
static bool try_bidiag(xrs_handle_t h, const double* A, size_t n, double* U, double* S, double* Vt) {
    double diag[4];
    if (svd_bidiag(h, A, int(n), U, S, Vt, diag)) return true;
    if (svd_bidiag_mode() == 2) {
        char msg[200];
        std::snprintf(msg, sizeof msg, "svd_bidiag: check failed (residual %.3g, orthogonality %.3g / %.3g, status %d)", diag[0],
                      diag[1], diag[2], int(diag[3]));
        throw Error{XRS_ENUMERIC, msg};
    }
    return false;
}

void svd(xrs_handle_t h, const double* A, size_t m, size_t n, double* U, double* S, double* Vt) {
    XRS_REQUIRE(m > 0 && n > 0, "Dimension m and n must be larger than zero");
    // square 16..128: the bidiagonal route on A itself (scale-safe by construction)
    if (m == n && n >= 16 && n <= 128 && svd_bidiag_mode() != 0 && try_bidiag(h, A, n, U, S, Vt)) return;
    // range control, dgesdd's dlascl of A into [smlnum, bignum] (here by an exact power of two, to max |A| ~ 1):
    // the Gram-based preconditioning and the Jacobi dots square the entries (unscaled, 1e150-sized entries
    // overflowed them)
    double* am_dev = static_cast<double*>(h->dev_scratch) + 48;
    hipLaunchKernelGGL(k_amax, dim3(1), dim3(1024), 0, h->stream, A, m * n, am_dev);
    check_launch("k_amax");
    double* am_host = static_cast<double*>(h->host_scratch) + 48;
    XRS_HIP(hipMemcpyAsync(am_host, am_dev, 8, hipMemcpyDeviceToHost, h->stream));
    XRS_HIP(hipStreamSynchronize(h->stream));
    const double am = am_host[0];
    if (am > 0.0 && std::isfinite(am) && (am > 0x1p+200 || am < 0x1p-200)) {
        const int ex = std::ilogb(am);
        DevBuf As(h, m * n * 8);
        XRS_HIP(hipMemcpyAsync(As.d(), A, m * n * 8, hipMemcpyDeviceToDevice, h->stream));
        scal(h, As.d(), std::ldexp(1.0, -ex), m * n);
        svd_core(h, As.d(), m, n, U, S, Vt);
        scal(h, S, std::ldexp(1.0, ex), std::min(m, n));
        return;
    }
    svd_core(h, A, m, n, U, S, Vt);
}

static void svd_core(xrs_handle_t h, const double* A, size_t m, size_t n, double* U, double* S, double* Vt) {
    if (std::min(m, n) > size_t(kSmallMax)) {
        svd_big(h, A, m, n, U, S, Vt);
        return;
    }
    const size_t k = std::min(m, n);
    // non-square with 24 <= min(m, n) <= 128: the bidiagonal route on the QR factor (profiles/r06/svd_bidiag_*:
    // 64 x 1000 0.61 vs 5.1 ms, 128 x 2560 1.11 vs 1.71 ms, 300 x 100 0.80 vs 1.45 ms against Jacobi)
    const bool bd = m != n && k >= 24 && k <= 128 && svd_bidiag_mode() != 0;
    // (square 256 / 512 through the QR factor as well: 5.46 vs 4.94 ms and 17.7 vs 18.6 ms -- no gain, r06)
    if (!bd && m <= n && jacobi_usv_fits(int(m), int(n))) {
        jacobi_svd_rows(h, A, int(m), int(n), U, S, Vt);   // rows of A directly
        return;
    }
    // preconditioned (the QR factor's rows are shorter and better conditioned for Jacobi):
    //   wide A = R Q: R = U S Vr, Vt = Vr Q;   tall A = Q R: R = U_R S Vt, U = Q U_R
    DevBuf R(h, k * k * 8), Qf(h, m * n * 8), F(h, k * k * 8);
    if (m <= n) {
        rq(h, A, m, n, R.d(), Qf.d());
        if (!(bd && try_bidiag(h, R.d(), k, U, S, F.d()))) jacobi_svd_rows(h, R.d(), int(k), int(k), U, S, F.d());
        gemm(h, Vt, k, n, 1.0, F.d(), k, false, k, Qf.d(), n, false);
    } else {
        qr(h, A, m, n, Qf.d(), R.d());
        if (!(bd && try_bidiag(h, R.d(), k, F.d(), S, Vt))) jacobi_svd_rows(h, R.d(), int(k), int(k), F.d(), S, Vt);
        gemm(h, U, m, k, 1.0, Qf.d(), k, false, k, F.d(), k, false);
    }
}

}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_qc(xrs_handle_t h, double* Q, double* C, size_t* rank, const double* A, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && Q && C && rank && A, "null argument");
        fence_readers(h);
        *rank = qc(h, A, m, n, Q, C);
    });
}

int xrs_cq(xrs_handle_t h, double* C, double* Q, size_t* rank, const double* A, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && Q && C && rank && A, "null argument");
        fence_readers(h);
        *rank = cq(h, A, m, n, C, Q);
    });
}

int xrs_qr(xrs_handle_t h, double* Q, double* R, const double* A, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && Q && R && A, "null argument");
        fence_readers(h);
        qr(h, A, m, n, Q, R);
    });
}

int xrs_rq(xrs_handle_t h, double* R, double* Q, const double* A, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && Q && R && A, "null argument");
        fence_readers(h);
        rq(h, A, m, n, R, Q);
    });
}

int xrs_svd(xrs_handle_t h, double* U, double* S, double* Vt, const double* A, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && U && S && Vt && A, "null argument");
        fence_readers(h);
        svd(h, A, m, n, U, S, Vt);
    });
}

int xrs_sym_eig_top(xrs_handle_t h, double* lam, double* Ut, int* status, const double* A, size_t n, size_t kk) {
    return guarded([&] {
        XRS_REQUIRE(h && lam && Ut && status && A, "null argument");
        XRS_REQUIRE(n >= 2 && n <= 256 && kk >= 1 && kk <= n, "xrs_sym_eig_top: need 2 <= n <= 256 and 1 <= kk <= n");
        fence_readers(h);
        DevBuf st(h, 64);
        XRS_HIP(hipMemsetAsync(st.d(), 0, 64, h->stream));
        sym_eig_top(h, A, int(n), int(n), int(kk), lam, nullptr, Ut, int(n), st.as<int>());
        read_status(h, st.as<int>(), 1, status);
    });
}

int xrs_sym_tridiag(xrs_handle_t h, double* d, double* e, const double* A, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && d && e && A, "null argument");
        XRS_REQUIRE(n >= 2 && n <= 256, "xrs_sym_tridiag: need 2 <= n <= 256");
        fence_readers(h);
        sym_tridiag(h, A, int(n), int(n), d, e);
        XRS_HIP(hipStreamSynchronize(h->stream));
    });
}

int xrs_svd_rows_vt(xrs_handle_t h, double* S, double* Vt, int* sweeps, const double* A, size_t p, size_t q, int kernel) {
    return guarded([&] {
        XRS_REQUIRE(h && S && Vt && A && sweeps, "null argument");
        XRS_REQUIRE(p >= 1 && p <= q && q <= 1024 && (kernel != 1 || p <= 512),
                    "xrs_svd_rows_vt: need 1 <= p <= q <= 1024 (kernel 1: p <= 512)");
        DevBuf st(h, 64);
        XRS_HIP(hipMemsetAsync(st.d(), 0, 64, h->stream));
        jacobi_vt(h, A, int(q), false, int(p), int(q), S, Vt, int(q), st.as<int>(), 40, kernel, stamps_enabled("svd"));
        int sts[9];
        read_status(h, st.as<int>(), 9, sts);
        *sweeps = sts[0];
        if (stamps_enabled("svd"))
            std::fprintf(stderr, "jacobi_vt p=%zu q=%zu kernel=%d: sweeps %d, 100 MHz ticks: total %d, grid barriers %d, exchange %d; "
                         "thread-0 cross-round cycles: dot %d, rotation %d, update %d, barrier %d, rotations %d\n",
                         p, q, kernel, sts[0], sts[1], sts[2], sts[3], sts[4], sts[5], sts[6], sts[7], sts[8]);
    });
}

}  // extern "C"
