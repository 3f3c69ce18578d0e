// Right singular vectors of a small dense matrix by one-sided Jacobi on its rows (the SVD inside TT
// truncation: round_edge's calculate_svd, tensorNetwork.cpp:764 -> tensor.cpp:1424-1489 ->
// blasWrapper::svd / dgesdd, blasLapackWrapper.cpp:201-232).
//
// For W (p x q, p <= q) the rows are rotated pairwise until mutually orthogonal: J W = Wr, so
// sigma_i = ||Wr_i||, Vt_i = Wr_i / sigma_i and W = U S Vt with U S = W Vt^T -- the caller never needs J,
// so nothing but W is stored and for p*q <= 18 K doubles W lives in LDS for the whole solve.
//
// Layout of one round (round-robin "circle" pairing of the P = p rounded up to even players): pair t is
// (player at position t, player at position P-1-t); position 0 is fixed, the others rotate by one per
// round, so P-1 rounds meet every pair once (a sweep). A pair is handled by a 16-lane group (a DPP row):
// its three dot products are reduced with row_ror DPP butterflies (identical bits in all 16 lanes, so
// every lane computes the same rotation), the rotation is applied in Rutishauser's form
// x' = x - s (y + tau x), y' = y + s (x - tau y) (O(u s) perturbation for nearly-identity rotations).
// 1024 threads = 64 groups: up to 64 pairs per round in flight, one barrier per round.
// Convergence: no pair with |w_i . w_j| > tol ||w_i|| ||w_j||, tol = sqrt(q) u (dgesvj's criterion).
#include <cmath>

#include "smallla.hpp"

namespace xrs {

namespace {

constexpr int SV_THREADS = 1024;
constexpr int SV_GROUPS = SV_THREADS / 16;
constexpr int SV_LDS = 18432;   // doubles (144 KiB)
constexpr int SV_MAXP = 512;

// DPP row_ror:n on a double (two 32-bit moves); all 16 lanes of a row take part
template <int N>
__device__ __forceinline__ double ror16(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x120 + N, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x120 + N, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// sum over the 16 lanes of a DPP row; every lane ends with the same bits (rotations of a periodic sequence)
__device__ __forceinline__ double sum16(double v) {
    v += ror16<8>(v);
    v += ror16<4>(v);
    v += ror16<2>(v);
    v += ror16<1>(v);
    return v;
}

// player at position x of round `round` (circle method, P players, position 0 fixed)
__device__ __forceinline__ int player(int x, int round, int P) { return x == 0 ? 0 : 1 + (x - 1 + round) % (P - 1); }

// W (ldw) is the working copy (LDS or global scratch); Win (row stride ldin) the input.
template <bool LDS>
__device__ void jacobi_rows_body(double* __restrict__ W, int ldw, const double* __restrict__ Win, int ldin, bool trans, int p, int q,
                                 int max_sweeps, double* __restrict__ S, double* __restrict__ Vt, int ldvt,
                                 int* __restrict__ status, double* __restrict__ scratch_norm) {
    const int tid = threadIdx.x, g = tid >> 4, l = tid & 15;
    __shared__ int rotated;
    __shared__ double sn[SV_MAXP];
    __shared__ int rk[SV_MAXP];
    for (int e = tid; e < p * q; e += SV_THREADS) {
        const int i = e / q, k = e - i * q;
        W[size_t(i) * ldw + k] = trans ? Win[size_t(k) * ldin + i] : Win[size_t(i) * ldin + k];
    }
    __syncthreads();
    const int P = (p + 1) & ~1;
    const double tol = sqrt(double(q)) * 1.1102230246251565e-16;
    int sweep = 0;
    bool converged = false;
    for (; sweep < max_sweeps && !converged; ++sweep) {
        if (tid == 0) rotated = 0;
        __syncthreads();
        for (int round = 0; round < P - 1; ++round) {
            for (int t = g; t < P / 2; t += SV_GROUPS) {
                int i = player(t, round, P), j = player(P - 1 - t, round, P);
                if (i >= p || j >= p) continue;
                double* wi = W + size_t(i) * ldw;
                double* wj = W + size_t(j) * ldw;
                double a = 0.0, b = 0.0, c = 0.0;
                for (int k = l; k < q; k += 16) {
                    const double x = wi[k], y = wj[k];
                    a = fma(x, x, a);
                    b = fma(y, y, b);
                    c = fma(x, y, c);
                }
                a = sum16(a);
                b = sum16(b);
                c = sum16(c);
                if (fabs(c) > tol * sqrt(a) * sqrt(b) && c != 0.0) {
                    const double zeta = (b - a) / (2.0 * c);
                    const double tn = copysign(1.0, zeta) / (fabs(zeta) + sqrt(fma(zeta, zeta, 1.0)));
                    const double cs = 1.0 / sqrt(fma(tn, tn, 1.0));
                    const double s = cs * tn;
                    const double tau = s / (1.0 + cs);
                    for (int k = l; k < q; k += 16) {
                        const double x = wi[k], y = wj[k];
                        wi[k] = x - s * fma(tau, x, y);
                        wj[k] = y + s * fma(-tau, y, x);
                    }
                    if (l == 0) rotated = 1;
                }
            }
            __syncthreads();
        }
        converged = rotated == 0;
        __syncthreads();
    }
    // singular values = row norms, ranked descending (ties by index: a stable order)
    for (int i = g; i < p; i += SV_GROUPS) {
        const double* wi = W + size_t(i) * ldw;
        double a = 0.0;
        for (int k = l; k < q; k += 16) a = fma(wi[k], wi[k], a);
        a = sum16(a);
        if (l == 0) sn[i] = sqrt(a);
    }
    __syncthreads();
    for (int i = tid; i < p; i += SV_THREADS) {
        const double si = sn[i];
        int r = 0;
        for (int j2 = 0; j2 < p; ++j2) r += (sn[j2] > si) || (sn[j2] == si && j2 < i);
        rk[i] = r;
        S[r] = si;
    }
    __syncthreads();
    for (int e = tid; e < p * q; e += SV_THREADS) {
        const int i = e / q, k = e - i * q;
        const double s = sn[i];
        Vt[size_t(rk[i]) * ldvt + k] = s > 0.0 ? W[size_t(i) * ldw + k] / s : 0.0;
    }
    if (tid == 0) status[0] = converged ? sweep : -1;
    (void)scratch_norm;
}

__global__ void __launch_bounds__(SV_THREADS) k_jacobi_vt_lds(const double* __restrict__ Win, int ldin, int trans, int p, int q, int max_sweeps,
                                                              double* __restrict__ S, double* __restrict__ Vt, int ldvt,
                                                              int* __restrict__ status) {
    __shared__ double Ws[SV_LDS];
    const int ldw = q + ((q & 1) ? 0 : 1);   // odd stride: the 4 rows a wave touches spread over the banks
    jacobi_rows_body<true>(Ws, ldw, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status, nullptr);
}

__global__ void __launch_bounds__(SV_THREADS) k_jacobi_vt_global(double* __restrict__ Wg, const double* __restrict__ Win, int ldin,
                                                                 int trans, int p, int q, int max_sweeps, double* __restrict__ S,
                                                                 double* __restrict__ Vt, int ldvt, int* __restrict__ status) {
    jacobi_rows_body<false>(Wg, q, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status, nullptr);
}

}  // namespace

bool jacobi_vt_fits_lds(int p, int q) { return size_t(p) * size_t(q + 1) <= size_t(SV_LDS); }

void jacobi_vt(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* S, double* Vt, int ldvt,
               int* status_dev, int max_sweeps) {
    XRS_REQUIRE(p >= 1 && p <= SV_MAXP && p <= q, "jacobi_vt: need 1 <= p <= min(q, 512)");
    KernelTimer timer(h, XRS_KFAM_SVD, 3.5 * double(p) * p * q * 6.0, 16.0 * double(p) * q);
    if (jacobi_vt_fits_lds(p, q)) {
        hipLaunchKernelGGL(k_jacobi_vt_lds, dim3(1), dim3(SV_THREADS), 0, h->stream, W, ldw, int(trans), p, q, max_sweeps, S, Vt,
                           ldvt, status_dev);
        check_launch("k_jacobi_vt_lds");
    } else {
        DevBuf Wg(h, size_t(p) * q * 8);
        hipLaunchKernelGGL(k_jacobi_vt_global, dim3(1), dim3(SV_THREADS), 0, h->stream, Wg.d(), W, ldw, int(trans), p, q, max_sweeps, S,
                           Vt, ldvt, status_dev);
        check_launch("k_jacobi_vt_global");
    }
}

}  // namespace xrs
