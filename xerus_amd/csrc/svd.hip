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
// round, so P-1 rounds meet every pair once (a sweep). A pair is handled by a group of 8 lanes (LDS
// kernel, 512 threads) or 16 lanes (global kernel): its three dot products are reduced with DPP
// butterflies (identical bits in every lane of the group, so all compute the same rotation), the
// rotation parameters come from hardware rcp/rsq estimates + Newton steps, and the rotation is applied
// in Rutishauser's form x' = x - s (y + tau x), y' = y + s (x - tau y) (O(u s) perturbation for
// nearly-identity rotations). 64 groups: up to 64 pairs per round in flight, one barrier per round.
// Convergence: no pair with |w_i . w_j| > tol ||w_i|| ||w_j||, tol = sqrt(q) u (dgesvj's criterion).
#include <cmath>

#include "smallla.hpp"

namespace xrs {

namespace {

constexpr int SV_LDS = 18432;   // doubles (144 KiB)
constexpr int SV_MAXP = 512;

// DPP move of a double (two 32-bit moves); CTRL is a DPP16 control word
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Sum over a group of G (8 or 16) consecutive lanes. Every lane of the group ends with the same bits:
// each step adds two values that are equal up to the order of operands of commutative adds.
//   G = 16: row_ror 8, 4, 2, 1 (rotations of an increasingly periodic sequence)
//   G = 8:  row_half_mirror (i <-> 7-i), quad_perm [2,3,0,1] (i <-> i^2), quad_perm [1,0,3,2] (i <-> i^1)
template <int G>
__device__ __forceinline__ double gsum(double v) {
    if constexpr (G == 16) {
        v += dpp<0x128>(v);
        v += dpp<0x124>(v);
        v += dpp<0x122>(v);
        v += dpp<0x121>(v);
    } else {
        static_assert(G == 8, "groups of 8 or 16 lanes");
        v += dpp<0x141>(v);
        v += dpp<0x4E>(v);
        v += dpp<0xB1>(v);
    }
    return v;
}

// 1/x and sqrt(x) to ~1 ulp from the hardware estimates + Newton steps (rotation parameters only need
// to be mutually consistent; no IEEE division / square-root sequences in the per-round critical path)
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double fsqrt(double x) {   // x > 0
    double y = __builtin_amdgcn_rsq(x);
    double h = 0.5 * y;
    double g = x * y;
    double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    r = fma(-g, h, 0.5);
    return fma(g, r, g);
}

// Jacobi rotation zeroing the (i,j) entry of [[a c][c b]]: t = tan(theta) = sign(b - a) 2c /
// (|b - a| + sqrt((b - a)^2 + 4 c^2)) (the smaller root), c = 1/sqrt(1+t^2), s = t c, tau = s / (1 + c)
__device__ __forceinline__ void rotation(double a, double b, double c, double& s, double& tau) {
    const double dd = b - a;
    const double hh = fsqrt(fma(dd, dd, 4.0 * c * c));
    const double tn = copysign(2.0, dd) * c * frcp(fabs(dd) + hh);
    const double qq = fsqrt(fma(tn, tn, 1.0));
    const double cs = frcp(qq);
    s = tn * cs;
    tau = s * frcp(1.0 + cs);   // Rutishauser: x' = x - s (y + tau x), y' = y + s (x - tau y)
}

// player at position x of round `round` (circle method, P players, position 0 fixed)
__device__ __forceinline__ int player(int x, int round, int P) { return x == 0 ? 0 : 1 + (x - 1 + round) % (P - 1); }

// W (ldw) is the working copy (LDS or global scratch); Win (row stride ldin, or transposed) the input.
// E > 0: q <= E * G, the lane's elements of a row pair are held in registers (unrolled); E = 0: any q
template <int G, int NT, int E>
__device__ void jacobi_rows_body(double* __restrict__ W, int ldw, const double* __restrict__ Win, int ldin, bool trans, int p, int q,
                                 int max_sweeps, double* __restrict__ S, double* __restrict__ Vt, int ldvt,
                                 int* __restrict__ status) {
    constexpr int GROUPS = NT / G;
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    __shared__ int rotated;
    __shared__ double sn[SV_MAXP];
    __shared__ int rk[SV_MAXP];
    if (trans) {   // W[i][k] = Win[k][i]: read along Win's rows
        for (int e = tid; e < p * q; e += NT) {
            const int k = e / p, i = e - k * p;
            W[size_t(i) * ldw + k] = Win[size_t(k) * ldin + i];
        }
    } else {
        for (int e = tid; e < p * q; e += NT) {
            const int i = e / q, k = e - i * q;
            W[size_t(i) * ldw + k] = Win[size_t(i) * ldin + k];
        }
    }
    __syncthreads();
    const int P = (p + 1) & ~1;
    const double tol = sqrt(double(q)) * 1.1102230246251565e-16;
    const double tol2 = tol * tol;
    int sweep = 0;
    bool converged = false;
    for (; sweep < max_sweeps && !converged; ++sweep) {
        if (tid == 0) rotated = 0;
        __syncthreads();
        for (int round = 0; round < P - 1; ++round) {
            for (int t = g; t < P / 2; t += GROUPS) {
                int i = 0, j;   // players at positions t and P-1-t (player() without the integer divisions)
                if (t > 0) {
                    i = t + round;
                    i = i >= P ? i - (P - 1) : i;
                }
                j = P - 1 - t + round;
                j = j >= P ? j - (P - 1) : j;
                if (i >= p || j >= p) continue;
                double* wi = W + size_t(i) * ldw;
                double* wj = W + size_t(j) * ldw;
                if constexpr (E > 0) {
                    // the lane's E elements of both rows in registers: all loads issued before any use
                    double x[E], y[E];
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int k = l + e * G;
                        x[e] = k < q ? wi[k] : 0.0;
                        y[e] = k < q ? wj[k] : 0.0;
                    }
                    double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        a = fma(x[e], x[e], a);
                        b = fma(y[e], y[e], b);
                        c = fma(x[e], y[e], c);
                    }
                    a = gsum<G>(a);
                    b = gsum<G>(b);
                    c = gsum<G>(c);
                    if (c * c > tol2 * a * b) {
                        double s, tau;
                        rotation(a, b, c, s, tau);
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int k = l + e * G;
                            if (k < q) {
                                wi[k] = x[e] - s * fma(tau, x[e], y[e]);
                                wj[k] = y[e] + s * fma(-tau, y[e], x[e]);
                            }
                        }
                        if (l == 0) rotated = 1;
                    }
                } else {
                    double a = 0.0, b = 0.0, c = 0.0;
                    for (int k = l; k < q; k += G) {
                        const double x = wi[k], y = wj[k];
                        a = fma(x, x, a);
                        b = fma(y, y, b);
                        c = fma(x, y, c);
                    }
                    a = gsum<G>(a);
                    b = gsum<G>(b);
                    c = gsum<G>(c);
                    if (c * c > tol2 * a * b) {
                        double s, tau;
                        rotation(a, b, c, s, tau);
                        for (int k = l; k < q; k += G) {
                            const double x = wi[k], y = wj[k];
                            wi[k] = x - s * fma(tau, x, y);
                            wj[k] = y + s * fma(-tau, y, x);
                        }
                        if (l == 0) rotated = 1;
                    }
                }
            }
            __syncthreads();
        }
        converged = rotated == 0;
        __syncthreads();
    }
    // singular values = row norms, ranked descending (ties by index: a stable order)
    for (int i = g; i < p; i += GROUPS) {
        const double* wi = W + size_t(i) * ldw;
        double a = 0.0;
        for (int k = l; k < q; k += G) a = fma(wi[k], wi[k], a);
        a = gsum<G>(a);
        if (l == 0) sn[i] = sqrt(a);
    }
    __syncthreads();
    for (int i = tid; i < p; i += NT) {
        const double si = sn[i];
        int r = 0;
        for (int j2 = 0; j2 < p; ++j2) r += (sn[j2] > si) || (sn[j2] == si && j2 < i);
        rk[i] = r;
        S[r] = si;
    }
    __syncthreads();
    for (int e = tid; e < p * q; e += NT) {
        const int i = e / q, k = e - i * q;
        const double s = sn[i];
        Vt[size_t(rk[i]) * ldvt + k] = s > 0.0 ? W[size_t(i) * ldw + k] / s : 0.0;
    }
    if (tid == 0) status[0] = converged ? sweep : -1;
}

// LDS-resident: 512 threads, 8 lanes per pair (64 pairs in flight, two waves per SIMD)
constexpr int SVL_THREADS = 512;
__global__ void __launch_bounds__(SVL_THREADS) k_jacobi_vt_lds(const double* __restrict__ Win, int ldin, int trans, int p, int q,
                                                               int max_sweeps, double* __restrict__ S, double* __restrict__ Vt,
                                                               int ldvt, int* __restrict__ status) {
    __shared__ double Ws[SV_LDS];
    const int ldw = q + ((q & 1) ? 0 : 1);   // odd stride: the rows a wave touches spread over the banks
    jacobi_rows_body<8, SVL_THREADS, 16>(Ws, ldw, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
}

// W in global memory (L2-resident) for larger matrices: 1024 threads, 16 lanes per pair
constexpr int SVG_THREADS = 1024;
__global__ void __launch_bounds__(SVG_THREADS) k_jacobi_vt_global(double* __restrict__ Wg, const double* __restrict__ Win, int ldin,
                                                                  int trans, int p, int q, int max_sweeps, double* __restrict__ S,
                                                                  double* __restrict__ Vt, int ldvt, int* __restrict__ status) {
    if (q <= 256) jacobi_rows_body<16, SVG_THREADS, 16>(Wg, q, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
    else jacobi_rows_body<16, SVG_THREADS, 0>(Wg, q, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
}

}  // namespace

bool jacobi_vt_fits_lds(int p, int q) { return q <= 128 && size_t(p) * size_t(q + 1) <= size_t(SV_LDS); }

void jacobi_vt(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* S, double* Vt, int ldvt,
               int* status_dev, int max_sweeps) {
    XRS_REQUIRE(p >= 1 && p <= SV_MAXP && p <= q, "jacobi_vt: need 1 <= p <= min(q, 512)");
    KernelTimer timer(h, XRS_KFAM_SVD, 3.5 * double(p) * p * q * 6.0, 16.0 * double(p) * q);
    if (jacobi_vt_fits_lds(p, q)) {
        hipLaunchKernelGGL(k_jacobi_vt_lds, dim3(1), dim3(SVL_THREADS), 0, h->stream, W, ldw, int(trans), p, q, max_sweeps, S, Vt,
                           ldvt, status_dev);
        check_launch("k_jacobi_vt_lds");
    } else {
        DevBuf Wg(h, size_t(p) * q * 8);
        hipLaunchKernelGGL(k_jacobi_vt_global, dim3(1), dim3(SVG_THREADS), 0, h->stream, Wg.d(), W, ldw, int(trans), p, q, max_sweeps, S,
                           Vt, ldvt, status_dev);
        check_launch("k_jacobi_vt_global");
    }
}

}  // namespace xrs
