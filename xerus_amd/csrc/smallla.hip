// Small dense factorisation kernels (n <= 512) used by the QR / SVD drivers in linalg.cpp.
//
//   k_potrf   one workgroup: blocked right-looking Cholesky G = L L^T (+ optional diagonal shift),
//             32x32 diagonal blocks factored in registers of one wave (v_readlane broadcasts),
//             panel staged in LDS, trailing update with 4x4 register tiles. Also emits the inverse
//             of every diagonal block for the TRSM kernel, and a failure code (column of the first
//             non-positive pivot).
//   k_trsm    many workgroups: X = L^{-1} Y for 32 right-hand sides per workgroup, RHS either the
//             rows (tall CholQR: Q1 = A L^{-T}) or the columns (wide CholQR: Q1 = L^{-1} B) of a
//             row-major matrix; left-looking over 32-row blocks with the RHS block resident in LDS.
//   k_qrcp    one workgroup: exact emulation of LAPACK dgeqp3 (dlaqp2 column pivoting with the
//             partial-norm downdate, dlarfg sign convention) + dorgqr, on a column-major copy. This is
//             the reference's QC (blasLapackWrapper.cpp:243-305) including its rank rule (:268-272).
//   k_jacobi  one workgroup: one-sided (Hestenes) Jacobi SVD of the rows of a p x q matrix, p <= q,
//             round-robin parallel ordering, rotations accumulated in J (U = J^T).
#include "smallla.hpp"

namespace xrs {

constexpr int NB = 32;
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int PMAX = 512;
constexpr int POT_THREADS = 512;   // 8 waves, two per SIMD: 256 VGPRs for the register-resident 32-wide steps

__device__ __forceinline__ double readlane_d(double v, int l) {
    union { double d; int i[2]; } u;
    u.d = v;
    u.i[0] = __builtin_amdgcn_readlane(u.i[0], l);
    u.i[1] = __builtin_amdgcn_readlane(u.i[1], l);
    return u.d;
}

// ---------------------------------------------------------------------------------------------
// Cholesky, one workgroup of 1024 threads, 32-wide blocks, right-looking. Per block column:
//   (1) wave 0 factors the 32x32 diagonal block in registers (lane r owns row r, v_readlane
//       broadcasts; 64 VGPRs so nothing spills at the 128-VGPR budget of a 1024-thread workgroup);
//   (2) wave 1 inverts it (D^{-1}, for the TRSM kernel) while the other waves solve the panel rows
//       x D^T = g by substitution against D in LDS (one row per thread, 32 registers);
//   (3) all waves apply the rank-32 trailing update from the LDS panel with 4x4 register tiles.
__global__ void __launch_bounds__(POT_THREADS) k_potrf(double* __restrict__ G, int n, double shift_rel, double* __restrict__ Dinv,
                                                 int* __restrict__ status, double* __restrict__ info) {
    __shared__ double P[PMAX * (NB + 1)];
    __shared__ double Ds[NB][NB + 1];
    __shared__ double red[16];
    __shared__ int fail;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double* dummy = Dinv + size_t(n + 31) * NB + (tid & 31);   // padding row of Dinv: sink for masked stores
    if (tid == 0) fail = 0;
    // trace(G) -> absolute shift (shift_rel * trace), no host round trip
    double tr = 0.0;
    for (int i = tid; i < n; i += POT_THREADS) tr += G[size_t(i) * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
    if (lane == 0) red[wave] = tr;
    __syncthreads();
    tr = 0.0;
    for (int w = 0; w < POT_THREADS / 64; ++w) tr += red[w];
    if (tid == 0 && info) info[0] = tr;
    const double shift = shift_rel * tr;
    if (shift != 0.0)
        for (int i = tid; i < n; i += POT_THREADS) G[size_t(i) * n + i] += shift;
    __syncthreads();
    for (int j0 = 0; j0 < n; j0 += NB) {
        const int jb = min(NB, n - j0);
        for (int e = tid; e < NB * NB; e += POT_THREADS) {
            const int r = e / NB, c = e % NB;
            double v = (r == c) ? 1.0 : 0.0;
            if (r < jb && c < jb && c <= r) v = G[size_t(j0 + r) * n + j0 + c];
            Ds[r][c] = v;
        }
        __syncthreads();
        // (1) diagonal block: wave 0, lane r holds row r in registers, v_readlane broadcasts
        if (wave == 0) {
            const int r = lane & 31;
            double row[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) row[c] = Ds[r][c];
            int bad = 0;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                double dkk = readlane_d(row[k], k);
                const bool okp = (dkk > 0.0) && (dkk < 1.0e300);   // rejects <= 0, NaN and Inf
                if (!okp && bad == 0 && k < jb) bad = k + 1;
                if (!okp) dkk = 1.0;
                const double d = sqrt(dkk);
                const double inv = 1.0 / d;
                row[k] = (r == k) ? d : ((r > k) ? row[k] * inv : row[k]);
#pragma unroll
                for (int l = k + 1; l < NB; ++l) {
                    const double v = readlane_d(row[k], l);
                    if (r >= l) row[l] -= row[k] * v;
                }
            }
            if (lane < 32) {
#pragma unroll
                for (int c = 0; c < NB; ++c) Ds[r][c] = (c <= r) ? row[c] : 0.0;
            }
            if (lane == 0 && bad && fail == 0) fail = j0 + bad;
        }
        __syncthreads();
        const int t = n - j0 - jb;
        if (wave == 1) {
            // (2a) D^{-1}: lane c computes column c by right-looking substitution in registers.
            // Stores are unconditional (Dinv is padded to n+32 rows): a runtime-bounded store loop
            // would make the compiler index x[] dynamically and spill it to scratch.
            const int c = lane & 31;
            double x[NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) x[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                x[k] = x[k] / Ds[k][k];
#pragma unroll
                for (int i = k + 1; i < NB; ++i) x[i] -= Ds[i][k] * x[k];
            }
            if (lane < 32) {
                double* out = Dinv + size_t(j0) * NB + c;
#pragma unroll
                for (int i = 0; i < NB; ++i) out[size_t(i) * NB] = x[i];
            }
        } else {
            const int wt = (tid >= 64) ? tid - 64 : tid;   // waves 0, 2, 3, ...
            for (int e = wt; e < NB * NB; e += POT_THREADS - 64) {
                const int r = e / NB, c = e % NB;
                if (r < jb && c < jb && c <= r) G[size_t(j0 + r) * n + j0 + c] = Ds[r][c];
            }
            // (2b) panel rows: x D^T = g  <=>  x_c = (g_c - sum_{k<c} x_k D[c][k]) / D[c][c]
            if (jb == NB) {
                for (int rr = wt; rr < t; rr += POT_THREADS - 64) {
                    double* grow = G + size_t(j0 + jb + rr) * n + j0;
                    // opaque LDS base per iteration: otherwise LICM hoists all 528 loop-invariant D loads
                    // out of the row loop and spills them
                    int off = 0;
                    asm volatile("" : "+v"(off));
                    const double* D = &Ds[0][0] + off;
                    double x[NB];
#pragma unroll
                    for (int c = 0; c < NB; ++c) x[c] = grow[c];
#pragma unroll
                    for (int k = 0; k < NB; ++k) {
                        x[k] = x[k] / D[k * (NB + 1) + k];
#pragma unroll
                        for (int c = k + 1; c < NB; ++c) x[c] -= x[k] * D[c * (NB + 1) + k];
                    }
                    double* prow = P + rr * (NB + 1);
#pragma unroll
                    for (int c = 0; c < NB; ++c) {
                        prow[c] = x[c];
                        grow[c] = x[c];
                    }
                }
            } else {
                // last partial block: plain loops (rare: only when n is not a multiple of 32)
                for (int rr = wt; rr < t; rr += POT_THREADS - 64) {
                    double* grow = G + size_t(j0 + jb + rr) * n + j0;
                    double* prow = P + rr * (NB + 1);
                    for (int c = 0; c < NB; ++c) prow[c] = (c < jb) ? grow[c] : 0.0;
                    for (int k = 0; k < jb; ++k) {
                        const double xk = prow[k] / Ds[k][k];
                        prow[k] = xk;
                        grow[k] = xk;
                        for (int c = k + 1; c < jb; ++c) prow[c] -= xk * Ds[c][k];
                    }
                }
            }
        }
        __syncthreads();
        if (t > 0) {
            // (3) trailing update G22 -= P P^T on 16x16 tiles with v_mfma_f64_16x16x4_f64 (K = 32 in
            //     8 steps); one wave per tile, lower tiles only (the strict upper triangle of diagonal
            //     tiles receives harmless garbage and is zeroed at the end).
            //     A frag: lane l -> P[i0 + (l&15)][c + (l>>4)]; B frag: P[k0 + (l&15)][c + (l>>4)];
            //     C/D (f64): row (l>>4) + 4r, col l&15.
            const int T = (t + 15) / 16;
            const int ntiles = T * (T + 1) / 2;
            const int lr = lane & 15, lk = lane >> 4;
            for (int tile = wave; tile < ntiles; tile += POT_THREADS / 64) {
                // decode lower-triangular tile index -> (ti, tk), tk <= ti
                int ti = int((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
                while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
                while (ti * (ti + 1) / 2 > tile) --ti;
                const int tk = tile - ti * (ti + 1) / 2;
                const int i0 = ti * 16, k0 = tk * 16;
                auto cptr = [&](int r) -> double* {
                    const int i = i0 + lk + 4 * r, k = k0 + lr;
                    const bool ok = (i < t) && (k < t);
                    return ok ? (G + size_t(j0 + jb + i) * n + j0 + jb + k) : dummy;
                };
                const double cv0 = *cptr(0), cv1 = *cptr(1), cv2 = *cptr(2), cv3 = *cptr(3);
                d4 acc = {0.0, 0.0, 0.0, 0.0};
                const int ra = min(i0 + lr, t - 1), rb = min(k0 + lr, t - 1);
#pragma unroll
                for (int c = 0; c < NB; c += 4) {
                    const double av = P[ra * (NB + 1) + c + lk];
                    const double bv = P[rb * (NB + 1) + c + lk];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
                *cptr(0) = cv0 - acc[0];
                *cptr(1) = cv1 - acc[1];
                *cptr(2) = cv2 - acc[2];
                *cptr(3) = cv3 - acc[3];
            }
        }
        __syncthreads();
    }
    for (int e = tid; e < n * n; e += POT_THREADS) {
        const int r = e / n, c = e % n;
        if (c > r) G[size_t(r) * n + c] = 0.0;
    }
    if (tid == 0) status[0] = fail;
}

// ---------------------------------------------------------------------------------------------
// Triangular solve X = L^{-1} Y for 32 right-hand sides per workgroup (256 threads). The RHS block
// lives in LDS as Xs[n][33]; per 32-row block I: T = Y_I - L[I, :i0] X[:i0] (2x2 register tiles,
// L read through L1) then X_I = Dinv_I T (the diagonal-block inverses from k_potrf).
template <bool COLS>
__global__ void __launch_bounds__(256) k_trsm(const double* __restrict__ L, const double* __restrict__ Dinv, int n,
                                              const double* __restrict__ Y, size_t ldy, double* __restrict__ X, size_t ldx,
                                              int nvec) {
    extern __shared__ double Xs[];  // [n][NB + 1]
    __shared__ double Ts[NB][NB + 1];
    constexpr int S = NB + 1;
    const int tid = threadIdx.x;
    const int v0 = blockIdx.x * NB;
    const int nv = min(NB, nvec - v0);
    for (int e = tid; e < n * NB; e += 256) {
        int i, v;
        if (COLS) { i = e / NB; v = e % NB; } else { v = e / n; i = e % n; }
        double y = 0.0;
        if (v < nv) y = COLS ? Y[size_t(i) * ldy + v0 + v] : Y[size_t(v0 + v) * ldy + i];
        Xs[i * S + v] = y;
    }
    __syncthreads();
    // 2x2 tile: rows r0, r0+16 ; vectors c0, c0+16
    const int r0 = tid >> 4;        // 0..15
    const int c0 = tid & 15;        // 0..15
    for (int i0 = 0; i0 < n; i0 += NB) {
        const int ib = min(NB, n - i0);
        {
            const int ra = min(i0 + r0, n - 1), rb = min(i0 + r0 + 16, n - 1);
            double t00 = Xs[ra * S + c0], t01 = Xs[ra * S + c0 + 16];
            double t10 = Xs[rb * S + c0], t11 = Xs[rb * S + c0 + 16];
            const double* la = L + size_t(ra) * n;
            const double* lb = L + size_t(rb) * n;
            for (int j = 0; j < i0; ++j) {
                const double a = la[j], b = lb[j];
                const double x0 = Xs[j * S + c0], x1 = Xs[j * S + c0 + 16];
                t00 -= a * x0; t01 -= a * x1;
                t10 -= b * x0; t11 -= b * x1;
            }
            Ts[r0][c0] = t00; Ts[r0][c0 + 16] = t01;
            Ts[r0 + 16][c0] = t10; Ts[r0 + 16][c0 + 16] = t11;
        }
        __syncthreads();
        {
            double x00 = 0, x01 = 0, x10 = 0, x11 = 0;
            const double* da = Dinv + size_t(min(i0 + r0, n - 1)) * NB;
            const double* db = Dinv + size_t(min(i0 + r0 + 16, n - 1)) * NB;
            for (int k = 0; k < NB; ++k) {
                const double a = da[k], b = db[k];
                const double t0 = Ts[k][c0], t1 = Ts[k][c0 + 16];
                x00 += a * t0; x01 += a * t1;
                x10 += b * t0; x11 += b * t1;
            }
            if (r0 < ib) { Xs[(i0 + r0) * S + c0] = x00; Xs[(i0 + r0) * S + c0 + 16] = x01; }
            if (r0 + 16 < ib) { Xs[(i0 + r0 + 16) * S + c0] = x10; Xs[(i0 + r0 + 16) * S + c0 + 16] = x11; }
        }
        __syncthreads();
    }
    for (int e = tid; e < n * NB; e += 256) {
        int i, v;
        if (COLS) { i = e / NB; v = e % NB; } else { v = e / n; i = e % n; }
        if (v < nv) {
            if (COLS) X[size_t(i) * ldx + v0 + v] = Xs[i * S + v];
            else X[size_t(v0 + v) * ldx + i] = Xs[i * S + v];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Block reductions for the single-workgroup kernels (1024 threads).
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// sum over the whole workgroup; every thread gets the result
__device__ double bsum(double v, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wsum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

// ---------------------------------------------------------------------------------------------
// Exact dgeqp3 (+ dorgqr) emulation. W: column-major m x n (column j at W + j*m), overwritten by the
// Householder vectors / R. Q: m x kmax output (row-major, ld kmax). Outputs rank per the reference's
// rule with R_00's sign taken from dlarfg. jpvt (0-based) and tau in scratch.
__global__ void __launch_bounds__(1024) k_qrcp(double* __restrict__ W, int m, int n, double* __restrict__ vn1,
                                                double* __restrict__ vn2, int* __restrict__ jpvt, double* __restrict__ tau,
                                                double* __restrict__ Q, double* __restrict__ Cout, int* __restrict__ rank_out,
                                                int pivot, int abs_r00, int rank_rule) {
    __shared__ double red[16];
    __shared__ double sh_beta, sh_tau, sh_scale;
    __shared__ int sh_p;
    __shared__ double sh_val[16];
    __shared__ int sh_idx[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kmax = min(m, n);
    const double tol3z = sqrt(1.1102230246251565e-16);  // sqrt(dlamch('Epsilon'))
    // initial column norms (one wave per column)
    for (int j = wave; j < n; j += 16) {
        const double* col = W + size_t(j) * m;
        double s = 0.0;
        for (int i = lane; i < m; i += 64) s += col[i] * col[i];
        s = wsum(s);
        if (lane == 0) {
            vn1[j] = sqrt(s);
            vn2[j] = vn1[j];
            jpvt[j] = j;
        }
    }
    __syncthreads();
    for (int k = 0; k < kmax; ++k) {
        // pivot: first index of max vn1[j], j >= k (IDAMAX)
        if (!pivot) {
            if (tid == 0) sh_p = k;
            __syncthreads();
        } else {
        double best = -1.0;
        int bi = n;
        for (int j = k + tid; j < n; j += 1024) {
            const double v = vn1[j];
            if (v > best || (v == best && j < bi)) { best = v; bi = j; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ov = __shfl_xor(best, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
        }
        if (lane == 0) { sh_val[wave] = best; sh_idx[wave] = bi; }
        __syncthreads();
        if (tid == 0) {
            double bv = -1.0;
            int b = n;
            for (int w = 0; w < 16; ++w)
                if (sh_val[w] > bv || (sh_val[w] == bv && sh_idx[w] < b)) { bv = sh_val[w]; b = sh_idx[w]; }
            sh_p = b;
        }
        __syncthreads();
        }
        const int p = (sh_p >= k && sh_p < n) ? sh_p : k;   // NaN norms never select an out-of-range column
        if (p != k) {
            double* ck = W + size_t(k) * m;
            double* cp = W + size_t(p) * m;
            for (int i = tid; i < m; i += 1024) {
                const double t = ck[i];
                ck[i] = cp[i];
                cp[i] = t;
            }
            __syncthreads();
            if (tid == 0) {
                const int t = jpvt[p]; jpvt[p] = jpvt[k]; jpvt[k] = t;
                vn1[p] = vn1[k];
                vn2[p] = vn2[k];
            }
        }
        __syncthreads();
        // dlarfg on column k rows k..m-1
        double* ck = W + size_t(k) * m;
        double s = 0.0;
        for (int i = k + 1 + tid; i < m; i += 1024) s += ck[i] * ck[i];
        const double xnorm = sqrt(bsum(s, red));
        if (tid == 0) {
            const double alpha = ck[k];
            if (m - k <= 1 || xnorm == 0.0) {
                sh_tau = 0.0;
                sh_beta = alpha;
            } else {
                const double beta = -copysign(hypot(alpha, xnorm), alpha);
                sh_tau = (beta - alpha) / beta;
                sh_beta = beta;
                sh_scale = 1.0 / (alpha - beta);
            }
        }
        __syncthreads();
        const double tk = sh_tau;
        if (tk != 0.0) {
            const double sc = sh_scale;
            for (int i = k + 1 + tid; i < m; i += 1024) ck[i] *= sc;
        }
        __syncthreads();
        if (tid == 0) {
            ck[k] = sh_beta;
            tau[k] = tk;
        }
        __syncthreads();
        // apply H = I - tau v v^T (v = [1, ck[k+1:]]) to columns j > k, one wave per column
        if (tk != 0.0) {
            for (int j = k + 1 + wave; j < n; j += 16) {
                double* cj = W + size_t(j) * m;
                double d = (lane == 0) ? cj[k] : 0.0;
                for (int i = k + 1 + lane; i < m; i += 64) d += ck[i] * cj[i];
                d = wsum(d) * tk;
                if (lane == 0) cj[k] -= d;
                for (int i = k + 1 + lane; i < m; i += 64) cj[i] -= d * ck[i];
            }
        }
        __syncthreads();
        // partial norm downdate (dlaqp2)
        for (int j = k + 1 + wave; j < n; j += 16) {
            const double v1 = vn1[j];
            if (v1 != 0.0) {
                const double* cj = W + size_t(j) * m;
                double temp = fabs(cj[k]) / v1;
                temp = fmax(0.0, 1.0 - temp * temp);
                const double r12 = v1 / vn2[j];
                const double temp2 = temp * r12 * r12;
                if (temp2 <= tol3z) {
                    double s2 = 0.0;
                    for (int i = k + 1 + lane; i < m; i += 64) s2 += cj[i] * cj[i];
                    s2 = wsum(s2);
                    if (lane == 0) {
                        const double nv = (k + 1 < m) ? sqrt(s2) : 0.0;
                        vn1[j] = nv;
                        vn2[j] = nv;
                    }
                } else if (lane == 0) {
                    vn1[j] = v1 * sqrt(temp);
                }
            }
        }
        __syncthreads();
    }
    // rank rule (blasLapackWrapper.cpp:268-272), R_00 NOT in abs
    __shared__ int sh_rank;
    if (tid == 0) {
        const double r00 = abs_r00 ? fabs(W[0]) : W[0];
        int rank = kmax;
        if (rank_rule) {
            for (rank = 1; rank <= kmax; ++rank) {
                if (rank == kmax || fabs(W[size_t(rank) * m + rank]) < 16.0 * 2.220446049250313e-16 * r00) break;
            }
        }
        sh_rank = rank;
        rank_out[0] = rank;
    }
    __syncthreads();
    const int rank = sh_rank;
    // C (rank x n, row-major): C[row][jpvt[col]] = R[row][col] for row <= col
    for (int e = tid; e < rank * n; e += 1024) {
        const int row = e / n, col = e % n;
        Cout[size_t(row) * n + jpvt[col]] = (row <= col) ? W[size_t(col) * m + row] : 0.0;
    }
    // Q = H_0 ... H_{kmax-1} [I; 0], m x kmax row-major (only the first `rank` columns are used)
    for (int e = tid; e < m * kmax; e += 1024) {
        const int i = e / kmax, j = e % kmax;
        Q[e] = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
    for (int i = kmax - 1; i >= 0; --i) {
        const double ti = tau[i];
        if (ti == 0.0) continue;
        const double* v = W + size_t(i) * m;
        for (int j = i + wave; j < kmax; j += 16) {
            double d = (lane == 0) ? Q[size_t(i) * kmax + j] : 0.0;
            for (int r = i + 1 + lane; r < m; r += 64) d += v[r] * Q[size_t(r) * kmax + j];
            d = wsum(d) * ti;
            if (lane == 0) Q[size_t(i) * kmax + j] -= d;
            for (int r = i + 1 + lane; r < m; r += 64) Q[size_t(r) * kmax + j] -= d * v[r];
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// One-sided Jacobi on the rows of W (p x q, row-major, p <= q). J (p x p) accumulates the
// rotations (J W_in = W_out with orthogonal rows). sweeps_out[0] = sweeps used (or -1 if not converged).
__global__ void __launch_bounds__(1024) k_jacobi(double* __restrict__ W, int p, int q, double* __restrict__ J,
                                                  int max_sweeps, double tol, int* __restrict__ sweeps_out) {
    __shared__ int rotated;
    __shared__ int perm[PMAX + 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = (p + 1) & ~1;  // even number of players (a dummy when p is odd)
    for (int e = tid; e < p * p; e += 1024) J[e] = ((e / p) == (e % p)) ? 1.0 : 0.0;
    for (int i = tid; i < P; i += 1024) perm[i] = i;
    __syncthreads();
    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        if (tid == 0) rotated = 0;
        __syncthreads();
        for (int round = 0; round < P - 1; ++round) {
            // pairs (perm[t], perm[P-1-t])
            for (int t = wave; t < P / 2; t += 16) {
                int i = perm[t], j = perm[P - 1 - t];
                if (i >= p || j >= p) continue;
                if (i > j) { const int s = i; i = j; j = s; }
                double* wi = W + size_t(i) * q;
                double* wj = W + size_t(j) * q;
                double a = 0, b = 0, c = 0;
                for (int k = lane; k < q; k += 64) {
                    const double x = wi[k], y = wj[k];
                    a += x * x; b += y * y; c += x * y;
                }
                a = wsum(a); b = wsum(b); c = wsum(c);
                if (fabs(c) > tol * sqrt(a * b) && c != 0.0) {
                    const double zeta = (b - a) / (2.0 * c);
                    const double t_ = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double cs = 1.0 / sqrt(1.0 + t_ * t_);
                    const double sn = cs * t_;
                    for (int k = lane; k < q; k += 64) {
                        const double x = wi[k], y = wj[k];
                        wi[k] = cs * x - sn * y;
                        wj[k] = sn * x + cs * y;
                    }
                    double* ji = J + size_t(i) * p;
                    double* jj = J + size_t(j) * p;
                    for (int k = lane; k < p; k += 64) {
                        const double x = ji[k], y = jj[k];
                        ji[k] = cs * x - sn * y;
                        jj[k] = sn * x + cs * y;
                    }
                    if (lane == 0) rotated = 1;
                }
            }
            __syncthreads();
            // rotate the tournament (player 0 fixed)
            if (tid == 0) {
                const int last = perm[P - 1];
                for (int s = P - 1; s > 1; --s) perm[s] = perm[s - 1];
                perm[1] = last;
            }
            __syncthreads();
        }
        if (!rotated) break;
    }
    if (tid == 0) sweeps_out[0] = (sweep < max_sweeps) ? sweep + 1 : -1;
}

// Finish of the Jacobi SVD: S = row norms of Wr, sorted descending; Vt rows = normalised rows; U[:, rank] = J[i, :].
__global__ void __launch_bounds__(1024) k_svd_finish(const double* __restrict__ Wr, int p, int q, const double* __restrict__ J,
                                                      double* __restrict__ U, double* __restrict__ S, double* __restrict__ Vt) {
    __shared__ double sn[PMAX];
    __shared__ int rk[PMAX];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = wave; i < p; i += 16) {
        const double* w = Wr + size_t(i) * q;
        double s = 0.0;
        for (int k = lane; k < q; k += 64) s += w[k] * w[k];
        s = wsum(s);
        if (lane == 0) sn[i] = sqrt(s);
    }
    __syncthreads();
    for (int i = tid; i < p; i += 1024) {
        int r = 0;
        const double si = sn[i];
        for (int j = 0; j < p; ++j) r += (sn[j] > si) || (sn[j] == si && j < i);
        rk[i] = r;
    }
    __syncthreads();
    for (int i = tid; i < p; i += 1024) S[rk[i]] = sn[i];
    for (int e = tid; e < p * q; e += 1024) {
        const int i = e / q, k = e % q;
        const double s = sn[i];
        Vt[size_t(rk[i]) * q + k] = (s > 0.0) ? Wr[e] / s : 0.0;
    }
    for (int e = tid; e < p * p; e += 1024) {
        const int i = e / p, r = e % p;   // U[r][rk[i]] = J[i][r]
        U[size_t(r) * p + rk[i]] = J[e];
    }
}

// ------------------------------------------------------------------------------------------------ launchers
void potrf(xrs_handle_t h, double* G, int n, double shift_rel, double* Dinv, int* status_dev, double* info_dev) {
    XRS_REQUIRE(n >= 1 && n <= PMAX, "potrf: n out of range for the single-workgroup kernel");
    KernelTimer timer(h, XRS_KFAM_QR, double(n) * n * n / 3.0, 16.0 * double(n) * n);
    hipLaunchKernelGGL(k_potrf, dim3(1), dim3(POT_THREADS), 0, h->stream, G, n, shift_rel, Dinv, status_dev, info_dev);
    check_launch("k_potrf");
}

void trsm(xrs_handle_t h, bool cols, const double* L, const double* Dinv, int n, const double* Y, size_t ldy, double* X,
          size_t ldx, int nvec) {
    if (nvec <= 0) return;
    XRS_REQUIRE(n >= 1 && n <= PMAX, "trsm: n out of range");
    KernelTimer timer(h, XRS_KFAM_QR, double(n) * n * nvec, 8.0 * (2.0 * double(n) * nvec + double(n) * n));
    const size_t lds = size_t(n) * (NB + 1) * sizeof(double);
    static bool attr_set = false;
    if (!attr_set) {
        XRS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_trsm<false>), hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024));
        XRS_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_trsm<true>), hipFuncAttributeMaxDynamicSharedMemorySize, 136 * 1024));
        attr_set = true;
    }
    const unsigned blocks = unsigned((nvec + NB - 1) / NB);
    if (cols)
        hipLaunchKernelGGL(k_trsm<true>, dim3(blocks), dim3(256), lds, h->stream, L, Dinv, n, Y, ldy, X, ldx, nvec);
    else
        hipLaunchKernelGGL(k_trsm<false>, dim3(blocks), dim3(256), lds, h->stream, L, Dinv, n, Y, ldy, X, ldx, nvec);
    check_launch("k_trsm");
}

size_t qrcp(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* C, bool pivot, bool abs_r00,
            bool rank_rule) {
    XRS_REQUIRE(m >= 1 && n >= 1, "qrcp: empty matrix");
    XRS_REQUIRE(m < (1u << 24) && n < (1u << 24), "qrcp: matrix too large");
    const size_t kmax = std::min(m, n);
    DevBuf W(h, m * n * 8), vn(h, 2 * n * 8), jp(h, n * 4 + 64), tau(h, kmax * 8), rk(h, 64);
    transpose(h, W.d(), A, m, n);  // column-major copy
    {
        KernelTimer timer(h, XRS_KFAM_QR, 4.0 * double(m) * n * kmax, 8.0 * 4.0 * double(m) * n);
        hipLaunchKernelGGL(k_qrcp, dim3(1), dim3(1024), 0, h->stream, W.d(), int(m), int(n), vn.d(), vn.d() + n, jp.as<int>(),
                           tau.d(), Q, C, rk.as<int>(), int(pivot), int(abs_r00), int(rank_rule));
        check_launch("k_qrcp");
    }
    int r = 0;
    read_status(h, rk.as<int>(), 1, &r);
    return size_t(r);
}

void jacobi_svd_rows(xrs_handle_t h, const double* W, int p, int q, double* U, double* S, double* Vt) {
    XRS_REQUIRE(p >= 1 && p <= PMAX && p <= q, "jacobi_svd_rows: need 1 <= p <= min(q, 512)");
    DevBuf Wc(h, size_t(p) * q * 8), J(h, size_t(p) * p * 8), st(h, 64);
    XRS_HIP(hipMemcpyAsync(Wc.d(), W, size_t(p) * q * 8, hipMemcpyDeviceToDevice, h->stream));
    {
        KernelTimer timer(h, XRS_KFAM_SVD, 8.0 * double(p) * p * (p + q), 0.0);
        hipLaunchKernelGGL(k_jacobi, dim3(1), dim3(1024), 0, h->stream, Wc.d(), p, q, J.d(), 60, 4.0 * 2.220446049250313e-16,
                           st.as<int>());
        check_launch("k_jacobi");
        hipLaunchKernelGGL(k_svd_finish, dim3(1), dim3(1024), 0, h->stream, Wc.d(), p, q, J.d(), U, S, Vt);
        check_launch("k_svd_finish");
    }
}

}  // namespace xrs
