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

#include <cstdio>

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
__device__ __forceinline__ void potrf32_body(double* __restrict__ G, int n, double shift_rel, double* __restrict__ Dinv,
                                             int* __restrict__ status, double* __restrict__ info,
                                             const double* src = nullptr) {
    __shared__ double P[PMAX * (NB + 1)];
    __shared__ double Ds[NB][NB + 1];
    __shared__ double red[16];
    __shared__ int fail;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (src != nullptr && src != G) {   // out of place: this workgroup copies, then factors G in place
        for (int e = tid; e < n * n; e += POT_THREADS) G[e] = src[e];
        __syncthreads();
    }
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

__global__ void __launch_bounds__(POT_THREADS) k_potrf(double* __restrict__ G, int n, double shift_rel, double* __restrict__ Dinv,
                                                 int* __restrict__ status, double* __restrict__ info) {
    potrf32_body(G, n, shift_rel, Dinv, status, info);
}

// ---------------------------------------------------------------------------------------------
// Register-resident Cholesky for n <= 256, one workgroup of 8 waves. The lower triangle of G lives
// in the MFMA accumulator layout of 16x16 tiles (tile t of the column-major lower enumeration
// belongs to wave t % 8, slot t / 8; <= 17 tiles = 136 VGPRs per lane), so the right-looking sweep
// never touches HBM/L2 between the initial load and the final store. Per 16-column block j:
//   (A) the owner of tile (j,j) publishes it to LDS;
//   (B) wave 0 factors it in registers (lane r owns row r of the symmetric Schur complement, so
//       column k of L is lane k's row: v_readlane broadcasts, rsqrt + Newton) and inverts it
//       (lane c forward-substitutes column c); the inverse also goes to Dinv for the TRSM;
//   (C) owners of the panel tiles form L_ij = G_ij L_jj^{-T} with 4 fp64 MFMAs and publish them;
//   (D) every wave applies G_ik -= L_ij L_kj^T to its trailing tiles (4 MFMAs per tile).
constexpr int PR_THREADS = 512;
constexpr int PR_WAVES = PR_THREADS / 64;
constexpr int PR_TMAX = 16;
constexpr int PR_SLOTS = (PR_TMAX * (PR_TMAX + 1) / 2 + PR_WAVES - 1) / PR_WAVES;
constexpr int PT = 17;           // LDS row stride of a 16x16 tile (conflict-free MFMA operand reads)
constexpr int PTILE = 16 * PT;

__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = fma(-x * y, y, 1.0);   // 1 - x y^2
        y = fma(0.5 * y, e, y);
    }
    return y;
}

// Wave-level ordering of LDS traffic between lanes of one wave (LDS executes a wave's ops in order).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifdef XRS_POTRF_STAMPS
__device__ long long* g_potrf_stamps;
#define PSTAMP(i) do { if (threadIdx.x == 0) g_potrf_stamps[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define PSTAMP(i) do { } while (0)
#endif
// Broadcast lane k of every 16-lane row to the whole row (DPP row_newbcast, gfx90a+): one VALU op per
// dword, no SGPR round trip.
template <int K>
__device__ __forceinline__ double row_bcast_d(double v) {
    union { double d; int i[2]; } u;
    u.d = v;
    u.i[0] = __builtin_amdgcn_mov_dpp(u.i[0], 0x150 + K, 0xF, 0xF, false);   // (every lane has a source:
    u.i[1] = __builtin_amdgcn_mov_dpp(u.i[1], 0x150 + K, 0xF, 0xF, false);   //  no zero-initialised "old")
    return u.d;
}

// One elimination step of the 16x16 diagonal block, LDL^T form so that the pivot dependency chain is
// only bcast -> rcp (+2 Newton) -> multiplier -> next pivot update. Lane r of every 16-lane row keeps
// row r of the symmetric Schur complement (a[l], all 16 columns, redundantly per row group) and 4
// columns (g + 4t, g = row group) of W = unit-L^{-1}, built by applying the same row operations to I.
template <int K>
__device__ __forceinline__ void factor_step(double (&a)[16], double (&w)[4], double* dsh, int lane, int valid, int& bad) {
    const double dkk = row_bcast_d<K>(a[K]);
    if (!((dkk > 0.0) && (dkk < 1.0e300)) && bad == 0 && K < valid) bad = K + 1;   // off the chain
    if (lane == 0) dsh[K] = dkk;
    double r = __builtin_amdgcn_rcp(dkk);
    r = fma(r, fma(-dkk, r, 1.0), r);
    r = fma(r, fma(-dkk, r, 1.0), r);
    const double m = a[K] * r;                              // S_rK / S_KK
#pragma unroll
    for (int l = K + 1; l < 16; ++l) a[l] = fma(-m, row_bcast_d<K>(a[l]), a[l]);
    const double mm = ((lane & 15) > K) ? m : 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) w[t] = fma(-mm, row_bcast_d<K>(w[t]), w[t]);
}

template <int K>
__device__ __forceinline__ void factor_all(double (&a)[16], double (&w)[4], double* dsh, int lane, int valid, int& bad) {
    if constexpr (K < 16) {
        factor_step<K>(a, w, dsh, lane, valid, bad);
        factor_all<K + 1>(a, w, dsh, lane, valid, bad);
    }
}

// (B): factor the 16x16 tile in Dt (full symmetric), leave L_jj (lower, zero upper) in Dt and
// L_jj^{-1} in Di and dinv_out (row-major 16x16). Returns 1 + first failing local column or 0.
// With d_c the pivots and a[c] the eliminated column values: L_rc = a[c] / sqrt(d_c) (c <= r) and
// L^{-1}_rc = W_rc / sqrt(d_r).
__device__ __forceinline__ int diag_factor16(double* Dt, double* Di, double* dsh, double* __restrict__ dinv_out,
                                             int lane, int valid) {
    const int r = lane & 15, g = lane >> 4;
    double a[16], w[4];
#pragma unroll
    for (int c = 0; c < 16; ++c) a[c] = Dt[r * PT + c];
#pragma unroll
    for (int t = 0; t < 4; ++t) w[t] = (g + 4 * t == r) ? 1.0 : 0.0;
    int bad = 0;
    factor_all<0>(a, w, dsh, lane, valid, bad);
    wave_lds_sync();
#ifdef XRS_POTRF_STAMPS
    if (lane == 0) g_potrf_stamps[1000 + blockIdx.x] = __builtin_amdgcn_s_memtime();
#endif
    if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) Dt[r * PT + c] = (c <= r) ? a[c] : 0.0;   // unscaled, rescaled below
    }
    const double rsr = rsqrt_nr(dsh[r]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const double v = w[t] * rsr;
        Di[r * PT + g + 4 * t] = v;
        dinv_out[r * 16 + g + 4 * t] = v;
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // element (row, col) = (lane >> 2, 4 (lane & 3) + e)
        const int rr = lane >> 2, cc = 4 * (lane & 3) + e;
        if (cc <= rr) Dt[rr * PT + cc] *= rsqrt_nr(dsh[cc]);
    }
    wave_lds_sync();
    return bad;
}

// (D) for a pair of slots (P, P-1): tiles (i,k) with k > j get G_ik -= L_ij L_kj^T. Slots are ordered by
// column, so the active ones are a suffix; the pair's operands are loaded together and the two MFMA
// chains interleaved (slot P-1 inactive -> zero operands, exact no-op on its accumulator).
template <int P>
__device__ __forceinline__ void trail_pair(d4 (&acc)[PR_SLOTS], const int (&ti)[PR_SLOTS], const int (&tk)[PR_SLOTS], int j,
                                           const double* Pbuf, int oa) {
    // slot P may be a padding slot (tk = -1) above an active slot P-1: test both
    const bool hi = tk[P] > j;
    bool lo = false;
    if constexpr (P > 0) lo = tk[P - 1] > j;
    if (!hi && !lo) return;
    auto op = [&](int tile, int c) -> double {
        return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(Pbuf + max(tile, 0) * PTILE) + oa + 32 * c);
    };
    double a1[4], b1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        a1[c] = hi ? -op(ti[P], c) : 0.0;
        b1[c] = hi ? op(tk[P], c) : 0.0;
    }
    if constexpr (P > 0) {
        double a0[4], b0[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = lo ? -op(ti[P - 1], c) : 0.0;
            b0[c] = lo ? op(tk[P - 1], c) : 0.0;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc[P] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[c], b1[c], acc[P], 0, 0, 0);
            acc[P - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[c], b0[c], acc[P - 1], 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[P] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[c], b1[c], acc[P], 0, 0, 0);
    }
}

template <int P>
__device__ __forceinline__ void trail_all(d4 (&acc)[PR_SLOTS], const int (&ti)[PR_SLOTS], const int (&tk)[PR_SLOTS], int j,
                                          const double* Pbuf, int oa) {
    if constexpr (P >= 0) {
        trail_pair<P>(acc, ti, tk, j, Pbuf, oa);
        trail_all<P - 2>(acc, ti, tk, j, Pbuf, oa);
    }
}

__device__ __forceinline__ void potrf_rr_body(double* __restrict__ G, int n, double shift_rel, double* __restrict__ Dinv,
                                              int* __restrict__ status, double* __restrict__ info,
                                              const double* __restrict__ src = nullptr) {
    const double* __restrict__ S = src != nullptr ? src : G;   // read from S, L to G (if G is given)
    __shared__ double Dt[PTILE];
    __shared__ double Di[PTILE];
    __shared__ double P[PR_TMAX * PTILE];
    __shared__ double ivs[16];
    __shared__ double red[PR_WAVES];
    __shared__ int fail;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lg = lane >> 4;
    const int T = (n + 15) >> 4;
    const int ntiles = T * (T + 1) / 2;
    if (tid == 0) fail = 0;
    PSTAMP(0);
    double tr = 0.0;
    for (int i = tid; i < n; i += PR_THREADS) tr += S[size_t(i) * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
    if (lane == 0) red[wave] = tr;
    __syncthreads();
    tr = 0.0;
#pragma unroll
    for (int w = 0; w < PR_WAVES; ++w) tr += red[w];
    if (tid == 0 && info) info[0] = tr;
    const double shift = shift_rel * tr;

    // tile ownership + load (identity padding beyond n)
    int ti[PR_SLOTS], tk[PR_SLOTS];
    d4 acc[PR_SLOTS];
#pragma unroll
    for (int s = 0; s < PR_SLOTS; ++s) {
        const int t = s * PR_WAVES + wave;
        int i = -1, k = -1;
        if (t < ntiles) {
            int start = 0;
            k = 0;
            while (t >= start + (T - k)) { start += T - k; ++k; }
            i = k + (t - start);
        }
        ti[s] = i;
        tk[s] = k;
        // unconditional loads from clamped addresses (no load-dependent arithmetic under a branch, so
        // all 4*PR_SLOTS loads are in flight together); padding / shift fixed up below
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = min(max(16 * i + lg + 4 * q, 0), n - 1), col = min(max(16 * k + lr, 0), n - 1);
            acc[s][q] = S[size_t(row) * n + col];
        }
    }
#pragma unroll
    for (int s = 0; s < PR_SLOTS; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * ti[s] + lg + 4 * q, col = 16 * tk[s] + lr;
            const bool inside = ti[s] >= 0 && row < n && col < n;
            const double pad = (row == col) ? 1.0 : 0.0;
            acc[s][q] = inside ? acc[s][q] + ((row == col) ? shift : 0.0) : pad;
        }

    for (int j = 0; j < T; ++j) {
        // lane offsets made opaque per iteration: otherwise LICM hoists one LDS address per slot out of
        // the j loop and the 17 accumulator tiles spill
        int oc = (lg * PT + lr) * 8, oa = (lr * PT + lg) * 8;
        asm volatile("" : "+v"(oc), "+v"(oa));
        auto cpos = [&](double* base, int q) -> double* {   // C layout (row lg + 4q, col lr)
            return reinterpret_cast<double*>(reinterpret_cast<char*>(base) + oc) + 4 * q * PT;
        };
        auto apos = [&](const double* base, int c) -> const double* {   // A/B operand (row lr, k 4c + lg)
            return reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + oa) + 4 * c;
        };
        // (A)
#pragma unroll
        for (int s = 0; s < PR_SLOTS; ++s)
            if (ti[s] == j && tk[s] == j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) *cpos(Dt, q) = acc[s][q];
            }
        __syncthreads();
        PSTAMP(2 + 4 * j);
        // (B)
        if (wave == 0) {
            const int bad = diag_factor16(Dt, Di, ivs, Dinv + size_t(j) * 256, lane, n - 16 * j);
            if (lane == 0 && bad && fail == 0) fail = 16 * j + bad;
        }
        __syncthreads();
        PSTAMP(3 + 4 * j);
        // (C)
#pragma unroll
        for (int s = 0; s < PR_SLOTS; ++s) {
            if (tk[s] != j) continue;
            if (ti[s] == j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[s][q] = *cpos(Dt, q);
                continue;
            }
            double* Pi = P + ti[s] * PTILE;
#pragma unroll
            for (int q = 0; q < 4; ++q) *cpos(Pi, q) = acc[s][q];
            wave_lds_sync();
            d4 rr = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 4; ++c) rr = __builtin_amdgcn_mfma_f64_16x16x4f64(*apos(Pi, c), *apos(Di, c), rr, 0, 0, 0);
            wave_lds_sync();
#pragma unroll
            for (int q = 0; q < 4; ++q) *cpos(Pi, q) = rr[q];
            acc[s] = rr;
        }
        __syncthreads();
        PSTAMP(4 + 4 * j);
        // (D)
        trail_all<PR_SLOTS - 1>(acc, ti, tk, j, P, oa);
    }
    __syncthreads();
    PSTAMP(1);
    // store L (lower) and zero the mirrored upper tiles (opaque lane indices: stops the compiler from
    // keeping every tile's global addresses live from the initial load)
    int sg = lg, sr = lr;
    asm volatile("" : "+v"(sg), "+v"(sr));
#pragma unroll
    for (int s = 0; s < PR_SLOTS; ++s) {
        if (ti[s] < 0 || G == nullptr) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * ti[s] + sg + 4 * q, col = 16 * tk[s] + sr;
            if (row < n && col < n) {
                G[size_t(row) * n + col] = (col <= row) ? acc[s][q] : 0.0;
                if (ti[s] != tk[s]) G[size_t(col) * n + row] = 0.0;
            }
        }
    }
    __syncthreads();
    if (tid == 0) status[0] = fail;
}

// ---------------------------------------------------------------------------------------------
// Lookahead variant of the register-resident Cholesky (n <= 256). Wave 0 factors the diagonal blocks
// and owns only the tiles of the first column (plus (1,1)), which receive no trailing update after
// step 0; the other tiles live on waves 1..7 (17 slots each, the plain kernel's register footprint).
// Step j:
//   (C_j)  owners of the panel tiles (i, j) form L_ij = G_ij L_jj^{-T} and publish them;
//   (D1_j) owners of column j+1 apply the rank-16 update of panel j to it; the owner of (j+1, j+1)
//          publishes it;
//   (B_{j+1} || D2_j) wave 0 factors block j+1 while waves 1..7 update the rest of the trailing matrix.
// The diagonal chain (42 % of the plain kernel) thus runs beside the trailing update.
constexpr int LA_THREADS = PR_THREADS;
constexpr int LA_WAVES = LA_THREADS / 64;
constexpr int LA_SLOTS = PR_SLOTS;   // wave 0: tiles 0..16 (column 0 and tile (1,1), final after step 0);
                                     // waves 1..7: tile 17 + 7 s + (wave - 1)

// slots P, P-1 with kmin <= tk <= kmax: G_ik -= L_ij L_kj^T (interleaved MFMA chains; inactive -> no-op)
template <int P>
__device__ __forceinline__ void la_trail_pair(d4 (&acc)[LA_SLOTS], const int (&ti)[LA_SLOTS], const int (&tk)[LA_SLOTS],
                                              int kmin, int kmax, const double* Pbuf, int oa) {
    const bool hi = tk[P] >= kmin && tk[P] <= kmax;
    bool lo = false;
    if constexpr (P > 0) lo = tk[P - 1] >= kmin && tk[P - 1] <= kmax;
    if (!hi && !lo) return;
    auto op = [&](int tile, int c) -> double {
        return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(Pbuf + max(tile, 0) * PTILE) + oa + 32 * c);
    };
    double a1[4], b1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        a1[c] = hi ? -op(ti[P], c) : 0.0;
        b1[c] = hi ? op(tk[P], c) : 0.0;
    }
    if constexpr (P > 0) {
        double a0[4], b0[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = lo ? -op(ti[P - 1], c) : 0.0;
            b0[c] = lo ? op(tk[P - 1], c) : 0.0;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc[P] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[c], b1[c], acc[P], 0, 0, 0);
            acc[P - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[c], b0[c], acc[P - 1], 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[P] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[c], b1[c], acc[P], 0, 0, 0);
    }
}

template <int P>
__device__ __forceinline__ void la_trail_all(d4 (&acc)[LA_SLOTS], const int (&ti)[LA_SLOTS], const int (&tk)[LA_SLOTS],
                                             int kmin, int kmax, const double* Pbuf, int oa) {
    if constexpr (P >= 0) {
        la_trail_pair<P>(acc, ti, tk, kmin, kmax, Pbuf, oa);
        la_trail_all<P - 2>(acc, ti, tk, kmin, kmax, Pbuf, oa);
    }
}

__device__ __forceinline__ void potrf_la_body(double* __restrict__ G, int n, double shift_rel, double* __restrict__ Dinv,
                                              int* __restrict__ status, double* __restrict__ info,
                                              const double* __restrict__ src = nullptr) {
    const double* __restrict__ S = src != nullptr ? src : G;
    __shared__ double Dt[PTILE];
    __shared__ double Di[PTILE];
    __shared__ double P[PR_TMAX * PTILE];
    __shared__ double ivs[16];
    __shared__ double red[LA_WAVES];
    __shared__ int fail;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lg = lane >> 4;
    const int T = (n + 15) >> 4;
    const int ntiles = T * (T + 1) / 2;
    if (tid == 0) fail = 0;
    PSTAMP(0);
    double tr = 0.0;
    for (int i = tid; i < n; i += LA_THREADS) tr += S[size_t(i) * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
    if (lane == 0) red[wave] = tr;
    __syncthreads();
    tr = 0.0;
#pragma unroll
    for (int w = 0; w < LA_WAVES; ++w) tr += red[w];
    if (tid == 0 && info) info[0] = tr;
    const double shift = shift_rel * tr;

    // tile ownership + load (identity padding beyond n)
    int ti[LA_SLOTS], tk[LA_SLOTS];
    d4 acc[LA_SLOTS];
#pragma unroll
    for (int s = 0; s < LA_SLOTS; ++s) {
        const int t = wave == 0 ? s : LA_SLOTS + s * (LA_WAVES - 1) + (wave - 1);
        int i = -1, k = -1;
        if (t < ntiles) {
            int start = 0;
            k = 0;
            while (t >= start + (T - k)) { start += T - k; ++k; }
            i = k + (t - start);
        }
        ti[s] = i;
        tk[s] = k;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = min(max(16 * i + lg + 4 * q, 0), n - 1), col = min(max(16 * k + lr, 0), n - 1);
            acc[s][q] = S[size_t(row) * n + col];
        }
    }
#pragma unroll
    for (int s = 0; s < LA_SLOTS; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * ti[s] + lg + 4 * q, col = 16 * tk[s] + lr;
            const bool inside = ti[s] >= 0 && row < n && col < n;
            const double pad = (row == col) ? 1.0 : 0.0;
            acc[s][q] = inside ? acc[s][q] + ((row == col) ? shift : 0.0) : pad;
        }

    int oc = (lg * PT + lr) * 8, oa = (lr * PT + lg) * 8;
    auto cpos = [&](double* base, int q) -> double* {   // C layout (row lg + 4q, col lr)
        return reinterpret_cast<double*>(reinterpret_cast<char*>(base) + oc) + 4 * q * PT;
    };
    auto apos = [&](const double* base, int c) -> const double* {   // A/B operand (row lr, k 4c + lg)
        return reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + oa) + 4 * c;
    };
    auto publish_diag = [&](int j) {   // owner of (j, j) -> Dt
#pragma unroll
        for (int s = 0; s < LA_SLOTS; ++s)
            if (ti[s] == j && tk[s] == j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) *cpos(Dt, q) = acc[s][q];
            }
    };
    auto factor_diag = [&](int j) {   // wave 0: Dt -> L_jj (Dt), L_jj^{-1} (Di, Dinv)
        if (wave == 0) {
            const int bad = diag_factor16(Dt, Di, ivs, Dinv + size_t(j) * 256, lane, n - 16 * j);
            if (lane == 0 && bad && fail == 0) fail = 16 * j + bad;
        }
    };
    publish_diag(0);
    __syncthreads();
    factor_diag(0);
    __syncthreads();
    for (int j = 0; j < T; ++j) {
        // opaque lane offsets per iteration (keeps LICM from hoisting per-slot LDS addresses -> spills)
        asm volatile("" : "+v"(oc), "+v"(oa));
        PSTAMP(2 + 4 * j);
        // (C_j) panel
#pragma unroll
        for (int s = 0; s < LA_SLOTS; ++s) {
            if (tk[s] != j) continue;
            if (ti[s] == j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[s][q] = *cpos(Dt, q);
                continue;
            }
            double* Pi = P + ti[s] * PTILE;
#pragma unroll
            for (int q = 0; q < 4; ++q) *cpos(Pi, q) = acc[s][q];
            wave_lds_sync();
            d4 rr = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 4; ++c) rr = __builtin_amdgcn_mfma_f64_16x16x4f64(*apos(Pi, c), *apos(Di, c), rr, 0, 0, 0);
            wave_lds_sync();
#pragma unroll
            for (int q = 0; q < 4; ++q) *cpos(Pi, q) = rr[q];
            acc[s] = rr;
        }
        __syncthreads();
        if (j + 1 >= T) break;
        PSTAMP(3 + 4 * j);
        // (D1_j) column j+1 first, then publish the new diagonal block
        la_trail_all<LA_SLOTS - 1>(acc, ti, tk, j + 1, j + 1, P, oa);
        publish_diag(j + 1);
        __syncthreads();
        PSTAMP(4 + 4 * j);
        // (B_{j+1} || D2_j); wave 0 factors first, then updates whatever trailing tiles it owns (none
        // for n = 256 after step 0)
        if (wave == 0) factor_diag(j + 1);
        la_trail_all<LA_SLOTS - 1>(acc, ti, tk, j + 2, T - 1, P, oa);
        __syncthreads();
    }
    PSTAMP(1);
    int sg = lg, sr = lr;
    asm volatile("" : "+v"(sg), "+v"(sr));
#pragma unroll
    for (int s = 0; s < LA_SLOTS; ++s) {
        if (ti[s] < 0 || G == nullptr) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * ti[s] + sg + 4 * q, col = 16 * tk[s] + sr;
            if (row < n && col < n) {
                G[size_t(row) * n + col] = (col <= row) ? acc[s][q] : 0.0;
                if (ti[s] != tk[s]) G[size_t(col) * n + row] = 0.0;
            }
        }
    }
    __syncthreads();
    if (tid == 0) status[0] = fail;
}

// The lookahead body (n = 256: 150.6 vs 158.8 us per factorisation; n = 100: 64 vs 54 us — one kernel
// holding both bodies spills, so the lookahead one serves every n <= 256). -DXRS_POTRF_NO_LOOKAHEAD
// builds the plain body (A/B timing, tools/potrf_bench.hip).
#ifdef XRS_POTRF_NO_LOOKAHEAD
#define XRS_POTRF_RR_BODY potrf_rr_body
#else
#define XRS_POTRF_RR_BODY potrf_la_body
#endif
#define XRS_POTRF_RR_THREADS PR_THREADS
__global__ void __launch_bounds__(XRS_POTRF_RR_THREADS) k_potrf_rr(double* __restrict__ G, int n, double shift_rel,
                                                         double* __restrict__ Dinv, int* __restrict__ status,
                                                         double* __restrict__ info) {
    XRS_POTRF_RR_BODY(G, n, shift_rel, Dinv, status, info);
}

// Independent factorisations, one workgroup each (e.g. the Gram matrices of every TT edge).
__global__ void __launch_bounds__(POT_THREADS) k_potrf32_batched(PotrfBatch b) {
    const int i = blockIdx.x;
    potrf32_body(b.G[i], b.n[i], b.shift[i], b.Dinv[i], b.status + b.slot[i], nullptr, b.src[i]);
}

__global__ void __launch_bounds__(XRS_POTRF_RR_THREADS) k_potrf_rr_batched(PotrfBatch b) {
    const int i = blockIdx.x;
    XRS_POTRF_RR_BODY(b.G[i], b.n[i], b.shift[i], b.Dinv[i], b.status + b.slot[i], nullptr, b.src[i]);
}

// ---------------------------------------------------------------------------------------------
// Triangular solve X = L^{-1} Y, 16 right-hand sides per workgroup of 4 waves, fp64 MFMA.
// Block-row I: T_I = Y_I - sum_{J<I} L_IJ X_J with the J-sum split over the waves (J = wave mod 4;
// the wave keeps its X_J tiles in registers in the MFMA C layout, which is exactly the B-operand
// layout of the next products), partials reduced through LDS, then every wave forms
// X_I = Dinv_I T_I redundantly (no second barrier). L_IJ and Dinv_I are read from L2 one block-row
// ahead (register prefetch). Dinv: 16x16 diagonal-block inverses; dld = 16 (k_potrf_rr layout,
// block J at Dinv + 256 J) or 32 (k_potrf layout: the 16x16 diagonal sub-blocks of the 32x32 block
// inverses are the 16-block inverses).
// RHS vectors v0 .. v0+15 of X = L^{-1} Y; ident: Y = I (n x n, COLS), i.e. 16 columns of L^{-1}.
template <bool COLS, int TMAX>
__device__ __forceinline__ void trsm16_body(const double* __restrict__ L, const double* __restrict__ Dinv, int dld,
                                            int n, const double* __restrict__ Y, size_t ldy, double* __restrict__ X,
                                            size_t ldx, int nvec, int v0, bool ident) {
    constexpr int JS = TMAX / 4;
    __shared__ double Xs[TMAX * 16 * PT];
    __shared__ double red[2][4][256];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 15, lg = lane >> 4;
    const int T = (n + 15) >> 4;
    const int np = T * 16;
    for (int e = tid; e < np * 16; e += 256) {
        int i, v;
        if (COLS) { i = e >> 4; v = e & 15; } else { v = e / np; i = e - v * np; }
        double y = 0.0;
        if (i < n && v0 + v < nvec) {
            if (ident) y = (i == v0 + v) ? 1.0 : 0.0;
            else y = COLS ? Y[size_t(i) * ldy + v0 + v] : Y[size_t(v0 + v) * ldy + i];
        }
        Xs[i * PT + v] = y;
    }
    auto dinv_at = [&](int I, int c) -> double {
        const int off = (dld == 32) ? 16 * (I & 1) : 0;
        return Dinv[size_t(16 * I + lr) * dld + off + 4 * c + lg];
    };
    d4 xr[JS];
    double la[JS][4], lb[JS][4], da[4], db[4];
#pragma unroll
    for (int js = 0; js < JS; ++js) {
        xr[js] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < 4; ++c) la[js][c] = 0.0;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) da[c] = dinv_at(0, c);
    __syncthreads();
    for (int I = 0; I < T; ++I) {
        if (I + 1 < T) {   // prefetch block-row I+1
            const int row = 16 * (I + 1) + lr;
#pragma unroll
            for (int js = 0; js < JS; ++js) {
                const int J = wave + 4 * js;
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    lb[js][c] = (J <= I && row < n) ? L[size_t(row) * n + 16 * J + 4 * c + lg] : 0.0;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) db[c] = dinv_at(I + 1, c);
        }
        d4 y;
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = Xs[(16 * I + lg + 4 * q) * PT + lr];
        // one accumulator per J tile: independent MFMA chains (a single chain is latency-bound)
        d4 accj[JS];
#pragma unroll
        for (int js = 0; js < JS; ++js) {
            accj[js] = d4{0.0, 0.0, 0.0, 0.0};
            if (wave + 4 * js >= I) continue;
#pragma unroll
            for (int c = 0; c < 4; ++c) accj[js] = __builtin_amdgcn_mfma_f64_16x16x4f64(la[js][c], xr[js][c], accj[js], 0, 0, 0);
        }
        d4 acc = accj[0];
#pragma unroll
        for (int js = 1; js < JS; ++js) acc += accj[js];
        double* rb = red[I & 1][0];
#pragma unroll
        for (int q = 0; q < 4; ++q) rb[wave * 256 + q * 64 + lane] = acc[q];
        __syncthreads();
        d4 t;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            t[q] = y[q] - ((rb[q * 64 + lane] + rb[256 + q * 64 + lane]) + (rb[512 + q * 64 + lane] + rb[768 + q * 64 + lane]));
        d4 x0 = {0.0, 0.0, 0.0, 0.0}, x1 = {0.0, 0.0, 0.0, 0.0};
        x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(da[0], t[0], x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(da[1], t[1], x1, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(da[2], t[2], x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(da[3], t[3], x1, 0, 0, 0);
        const d4 x = x0 + x1;
        if ((I & 3) == wave) {
#pragma unroll
            for (int js = 0; js < JS; ++js)
                if (js == (I >> 2)) xr[js] = x;
#pragma unroll
            for (int q = 0; q < 4; ++q) Xs[(16 * I + lg + 4 * q) * PT + lr] = x[q];
        }
#pragma unroll
        for (int js = 0; js < JS; ++js)
#pragma unroll
            for (int c = 0; c < 4; ++c) la[js][c] = lb[js][c];
#pragma unroll
        for (int c = 0; c < 4; ++c) da[c] = db[c];
    }
    __syncthreads();
    for (int e = tid; e < np * 16; e += 256) {
        int i, v;
        if (COLS) { i = e >> 4; v = e & 15; } else { v = e / np; i = e - v * np; }
        if (i < n && v0 + v < nvec) {
            const double x = (ident && i < v0 + v) ? 0.0 : Xs[i * PT + v];   // L^{-1}: exact zero upper triangle
            if (COLS) X[size_t(i) * ldx + v0 + v] = x;
            else X[size_t(v0 + v) * ldx + i] = x;
        }
    }
}

template <bool COLS, int TMAX>
__global__ void __launch_bounds__(256) k_trsm16(const double* __restrict__ L, const double* __restrict__ Dinv, int dld,
                                                int n, const double* __restrict__ Y, size_t ldy, double* __restrict__ X,
                                                size_t ldx, int nvec) {
    trsm16_body<COLS, TMAX>(L, Dinv, dld, n, Y, ldy, X, ldx, nvec, int(blockIdx.x) * 16, false);
}

// Batched triangular inverses X_i = L_i^{-1} (n_i x n_i, lower; blockIdx.y = matrix, blockIdx.x = 16 columns)
template <int TMAX>
__global__ void __launch_bounds__(256) k_trinv_batched(const TrinvBatch b, int dld) {
    const int i = blockIdx.y, n = b.n[i];
    if (int(blockIdx.x) * 16 >= n) return;
    trsm16_body<true, TMAX>(b.L[i], b.Dinv[i], dld, n, nullptr, 0, b.X[i], size_t(n), n, int(blockIdx.x) * 16, true);
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
                    // Rutishauser's form x' = x - s (y + tau x), y' = y + s (x - tau y), tau = s / (1 + c):
                    // a nearly-identity rotation perturbs the rows by O(u s) instead of O(u), so the
                    // accumulated J stays orthogonal to working precision over thousands of rotations
                    const double tau = sn / (1.0 + cs);
                    for (int k = lane; k < q; k += 64) {
                        const double x = wi[k], y = wj[k];
                        wi[k] = x - sn * (y + tau * x);
                        wj[k] = y + sn * (x - tau * y);
                    }
                    double* ji = J + size_t(i) * p;
                    double* jj = J + size_t(j) * p;
                    for (int k = lane; k < p; k += 64) {
                        const double x = ji[k], y = jj[k];
                        ji[k] = x - sn * (y + tau * x);
                        jj[k] = y + sn * (x - tau * y);
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
// Dinv row stride: k_potrf_rr (n <= 256) writes 16x16 blocks, k_potrf 32x32 blocks.
static int dinv_ld(int n) { return n <= PR_TMAX * 16 ? 16 : 32; }
size_t dinv_elems(int n) { return dinv_ld(n) == 16 ? size_t((n + 15) / 16) * 256 : size_t(n + 32) * 32; }

void potrf(xrs_handle_t h, double* G, int n, double shift_rel, double* Dinv, int* status_dev, double* info_dev) {
    XRS_REQUIRE(n >= 1 && n <= PMAX, "potrf: n out of range for the single-workgroup kernel");
    KernelTimer timer(h, XRS_KFAM_QR, double(n) * n * n / 3.0, 16.0 * double(n) * n);
    if (dinv_ld(n) == 16) {
        hipLaunchKernelGGL(k_potrf_rr, dim3(1), dim3(XRS_POTRF_RR_THREADS), 0, h->stream, G, n, shift_rel, Dinv, status_dev, info_dev);
        check_launch("k_potrf_rr");
    } else {
        hipLaunchKernelGGL(k_potrf, dim3(1), dim3(POT_THREADS), 0, h->stream, G, n, shift_rel, Dinv, status_dev, info_dev);
        check_launch("k_potrf");
    }
}

void potrf_batched(xrs_handle_t h, const PotrfBatch& b, int count) {
    XRS_REQUIRE(count >= 0 && count <= kPotrfBatchMax, "potrf_batched: batch too large");
    if (count == 0) return;
    // n <= 256: register-resident kernel (16-block Dinv); larger (<= 512): 32-block kernel. One launch
    // per kind, each entry's Dinv layout matching dinv_ld(n) (what trsm() expects).
    PotrfBatch small{}, large{};
    int ns = 0, nl = 0;
    double fl_s = 0.0, fl_l = 0.0;
    for (int i = 0; i < count; ++i) {
        XRS_REQUIRE(b.n[i] >= 1 && b.n[i] <= PMAX, "potrf_batched: n out of range");
        const bool rr = dinv_ld(b.n[i]) == 16;
        PotrfBatch& d = rr ? small : large;
        int& c = rr ? ns : nl;
        XRS_REQUIRE(b.G[i] != nullptr || (rr && b.src[i] != nullptr), "potrf_batched: no input / output");
        d.src[c] = b.src[i];
        d.G[c] = b.G[i];
        d.Dinv[c] = b.Dinv[i];
        d.shift[c] = b.shift[i];
        d.n[c] = b.n[i];
        d.slot[c] = i;   // statuses land directly in the caller's order
        (rr ? fl_s : fl_l) += double(b.n[i]) * b.n[i] * b.n[i] / 3.0;
        ++c;
    }
    small.status = b.status;
    large.status = b.status;
    if (ns) {
        KernelTimer timer(h, XRS_KFAM_QR, fl_s, 0.0);
        hipLaunchKernelGGL(k_potrf_rr_batched, dim3(ns), dim3(XRS_POTRF_RR_THREADS), 0, h->stream, small);
        check_launch("k_potrf_rr_batched");
    }
    if (nl) {
        KernelTimer timer(h, XRS_KFAM_QR, fl_l, 0.0);
        hipLaunchKernelGGL(k_potrf32_batched, dim3(nl), dim3(POT_THREADS), 0, h->stream, large);
        check_launch("k_potrf32_batched");
    }
}

void trsm(xrs_handle_t h, bool cols, const double* L, const double* Dinv, int n, const double* Y, size_t ldy, double* X,
          size_t ldx, int nvec) {
    if (nvec <= 0) return;
    XRS_REQUIRE(n >= 1 && n <= PMAX, "trsm: n out of range");
    KernelTimer timer(h, XRS_KFAM_QR, double(n) * n * nvec, 8.0 * (2.0 * double(n) * nvec + double(n) * n));
    const unsigned blocks = unsigned((nvec + 15) / 16);
    const int dld = dinv_ld(n);
#define XRS_TRSM(C_, T_) \
    hipLaunchKernelGGL((k_trsm16<C_, T_>), dim3(blocks), dim3(256), 0, h->stream, L, Dinv, dld, n, Y, ldy, X, ldx, nvec)
    if (n <= 256) {
        if (cols) XRS_TRSM(true, 16); else XRS_TRSM(false, 16);
    } else {
        if (cols) XRS_TRSM(true, 32); else XRS_TRSM(false, 32);
    }
#undef XRS_TRSM
    check_launch("k_trsm16");
}

void trinv_batched(xrs_handle_t h, const TrinvBatch& b, int count) {
    XRS_REQUIRE(count >= 0 && count <= kTrinvBatchMax, "trinv_batched: batch too large");
    // one launch per Dinv layout (n <= 256: 16-blocks, else 32-blocks), as in potrf_batched
    for (int big = 0; big < 2; ++big) {
        TrinvBatch g{};
        int c = 0, nmax = 0;
        double fl = 0.0;
        for (int i = 0; i < count; ++i) {
            XRS_REQUIRE(b.n[i] >= 1 && b.n[i] <= PMAX, "trinv_batched: n out of range");
            if ((dinv_ld(b.n[i]) == 32) != bool(big)) continue;
            g.L[c] = b.L[i];
            g.Dinv[c] = b.Dinv[i];
            g.X[c] = b.X[i];
            g.n[c] = b.n[i];
            nmax = std::max(nmax, b.n[i]);
            fl += double(b.n[i]) * b.n[i] * b.n[i];
            ++c;
        }
        if (c == 0) continue;
        KernelTimer timer(h, XRS_KFAM_QR, fl, 0.0);
        const dim3 grid(unsigned((nmax + 15) / 16), unsigned(c));
        if (big) hipLaunchKernelGGL((k_trinv_batched<32>), grid, dim3(256), 0, h->stream, g, 32);
        else hipLaunchKernelGGL((k_trinv_batched<16>), grid, dim3(256), 0, h->stream, g, 16);
        check_launch("k_trinv_batched");
    }
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
    if (jacobi_usv_fits(p, q)) {
        // multi-workgroup block Jacobi with the rotations accumulated (svd.hip); non-convergence is a
        // warning, as the reference's dgesdd failure (blasLapackWrapper.cpp:216-224)
        DevBuf st(h, 64);
        jacobi_usv(h, W, q, false, p, q, U, p, S, Vt, q, st.as<int>(), 60);
        int sweeps = 0;
        read_status(h, st.as<int>(), 1, &sweeps);
        if (sweeps != -2) {
            if (sweeps < 0)
                std::fprintf(stderr, "[xerus_amd warning] SVD failed: one-sided Jacobi of a %d x %d matrix did not converge (status %d)\n",
                             p, q, sweeps);
            return;
        }
        // -2: a bounded grid-barrier poll timed out (a workgroup was not scheduled), so the multi-workgroup
        // result is not valid at all -- not a convergence failure: redo the SVD in one workgroup below
        std::fprintf(stderr, "[xerus_amd warning] multi-workgroup Jacobi barrier timed out (%d x %d); rerun in one workgroup\n", p, q);
    }
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
