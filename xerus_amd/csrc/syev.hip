// Top-kk eigenpairs of a symmetric n x n matrix (n <= 256) for the certified truncating round: the
// reference computes the edge's singular vectors with dgesdd (tensor.cpp:1424-1489); where the round has
// certified the edge Gram P = B B^T to be well conditioned and the kept rank kk is fixed in advance
// (tt_trunc.hip round_truncate), the kept left singular vectors of B are the eigenvectors of P's kk
// largest eigenvalues. Three launches, LAPACK's dsytrd / dstebz / dstein / dormtr structure:
//   1. k_sytrd: Householder tridiagonalisation A = Q T Q^T in ONE workgroup, the matrix register-resident
//      (n <= 128: 1024 threads on a 32 x 32 grid, element (i, k) on thread (i mod 32, k mod 32): the
//      shrinking trailing block stays spread over every thread; 129..256: k_sytrd_l512, 512 threads holding
//      the lower block triangle). Per column: the reflector from one wave, the symmetric matrix-vector
//      product with in-wave DPP / permlane reductions, the rank-2 update in registers -- LDS-only barriers.
//   2. k_stebz_stein: one wave per wanted eigenvalue (kk workgroups in parallel): Sturm-count
//      multisection on 64 points per round (~9 rounds to full precision), then inverse iteration with the
//      partially pivoted LU of T - lambda I (dgttrf / dgttrs), three solves from a fixed start vector.
//      Measured alternatives (profiles/r03/stein_variants_r03r.txt): a single twisted-factorisation solve
//      (orthogonality only 1e-12..1e-11 on flat spectra, T - lambda I not being a relatively robust
//      representation); 4 waves with 512 points per round and register-prefetched chains (6 instead of 9
//      rounds, same 105 us: every O(n) chain is bound by its ~20-cycle dependent FP64 latency per level).
//   3. k_ormtr: the eigenvectors back to A's coordinates, u = H_0 ... H_{n-2} z, one wave per vector
//      (64 lanes, 4 vectors per workgroup), the reflectors staged through LDS in chunks.
// Inverse iteration is accurate for eigenvalues separated relative to ||T|| (the certified rounds' random
// spectra); a cluster would give non-orthogonal vectors, which the round's final orthonormality check
// rejects (then the reference's algorithm runs).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "smallla.hpp"

namespace xrs {

namespace {

constexpr int SY_MAX = 256;
typedef double d4 __attribute__((ext_vector_type(4)));

// Cross-lane sums without the LDS crossbar (a __shfl_xor of a double is two ds_bpermute round trips, the
// bulk of a column step when chained): DPP row rotations within 16 lanes, v_permlane16_swap across the
// two rows of a 32-lane half, v_permlane32_swap across the halves.
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double xor16(double v) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    return (threadIdx.x & 16) ? __hiloint2double(hi[0], lo[0]) : __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double sum16(double v) {   // every lane of the 16-lane row gets the row's sum
    v += dpp<0x128>(v);
    v += dpp<0x124>(v);
    v += dpp<0x122>(v);
    v += dpp<0x121>(v);
    return v;
}
__device__ __forceinline__ double sum32(double v) { v = sum16(v); return v + xor16(v); }
__device__ __forceinline__ double xor32(double v) {   // the value of lane l ^ 32 (v_permlane32_swap)
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    return (threadIdx.x & 32) ? __hiloint2double(hi[0], lo[0]) : __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double sum64(double v) { v = sum32(v); return v + xor32(v); }

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global
// stores (__syncthreads' release fence would drain the per-column stores of the reflectors, d, e and tau
// to memory at every barrier of the column loop)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int NEWTON>
__device__ __forceinline__ double rcpn(double x) {   // 1/x: hardware estimate + NEWTON Newton steps
    double r = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int it = 0; it < NEWTON; ++it) r = fma(r, fma(-x, r, 1.0), r);
    return r;
}

__device__ __forceinline__ double rcp2(double x) {   // 1/x to ~1 ulp (hardware estimate + 2 Newton steps)
    double r = __builtin_amdgcn_rcp(x);
    double t = fma(-x, r, 1.0);
    r = fma(r, t, r);
    t = fma(-x, r, 1.0);
    return fma(r, t, r);
}

// LAPACK dsytd2 (lower) on the register grid (element (i, k) on thread (i mod GRID, k mod GRID)). V: row j = Householder vector v_j (v_j[i] = 0 for i <= j,
// v_j[j + 1] = 1); d (n), e (n - 1), tau (n - 1). A is read from its lower triangle.
// GRID x GRID threads (GRID = 32: 16 waves; GRID = 16: 4 waves, one per SIMD, NB x NB = 64 elements per
// thread at n = 128 -- fewer waves to wait for at every barrier and no SIMD shared between waves)
template <int GRID, int NB>
__global__ void __launch_bounds__(GRID * GRID) k_sytrd(const double* __restrict__ A, int lda, int n, double* __restrict__ d,
                                                double* __restrict__ e, double* __restrict__ tau, double* __restrict__ V,
                                                unsigned long long* __restrict__ stamps) {
    // diagnostics (stamps != null): threads 0 and 64 record s_memtime at 6 points of every column step
#define SYTRD_STAMP(p)                                                                                  \
    do {                                                                                                \
        if (stamps && (threadIdx.x == 0 || threadIdx.x == 64) && j < 64)                                 \
            stamps[(threadIdx.x == 0 ? 0 : 384) + 6 * j + (p)] = __builtin_amdgcn_s_memtime();           \
    } while (0)
    __shared__ double xs[SY_MAX], vs[SY_MAX], ps[SY_MAX];
    __shared__ double sh_tau;
    const int t = threadIdx.x, tr = t / GRID, tc = t % GRID, lane = t & 63, wave = t >> 6;
    constexpr int NP = GRID * NB;   // padded order
    double a[NB][NB];
#pragma unroll
    for (int ia = 0; ia < NB; ++ia)
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) {
            const int i = tr + GRID * ia, k = tc + GRID * ib;
            a[ia][ib] = (i < n && k < n) ? (i >= k ? A[size_t(i) * lda + k] : A[size_t(k) * lda + i]) : 0.0;
        }
    // column j of the current matrix to LDS (xs) and its diagonal entry to d, by the column's owners
    auto publish_column = [&](int j) {
        if (tc == (j % GRID)) {
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) {
                const int i = tr + GRID * ia;
#pragma unroll
                for (int ib = 0; ib < NB; ++ib)
                    if (ib == (j / GRID)) {
                        if (i > j && i < n) xs[i] = a[ia][ib];
                        if (i == j) d[j] = a[ia][ib];
                    }
            }
        }
    };
    publish_column(0);
    for (int j = 0; j + 2 < n; ++j) {
        SYTRD_STAMP(0);
        lds_barrier();
        SYTRD_STAMP(1);
        // (b) reflector (dlarfg): beta = -sign(alpha) ||(alpha, x)||, tau = (beta - alpha) / beta,
        //     v = (1, x / (alpha - beta))
        if (wave == 0) {
            constexpr int E = NP >= 64 ? NP / 64 : 1;   // entries per lane of the NP padded indices
            double x[E];
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = (lane + 64 * q < NP) ? xs[lane + 64 * q] : 0.0;
            const double alpha = xs[j + 1];
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int i = lane + 64 * q;
                if (i >= j + 2 && i < n) s = fma(x[q], x[q], s);
            }
            s = sum64(s);
            double tv = 0.0, beta = alpha, scal = 0.0;
            if (s > 0.0) {
                beta = -copysign(sqrt(fma(alpha, alpha, s)), alpha);
                tv = (beta - alpha) * rcp2(beta);
                scal = rcp2(alpha - beta);
            }
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int i = lane + 64 * q;
                const double v = (i <= j || i >= n) ? 0.0 : (i == j + 1 ? 1.0 : x[q] * scal);
                if (i < NP) vs[i] = v;
                if (i < n) V[size_t(j) * n + i] = v;
            }
            if (lane == 0) {
                sh_tau = tv;
                e[j] = beta;
                tau[j] = tv;
            }
        }
        SYTRD_STAMP(2);
        lds_barrier();
        SYTRD_STAMP(3);
        const double tj = sh_tau;   // (tau = 0: p = w = 0, the update leaves A unchanged; no second latch)
        // (c) p = tau A v on the trailing block: row partials (NB independent chains), reduced over the 32
        //     column threads of a row level by level across the rows (ILP in the DPP chain)
        {
            double part[NB], vcol[NB];
#pragma unroll
            for (int ib = 0; ib < NB; ++ib) vcol[ib] = vs[tc + GRID * ib];
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) {
                part[ia] = 0.0;
#pragma unroll
                for (int ib = 0; ib < NB; ++ib) part[ia] = fma(a[ia][ib], vcol[ib], part[ia]);
            }
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) part[ia] += dpp<0x128>(part[ia]);
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) part[ia] += dpp<0x124>(part[ia]);
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) part[ia] += dpp<0x122>(part[ia]);
#pragma unroll
            for (int ia = 0; ia < NB; ++ia) part[ia] += dpp<0x121>(part[ia]);
            if constexpr (GRID == 32) {
#pragma unroll
                for (int ia = 0; ia < NB; ++ia) part[ia] += xor16(part[ia]);
            }
            if (tc == 0) {
#pragma unroll
                for (int ia = 0; ia < NB; ++ia) {
                    const int i = tr + GRID * ia;
                    ps[i] = (i > j && i < n) ? tj * part[ia] : 0.0;
                }
            }
        }
        for (int q = NP + t; q < SY_MAX; q += GRID * GRID) ps[q] = 0.0;
        SYTRD_STAMP(4);
        lds_barrier();
        SYTRD_STAMP(5);
        // (d) every wave forms K = -(tau / 2) (p . v) itself (no extra barrier), w = p + K v on the fly;
        //     the update's operands are read before the reduction so their LDS latency overlaps it
        double vr[NB], pr[NB], vc[NB], pc[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            vr[q] = vs[tr + GRID * q];
            pr[q] = ps[tr + GRID * q];
            vc[q] = vs[tc + GRID * q];
            pc[q] = ps[tc + GRID * q];
        }
        double sk = 0.0;
#pragma unroll
        for (int i = lane; i < NP; i += 64) sk = fma(ps[i], vs[i], sk);
        const double K = -0.5 * tj * sum64(sk);
        // (e) A -= v w^T + w v^T (v, w vanish at indices <= j: finished rows and columns stay untouched), on
        //     the active blocks only: block rows / columns below (j + 1) / GRID are finished, so one
        //     compile-time loop nest per first active block (a switch, not per-block branches)
        auto update_from = [&](auto jb_c) {
            constexpr int JB = decltype(jb_c)::value;
#pragma unroll
            for (int ib = JB; ib < NB; ++ib) {
                const double wc = fma(K, vc[ib], pc[ib]);
#pragma unroll
                for (int ia = JB; ia < NB; ++ia) a[ia][ib] = fma(-vr[ia], wc, fma(-fma(K, vr[ia], pr[ia]), vc[ib], a[ia][ib]));
            }
        };
        switch ((j + 1) / GRID) {
            case 0: update_from(std::integral_constant<int, 0>{}); break;
            case 1: if constexpr (NB > 1) update_from(std::integral_constant<int, (NB > 1 ? 1 : 0)>{}); break;
            case 2: if constexpr (NB > 2) update_from(std::integral_constant<int, (NB > 2 ? 2 : 0)>{}); break;
            default: if constexpr (NB > 3) update_from(std::integral_constant<int, (NB > 3 ? 3 : 0)>{}); break;
        }
        publish_column(j + 1);
    }
#undef SYTRD_STAMP
    // the last 2 x 2 block: d[n-2], d[n-1], e[n-2] (tau = 0, H = I)
#pragma unroll
    for (int ia = 0; ia < NB; ++ia)
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) {
            const int i = tr + GRID * ia, k = tc + GRID * ib;
            if (n >= 2 && i == n - 2 && k == n - 2) d[n - 2] = a[ia][ib];
            if (n >= 1 && i == n - 1 && k == n - 1) d[n - 1] = a[ia][ib];
            if (n >= 2 && i == n - 1 && k == n - 2) {
                e[n - 2] = a[ia][ib];
                tau[n - 2] = 0.0;
                for (int q = 0; q < n; ++q) V[size_t(n - 2) * n + q] = 0.0;
            }
        }
}

// Orders 129..256: the same column steps on 512 threads (8 waves, two per SIMD: 256 VGPRs each) holding
// the lower triangle by blocks. Thread (tr, tc) = (t / 16, t % 16) of a 32 x 16 grid owns the elements
// (tr + 32 ia, tc + 16 ib) of the blocks with ib <= 2 ia + 1 (the ones meeting the lower triangle:
// 72 doubles); the entries above the diagonal in the two diagonal-crossing blocks of a block row stay zero.
// The symmetric product sums the rows of the stored entries (over the 16 column threads of a row: one DPP
// row) plus, for the mirrored upper triangle, the columns of the strictly lower ones (over the 4 rows of a
// wave by permlane16 / shuffle, then over the 8 waves through LDS). The column halves (ib < 8, ib >= 8) are
// processed one after the other to bound the live operand registers.
__global__ void __launch_bounds__(512) k_sytrd_l512(const double* __restrict__ A, int lda, int n, double* __restrict__ d,
                                                   double* __restrict__ e, double* __restrict__ tau, double* __restrict__ V) {
    constexpr int NR = 8, NW = 8, NP = 256;
    constexpr int NL = NR * (NR + 1);   // block row ia holds column blocks 0 .. 2 ia + 1: offset ia (ia + 1)
    __shared__ double xs[SY_MAX], vs[SY_MAX], ps[SY_MAX], psr[SY_MAX], cbuf[NW][SY_MAX];
    __shared__ double sh_tau;
    const int t = threadIdx.x, tr = t >> 4, tc = t & 15, lane = t & 63, wave = t >> 6;
    // diagonal-crossing blocks of block row ia: ib = 2 ia (i - k = tr - tc), ib = 2 ia + 1 (i - k = tr - tc - 16)
    const bool keep0 = tr >= tc, keep1 = tr >= tc + 16;   // on or below the diagonal
    const bool low0 = tr > tc, low1 = tr > tc + 16;       // strictly below
    double a[NL];
#pragma unroll
    for (int ia = 0; ia < NR; ++ia)
#pragma unroll
        for (int ib = 0; ib <= 2 * ia + 1; ++ib) {
            const int i = tr + 32 * ia, k = tc + 16 * ib;
            const bool keep = (ib < 2 * ia || (ib == 2 * ia ? keep0 : keep1)) && i < n && k < n;
            const double x = A[size_t(keep ? i : 0) * lda + (keep ? k : 0)];
            a[ia * (ia + 1) + ib] = keep ? x : 0.0;
        }
    // column jj of the current matrix to LDS (xs) and its diagonal entry to d, by the column's owners
#define L512_PUBLISH_CASE(IB)                                                             \
    case IB:                                                                              \
        _Pragma("unroll") for (int ia = (IB) / 2; ia < NR; ++ia) {                        \
            const int i = tr + 32 * ia;                                                   \
            const double av = a[ia * (ia + 1) + (IB)];                                    \
            if (i > pj && i < n) xs[i] = av;                                              \
            if (i == pj) d[pj] = av;                                                      \
        }                                                                                 \
        break;
#define L512_PUBLISH(jj)                                                                  \
    do {                                                                                  \
        const int pj = (jj);                                                              \
        if (tc == (pj & 15)) {                                                            \
            switch (pj >> 4) {                                                            \
                L512_PUBLISH_CASE(0) L512_PUBLISH_CASE(1) L512_PUBLISH_CASE(2)            \
                L512_PUBLISH_CASE(3) L512_PUBLISH_CASE(4) L512_PUBLISH_CASE(5)            \
                L512_PUBLISH_CASE(6) L512_PUBLISH_CASE(7) L512_PUBLISH_CASE(8)            \
                L512_PUBLISH_CASE(9) L512_PUBLISH_CASE(10) L512_PUBLISH_CASE(11)          \
                L512_PUBLISH_CASE(12) L512_PUBLISH_CASE(13) L512_PUBLISH_CASE(14)         \
                L512_PUBLISH_CASE(15)                                                     \
                default: break;                                                           \
            }                                                                             \
        }                                                                                 \
    } while (0)
    L512_PUBLISH(0);
    for (int j = 0; j + 2 < n; ++j) {
        lds_barrier();
        if (wave == 0) {   // reflector (dlarfg), as in k_sytrd
            constexpr int E = NP / 64;
            double x[E];
#pragma unroll
            for (int q = 0; q < E; ++q) x[q] = xs[lane + 64 * q];
            const double alpha = xs[j + 1];
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int i = lane + 64 * q;
                if (i >= j + 2 && i < n) s = fma(x[q], x[q], s);
            }
            s = sum64(s);
            double tv = 0.0, beta = alpha, scal = 0.0;
            if (s > 0.0) {
                beta = -copysign(sqrt(fma(alpha, alpha, s)), alpha);
                tv = (beta - alpha) * rcp2(beta);
                scal = rcp2(alpha - beta);
            }
#pragma unroll
            for (int q = 0; q < E; ++q) {
                const int i = lane + 64 * q;
                const double v = (i <= j || i >= n) ? 0.0 : (i == j + 1 ? 1.0 : x[q] * scal);
                vs[i] = v;
                if (i < n) V[size_t(j) * n + i] = v;
            }
            if (lane == 0) {
                sh_tau = tv;
                e[j] = beta;
                tau[j] = tv;
            }
        }
        lds_barrier();
        // (no early exit for tau = 0: p = w = 0 then and the update leaves every entry unchanged; a second
        // loop latch would double the live matrix registers at the merge)
        const double tj = sh_tau;
        // symmetric product: row sums of the stored entries, column sums of the strictly lower ones
        double rp[NR];
#pragma unroll
        for (int ia = 0; ia < NR; ++ia) rp[ia] = 0.0;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            double cp[8], vk[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                cp[q] = 0.0;
                vk[q] = vs[tc + 16 * (8 * hh + q)];
            }
#pragma unroll
            for (int ia = 0; ia < NR; ++ia) {
                __builtin_amdgcn_sched_barrier(0);
                const double vi = vs[tr + 32 * ia];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int ib = 8 * hh + q;
                    if (ib <= 2 * ia + 1) {
                        const double av = a[ia * (ia + 1) + ib];
                        rp[ia] = fma(av, vk[q], rp[ia]);
                        if (ib < 2 * ia) cp[q] = fma(av, vi, cp[q]);
                        else cp[q] = fma((ib == 2 * ia ? low0 : low1) ? av : 0.0, vi, cp[q]);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                cp[q] += xor16(cp[q]);
                cp[q] += xor32(cp[q]);
            }
            if (lane < 16) {
#pragma unroll
                for (int q = 0; q < 8; ++q) cbuf[wave][tc + 16 * (8 * hh + q)] = cp[q];
            }
        }
#pragma unroll
        for (int ia = 0; ia < NR; ++ia) {
            const double r = sum16(rp[ia]);
            if (tc == 0) psr[tr + 32 * ia] = r;
        }
        lds_barrier();
        if (t < SY_MAX) {
            double c = 0.0;
#pragma unroll
            for (int w = 0; w < NW; ++w) c += cbuf[w][t];
            ps[t] = (t > j && t < n) ? tj * (psr[t] + c) : 0.0;
        }
        lds_barrier();
        // K = -(tau / 2) (p . v) in every wave, w = p + K v on the fly; A -= v w^T + w v^T on the kept entries
        double sk = 0.0;
#pragma unroll
        for (int q = 0; q < NP / 64; ++q) sk = fma(ps[lane + 64 * q], vs[lane + 64 * q], sk);
        const double K = -0.5 * tj * sum64(sk);
        {
            double vi[NR], wi[NR];
#pragma unroll
            for (int ia = 0; ia < NR; ++ia) {
                vi[ia] = vs[tr + 32 * ia];
                wi[ia] = fma(K, vi[ia], ps[tr + 32 * ia]);
            }
#pragma unroll
            for (int ib = 0; ib < 16; ++ib) {
                __builtin_amdgcn_sched_barrier(0);   // one column block at a time (hoisted operands spill)
                const double vk = vs[tc + 16 * ib];
                const double wk = fma(K, vk, ps[tc + 16 * ib]);
#pragma unroll
                for (int ia = ib / 2; ia < NR; ++ia) {
                    const int ix = ia * (ia + 1) + ib;
                    const double u = fma(-vi[ia], wk, fma(-wi[ia], vk, a[ix]));
                    a[ix] = (ib < 2 * ia || (ib == 2 * ia ? keep0 : keep1)) ? u : 0.0;
                }
            }
        }
        L512_PUBLISH(j + 1);
    }
#undef L512_PUBLISH
#undef L512_PUBLISH_CASE
    // the last 2 x 2 block: d[n-2], d[n-1], e[n-2] (tau = 0, H = I)
#pragma unroll
    for (int ia = 0; ia < NR; ++ia)
#pragma unroll
        for (int ib = 0; ib <= 2 * ia + 1; ++ib) {
            const int i = tr + 32 * ia, k = tc + 16 * ib;
            const double av = a[ia * (ia + 1) + ib];
            if (i == n - 2 && k == n - 2) d[n - 2] = av;
            if (i == n - 1 && k == n - 1) d[n - 1] = av;
            if (i == n - 1 && k == n - 2) {
                e[n - 2] = av;
                tau[n - 2] = 0.0;
                for (int q = 0; q < n; ++q) V[size_t(n - 2) * n + q] = 0.0;
            }
        }
}

// one 64-lane workgroup per wanted eigenvalue: block q -> the q-th largest (ascending index n - 1 - q).
// Zt (kk x ldz): row q = the eigenvector of T (normalised); lam[q]. status[0] <- -1 if a multisection
// did not reach full precision.
//
// Every O(n) recurrence here is a dependent chain, so the kernel is written for chain latency:
//  * Sturm counts (multisection, lane l at the point lo + (hi - lo)(l + 1)/65) by the three-term recurrence
//    p_k = (d_k - x) p_{k-1} - e_{k-1}^2 p_{k-2} (one FMA per level on the chain, instead of a reciprocal
//    and its Newton steps in the ratio form q_k = p_k / p_{k-1}); #{lambda < x} = sign changes of p_0..p_n
//    (Barth, Martin & Wilkinson), an exact zero p_k taken as q_k = -pivmin (dlaebz's rule), the pair
//    (p_{k-1}, p_k) rescaled by a power of two every 8 levels (no over/underflow, signs unchanged). The
//    operands are uniform across lanes: blocks of 8 are read from LDS one block ahead of the chain.
//  * inverse iteration: the partially pivoted LU of T - lambda I (dgttrf) as a streaming recurrence whose
//    running pivot row stays in registers (factors stored to LDS, off the chain), the solves (dgttrs) with
//    their operands prefetched a block ahead. (The first version kept every running value in LDS: each
//    level waited on LDS round trips, ~100 us per eigenvalue set at n = 128.)
template <int NEWTON>
__global__ void __launch_bounds__(64) k_stebz_stein(const double* __restrict__ d, const double* __restrict__ e, int n,
                                                     double* __restrict__ lam, double* __restrict__ Zt, int ldz, int* __restrict__ status) {
    constexpr int B8 = 8;
    __shared__ double sd[SY_MAX + 2 * B8], se[SY_MAX + 2 * B8], se2[SY_MAX + 2 * B8];
    __shared__ double ud[SY_MAX], uu[SY_MAX], uu2[SY_MAX], ul[SY_MAX], lb[SY_MAX];
    __shared__ int upv[SY_MAX];
    const int lane = threadIdx.x, q = blockIdx.x, m = n - 1 - q;
    double gl = 1e300, gu = -1e300, emax2 = 0.0, amax = 0.0;
    for (int i = lane; i < n + 2 * B8; i += 64) {
        const bool in = i < n;
        const double di = in ? d[i] : 0.0, ei = i + 1 < n ? e[i] : 0.0, em = (in && i > 0) ? e[i - 1] : 0.0;
        sd[i] = di;
        se[i] = ei;
        se2[i] = ei * ei;
        if (in) {
            const double r = fabs(ei) + fabs(em);
            gl = fmin(gl, di - r);
            gu = fmax(gu, di + r);
            emax2 = fmax(emax2, ei * ei);
            amax = fmax(amax, fabs(di) + r);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        gl = fmin(gl, __shfl_xor(gl, o, 64));
        gu = fmax(gu, __shfl_xor(gu, o, 64));
        emax2 = fmax(emax2, __shfl_xor(emax2, o, 64));
        amax = fmax(amax, __shfl_xor(amax, o, 64));
    }
    // T scaled by a power of two to ||T|| ~ 1 (the recurrences then neither overflow nor underflow within
    // their 8-level rescaling blocks); the eigenvalue is scaled back, the eigenvector is unaffected
    const int tex = amax > 0.0 ? __builtin_amdgcn_frexp_exp(amax) : 0;
    const double tsc = __builtin_amdgcn_ldexp(1.0, -tex);
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        sd[i] *= tsc;
        se[i] *= tsc;
        se2[i] *= tsc * tsc;
    }
    gl *= tsc;
    gu *= tsc;
    emax2 *= tsc * tsc;
    amax *= tsc;
    __syncthreads();
    const double pivmin = 1e-290 * fmax(1.0, emax2);
    const double span = fmax(gu - gl, 1e-300);
    double lo = gl - 2.2e-16 * span - pivmin, hi = gu + 2.2e-16 * span + pivmin;
    // multisection: lane l counts the eigenvalues below lo + (hi - lo) (l + 1) / 65
    int rounds = 0;
    bool done = false;
    for (; rounds < 16 && !done; ++rounds) {
        const double x = lo + (hi - lo) * double(lane + 1) * (1.0 / 65.0);
        double pm = 1.0, p = sd[0] - x;   // p_0 = 1, p_1 = d_0 - x
        if (p == 0.0) p = -pivmin;
        int c = p < 0.0;
        double dn[B8], en[B8];
#pragma unroll
        for (int u = 0; u < B8; ++u) {
            dn[u] = sd[1 + u];
            en[u] = se2[u];
        }
        for (int i0 = 1; i0 < n; i0 += B8) {
            double dc[B8], ec[B8];
#pragma unroll
            for (int u = 0; u < B8; ++u) {
                dc[u] = dn[u];
                ec[u] = en[u];
                dn[u] = sd[i0 + B8 + u];   // next block (padded: reads stay inside the arrays)
                en[u] = se2[i0 + B8 - 1 + u];
            }
#pragma unroll
            for (int u = 0; u < B8; ++u) {
                if (i0 + u < n) {
                    double pn = fma(dc[u] - x, p, -ec[u] * pm);
                    if (pn == 0.0) pn = -pivmin * p;
                    c += (pn < 0.0) != (p < 0.0);
                    pm = p;
                    p = pn;
                }
            }
            // rescale the pair by a power of two (signs and ratios unchanged)
            const int ex = __builtin_amdgcn_frexp_exp(fmax(fabs(p), fabs(pm)));
            p = __builtin_amdgcn_ldexp(p, -ex);
            pm = __builtin_amdgcn_ldexp(pm, -ex);
        }
        double nlo = c <= m ? x : -1e300, nhi = c >= m + 1 ? x : 1e300;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            nlo = fmax(nlo, __shfl_xor(nlo, o, 64));
            nhi = fmin(nhi, __shfl_xor(nhi, o, 64));
        }
        if (nlo > lo) lo = nlo;
        if (nhi < hi) hi = nhi;
        // absolute accuracy u ||T|| (dstebz's default abstol): all a backward-stable reduction delivers
        done = (hi - lo) <= 2.2204460492503131e-16 * (2.0 * fmax(fabs(lo), fabs(hi)) + 4.0 * span) + 2.0 * pivmin;
    }
    const double lmb = 0.5 * (lo + hi);
    const double tiny = 2.2204460492503131e-16 * fmax(amax, 1e-300);
    if (lane == 0) {
        lam[q] = __builtin_amdgcn_ldexp(lmb, tex);
        if (!done) atomicMin(status, -1);
        // LU of T - lambda I with row interchanges where the subdiagonal entry is larger (dgttrf); the
        // running pivot row (a, b) = (diagonal, superdiagonal) of row i after the earlier eliminations.
        // Outputs per row: U diagonal ud (tiny pivots replaced by u ||T||, dlagtf's perturbation, stored
        // inverted), U super- / second superdiagonal uu, uu2, multiplier ul, interchange flag upv.
        double a = sd[0] - lmb, b = se[0];
        double sub[B8], dnx[B8], unx[B8];
#pragma unroll
        for (int u = 0; u < B8; ++u) {
            sub[u] = se[u];
            dnx[u] = sd[1 + u] - lmb;
            unx[u] = se[1 + u];
        }
        for (int i0 = 0; i0 + 1 < n; i0 += B8) {
            double s_[B8], dx[B8], ux[B8];
#pragma unroll
            for (int u = 0; u < B8; ++u) {
                s_[u] = sub[u];
                dx[u] = dnx[u];
                ux[u] = unx[u];
                sub[u] = se[i0 + B8 + u];
                dnx[u] = sd[i0 + B8 + 1 + u] - lmb;
                unx[u] = se[i0 + B8 + 1 + u];
            }
#pragma unroll
            for (int u = 0; u < B8; ++u) {
                const int i = i0 + u;
                if (i + 1 < n) {
                    if (fabs(a) >= fabs(s_[u])) {   // no interchange
                        const double f = a != 0.0 ? s_[u] * rcpn<NEWTON>(a) : 0.0;
                        ud[i] = a;
                        uu[i] = b;
                        uu2[i] = 0.0;
                        ul[i] = f;
                        upv[i] = 0;
                        a = fma(-f, b, dx[u]);
                        b = ux[u];
                    } else {                        // rows i and i+1 interchanged
                        const double f = a * rcpn<NEWTON>(s_[u]);
                        ud[i] = s_[u];
                        uu[i] = dx[u];
                        uu2[i] = i + 2 < n ? ux[u] : 0.0;
                        ul[i] = f;
                        upv[i] = 1;
                        a = fma(-f, dx[u], b);
                        b = i + 2 < n ? -f * ux[u] : 0.0;
                    }
                }
            }
        }
        ud[n - 1] = a;
    }
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        double p = ud[i];
        if (fabs(p) < tiny) p = copysign(tiny, p == 0.0 ? 1.0 : p);
        ud[i] = rcp2(p);   // inverse pivots
        lb[i] = 1.0 + double((i * 37 + q * 11) % 17) * (1.0 / 17.0);
    }
    __syncthreads();
    for (int it = 0; it < 3; ++it) {
        if (lane == 0) {   // dgttrs: forward with the interchanges, then back substitution, operands a block ahead
            double cur = lb[0];
            for (int i0 = 0; i0 + 1 < n; i0 += B8) {
                double f[B8], nx[B8];
                int pv[B8];
#pragma unroll
                for (int u = 0; u < B8; ++u) {
                    const int i = i0 + u;
                    const bool in = i + 1 < n;
                    f[u] = in ? ul[i] : 0.0;
                    nx[u] = in ? lb[i + 1] : 0.0;
                    pv[u] = in ? upv[i] : 0;
                }
#pragma unroll
                for (int u = 0; u < B8; ++u) {
                    const int i = i0 + u;
                    if (i + 1 < n) {
                        if (pv[u] == 0) {
                            lb[i] = cur;
                            cur = fma(-f[u], cur, nx[u]);
                        } else {
                            lb[i] = nx[u];
                            cur = fma(-f[u], nx[u], cur);
                        }
                    }
                }
            }
            double x1 = cur * ud[n - 1], x2 = 0.0;
            lb[n - 1] = x1;
            for (int i1 = n - 2; i1 >= 0; i1 -= B8) {
                double rb[B8], u1[B8], u2[B8], iv[B8];
#pragma unroll
                for (int u = 0; u < B8; ++u) {
                    const int i = i1 - u;
                    const bool in = i >= 0;
                    rb[u] = in ? lb[i] : 0.0;
                    u1[u] = in ? uu[i] : 0.0;
                    u2[u] = in ? uu2[i] : 0.0;
                    iv[u] = in ? ud[i] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < B8; ++u) {
                    const int i = i1 - u;
                    if (i >= 0) {
                        const double x0 = fma(-u1[u], x1, fma(-u2[u], x2, rb[u])) * iv[u];
                        lb[i] = x0;
                        x2 = x1;
                        x1 = x0;
                    }
                }
            }
        }
        __syncthreads();
        // normalise (scaled 2-norm over the wave)
        double mx = 0.0;
        for (int i = lane; i < n; i += 64) mx = fmax(mx, fabs(lb[i]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
        const double inv_mx = mx > 0.0 ? 1.0 / mx : 1.0;
        double ss = 0.0;
        for (int i = lane; i < n; i += 64) {
            const double v = lb[i] * inv_mx;
            ss = fma(v, v, ss);
        }
        ss = sum64(ss);
        const double sc = inv_mx / sqrt(ss);
        __syncthreads();
        for (int i = lane; i < n; i += 64) lb[i] *= sc;
        __syncthreads();
    }
    for (int i = lane; i < n; i += 64) Zt[size_t(q) * ldz + i] = lb[i];
}


// u = H_0 H_1 ... H_{n-2} z for every row z of Zt (in place): one wave per vector (entry i on lane i mod
// 64, ZE = n / 64 per lane), 4 vectors per 256-thread workgroup, so the dependent chain per reflector is
// two FMAs, a 64-lane reduction without the LDS crossbar (DPP, permlane16 / permlane32 swaps) and one
// FMA; the reflectors pass through LDS in chunks of 16384 / n rows, staged by the whole workgroup with
// coalesced loads. (The first version, 16 lanes per vector and 16 vectors per workgroup, ran a 16-deep
// FMA chain per reflector on only kk / 16 workgroups: 150 us at n = 256, kk = 128.)
template <int ZE>
__global__ void __launch_bounds__(256) k_ormtr(const double* __restrict__ V, const double* __restrict__ tau, int n, int kk,
                                               double* __restrict__ Zt, int ldz) {
    constexpr int CHUNK_ELEMS = 16384;
    __shared__ double sv[CHUNK_ELEMS], st[SY_MAX];
    for (int e = threadIdx.x; e < n; e += 256) st[e] = e + 1 < n ? tau[e] : 0.0;
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool live = q < kk;
    double z[ZE];
#pragma unroll
    for (int s = 0; s < ZE; ++s) {
        const int i = lane + 64 * s;
        z[s] = (live && i < n) ? Zt[size_t(q) * ldz + i] : 0.0;
    }
    const int rows = CHUNK_ELEMS / n;
    for (int hi = n - 2; hi >= 0; hi -= rows) {
        const int lo = hi - rows + 1 > 0 ? hi - rows + 1 : 0;
        __syncthreads();
        for (int e = threadIdx.x; e < (hi - lo + 1) * n; e += 256) sv[e] = V[size_t(lo) * n + e];
        __syncthreads();
        for (int j = hi; j >= lo; --j) {   // (tau_j = 0: f = 0, z unchanged)
            const double* v = sv + size_t(j - lo) * n;
            double vv[ZE];
            double d0 = 0.0, d1 = 0.0;
#pragma unroll
            for (int s = 0; s < ZE; ++s) {
                const int i = lane + 64 * s;
                vv[s] = i < n ? v[i] : 0.0;
                if (s & 1) d1 = fma(vv[s], z[s], d1);
                else d0 = fma(vv[s], z[s], d0);
            }
            const double f = st[j] * sum64(d0 + d1);
#pragma unroll
            for (int s = 0; s < ZE; ++s) z[s] = fma(-f, vv[s], z[s]);
        }
    }
    if (live) {
#pragma unroll
        for (int s = 0; s < ZE; ++s) {
            const int i = lane + 64 * s;
            if (i < n) Zt[size_t(q) * ldz + i] = z[s];
        }
    }
}

__global__ void k_sqrt_lam(const double* __restrict__ lam, int kk, double* __restrict__ S) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < kk) S[i] = sqrt(fmax(lam[i], 0.0));
}

// ---------------------------------------------------------------------------------------------------------
// Two-stage tridiagonalisation (orders 33..256): dense -> band of width SB by blocked Householder panels
// whose two-sided trailing updates are MFMA products (k_sy2sb), then band -> tridiagonal by bulge chasing
// with one wave per sweep and the sweeps pipelined across the workgroup's waves (k_sb2st). The one-stage
// kernels above spend every column step on a workgroup-wide latency chain (3 barriers, ~3 us per column);
// here the dense work is blocked (16 columns per panel, one chain of MFMA launches per panel) and the
// column-by-column work runs on 16 x 16 blocks inside single waves. Back-transformation: the stage-2
// reflectors by wavefront-parallel application (k_apply_q2), the panel reflectors as block reflectors
// I - V T V^T with MFMA (k_apply_q1).
constexpr int SB = 16;              // band width
constexpr int AB_LD = 2 * SB;       // band + bulge storage per column in k_sb2st
constexpr int SB_WAVES = 8;         // waves of k_sb2st (concurrent sweeps)

__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); }

struct Sy2sbArgs {
    const double* A;   // input, lower triangle read (lda)
    int lda, n;
    double* W;         // n x n work matrix (lower triangle maintained)
    double* band;      // (SB + 1) x n: band[k n + j] = A[j + k][j]
    double* V;         // panel p's reflectors (m_p x SB, row-major) at p * SB * n
    double* T;         // panel p's block-reflector factor (SB x SB upper) at p * SB * SB
};

// stage 1: A = Q1 Bd Q1^T, Q1 = prod_p (I - V_p T_p V_p^T) acting on rows r0_p = SB (p + 1) .. n-1
__global__ void __launch_bounds__(256) k_sy2sb(const Sy2sbArgs g) {
    __shared__ double Vs[SY_MAX * SB], Xs[SY_MAX * SB], Ws[SY_MAX * SB];
    __shared__ double Gp[4][SB * SB], Ts[SB * SB], Zs[SB * SB];
    __shared__ double vcol[2][SY_MAX], taus[SB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = g.n;
    double* __restrict__ W = g.W;
    for (int e = tid; e < n * n; e += 256) {
        const int r = e / n, c = e - r * n;
        if (c <= r) W[e] = g.A[size_t(r) * g.lda + c];
    }
    __syncthreads();
    for (int p = 0;; ++p) {
        const int c0 = SB * p, r0 = c0 + SB, m = n - r0;
        {   // the diagonal block of the band is final (later panels touch rows / columns >= r0 only)
            const int r = tid >> 4, c = tid & 15;
            if (c0 + r < n && c <= r) g.band[(r - c) * n + c0 + c] = W[(c0 + r) * n + c0 + c];
        }
        if (m < 2) {   // nothing left to annihilate (a single row below is inside the band)
            if (m == 1) {
                if (tid < SB) g.band[(SB - tid) * n + c0 + tid] = W[(n - 1) * n + c0 + tid];
                if (tid == 0) g.band[n - 1] = W[(n - 1) * n + n - 1];
            }
            break;
        }
        const int MT = (m + SB - 1) / SB, KS = (m + 3) / 4;
        // (1) panel QR, m x SB: wave w holds columns 4w .. 4w+3 of rows lane + 64 t
        double P[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int i = lane + 64 * t;
                P[t][cc] = i < m ? W[(r0 + i) * n + c0 + 4 * wave + cc] : 0.0;
            }
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int jc = j & 3;
            double* vc = vcol[j & 1];   // double-buffered: one barrier per column
            if (wave == (j >> 2)) {     // dlarfg on column j
                const double alpha = __shfl(P[0][jc], j, 64);
                double s = 0.0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int i = lane + 64 * t;
                    if (i > j && i < m) s = fma(P[t][jc], P[t][jc], s);
                }
                s = sum64(s);
                double tv = 0.0, beta = alpha, scal = 0.0;
                if (s > 0.0) {
                    beta = -copysign(sqrt(fma(alpha, alpha, s)), alpha);
                    tv = (beta - alpha) * rcp2(beta);
                    scal = rcp2(alpha - beta);
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int i = lane + 64 * t;
                    const double v = (i < j || i >= m) ? 0.0 : (i == j ? 1.0 : P[t][jc] * scal);
                    vc[i] = v;
                    Vs[i * SB + j] = v;
                    if (i == j) P[t][jc] = beta;
                    else if (i > j) P[t][jc] = 0.0;
                }
                if (lane == 0) taus[j] = tv;
            }
            __syncthreads();
            const double tj = taus[j];
            if (4 * wave + 3 > j && tj != 0.0) {   // H_j on the wave's columns right of j
                double dots[4], vv[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) vv[t] = vc[lane + 64 * t];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    double a = 0.0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) a = fma(vv[t], P[t][cc], a);
                    dots[cc] = (4 * wave + cc > j) ? sum64(a) : 0.0;
                }
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc)
                        if (4 * wave + cc > j) P[t][cc] = fma(-tj * dots[cc], vv[t], P[t][cc]);
            }
        }
        // R (rows 0..15 of the panel, lanes 0..15) into the band; V to global for the back-transformation
        if (lane < SB && lane < m) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int c = 4 * wave + cc;
                if (c >= lane) g.band[(SB + lane - c) * n + c0 + c] = P[0][cc];
            }
        }
        for (int e = tid; e < m * SB; e += 256) g.V[size_t(p) * SB * n + e] = Vs[e];
        // (2) T (dlarft, forward columnwise) from G = V^T V (MFMA, K split over the waves)
        {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int ks = wave; ks < KS; ks += 4) {
                const double v = Vs[(4 * ks + (lane >> 4)) * SB + (lane & 15)];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) Gp[wave][((lane >> 4) + 4 * q) * SB + (lane & 15)] = acc[q];
        }
        __syncthreads();
        if (wave == 0 && lane < SB) {
            const int i = lane;
            double trow[SB];
#pragma unroll
            for (int j = 0; j < SB; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < j; ++k) {
                    const double gkj = (Gp[0][k * SB + j] + Gp[1][k * SB + j]) + (Gp[2][k * SB + j] + Gp[3][k * SB + j]);
                    if (k >= i) s = fma(trow[k], gkj, s);
                }
                trow[j] = (i == j) ? taus[j] : (i < j ? -taus[j] * s : 0.0);
            }
#pragma unroll
            for (int j = 0; j < SB; ++j) {
                Ts[i * SB + j] = trow[j];
                g.T[p * SB * SB + i * SB + j] = trow[j];
            }
        }
        __syncthreads();
        // (3) X = A22 V (A22: rows / columns r0.., symmetric reads of the lower triangle), MFMA tiles
        for (int I = wave; I < MT; I += 4) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            const int ra = SB * I + (lane & 15);
            for (int J = 0; J < MT; ++J) {
                double av[4], bv[4];
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int ca = SB * J + 4 * ks + (lane >> 4);
                    const int hi = ra > ca ? ra : ca, lo = ra > ca ? ca : ra;
                    av[ks] = (hi < m) ? W[(r0 + hi) * n + r0 + lo] : 0.0;
                    bv[ks] = Vs[ca * SB + (lane & 15)];
                }
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) Xs[(SB * I + (lane >> 4) + 4 * q) * SB + (lane & 15)] = acc[q];
        }
        __syncthreads();
        // (4) Y = X T (in place, one row per thread), S = V^T Y, Z = T^T S, W = Y - V Z / 2
        if (tid < SB * MT) {
            double x[SB], y[SB];
#pragma unroll
            for (int k = 0; k < SB; ++k) x[k] = Xs[tid * SB + k];
#pragma unroll
            for (int c = 0; c < SB; ++c) {
                double a = 0.0;
#pragma unroll
                for (int k = 0; k <= c; ++k) a = fma(x[k], Ts[k * SB + c], a);
                y[c] = a;
            }
#pragma unroll
            for (int c = 0; c < SB; ++c) Xs[tid * SB + c] = y[c];
        }
        __syncthreads();
        {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int ks = wave; ks < KS; ks += 4) {
                const int k = 4 * ks + (lane >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Vs[k * SB + (lane & 15)], Xs[k * SB + (lane & 15)], acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) Gp[wave][((lane >> 4) + 4 * q) * SB + (lane & 15)] = acc[q];
        }
        __syncthreads();
        {
            const int a = tid >> 4, c = tid & 15;
            double z = 0.0;
            for (int k = 0; k <= a; ++k) {
                const double skc = (Gp[0][k * SB + c] + Gp[1][k * SB + c]) + (Gp[2][k * SB + c] + Gp[3][k * SB + c]);
                z = fma(Ts[k * SB + a], skc, z);
            }
            Zs[a * SB + c] = z;
        }
        __syncthreads();
        if (tid < SB * MT) {
            double v[SB];
#pragma unroll
            for (int k = 0; k < SB; ++k) v[k] = Vs[tid * SB + k];
#pragma unroll
            for (int c = 0; c < SB; ++c) {
                double a = 0.0;
#pragma unroll
                for (int k = 0; k < SB; ++k) a = fma(v[k], Zs[k * SB + c], a);
                Ws[tid * SB + c] = fma(-0.5, a, Xs[tid * SB + c]);
            }
        }
        __syncthreads();
        // (5) A22 -= V W^T + W V^T on the lower tiles (MFMA, C layout: row (l >> 4) + 4 q, column l & 15)
        const int ntl = MT * (MT + 1) / 2;
        for (int tile = wave; tile < ntl; tile += 4) {
            int I = int((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
            while ((I + 1) * (I + 2) / 2 <= tile) ++I;
            while (I * (I + 1) / 2 > tile) --I;
            const int J = tile - I * (I + 1) / 2;
            const int cj = SB * J + (lane & 15);
            d4 acc;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ri = SB * I + (lane >> 4) + 4 * q;
                acc[q] = (ri < m && cj < m && ri >= cj) ? W[(r0 + ri) * n + r0 + cj] : 0.0;
            }
            const int ar = (SB * I + (lane & 15)) * SB, br = (SB * J + (lane & 15)) * SB;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int k = 4 * ks + (lane >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-Vs[ar + k], Ws[br + k], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-Ws[ar + k], Vs[br + k], acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ri = SB * I + (lane >> 4) + 4 * q;
                if (ri < m && cj < m && ri >= cj) W[(r0 + ri) * n + r0 + cj] = acc[q];
            }
        }
        __syncthreads();
    }
}

// stage 2: band (width SB, lower storage) -> tridiagonal by bulge chasing (sweep s annihilates column s;
// its block k >= 1 applies the previous reflector from the right to the block below (creating the bulge),
// annihilates the bulge's first column with a new reflector from the left, and applies that reflector to
// the next diagonal block from both sides). One wave per sweep (a 16 x 16 block: lane l holds row l & 15,
// columns (l >> 4) + 4 t); sweep s waits until sweep s - 1 has finished two more blocks than it is about to
// start (the blocks that overlap). Reflector (s, k) -> refl[((2 s + k) nslot + k / 2) 17]: v[0..15], tau
// (grouped by the wavefront t = 2 s + k: the reflectors of one t act on disjoint rows, see k_apply_q2).
__global__ void __launch_bounds__(SB_WAVES * 64) k_sb2st(const double* __restrict__ band, int n, double* __restrict__ d,
                                                        double* __restrict__ e, double* __restrict__ refl, int nslot) {
    __shared__ double ab[SY_MAX * AB_LD];
    __shared__ int prog[SY_MAX];
    __shared__ double sv[SB_WAVES][SB], sw[SB_WAVES][SB], sx[SB_WAVES][SB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int q = tid; q < n * AB_LD; q += SB_WAVES * 64) {
        const int j = q / AB_LD, k = q - j * AB_LD;
        ab[q] = (k <= SB && j + k < n) ? band[k * n + j] : 0.0;
    }
    for (int q = tid; q < SY_MAX; q += SB_WAVES * 64) prog[q] = 0;
    __syncthreads();
    const int r = lane & 15, gq = lane >> 4;
    double* vsh = sv[wave];
    double* wsh = sw[wave];
    double* xsh = sx[wave];
    // A[row][col] of the lower band + bulge (row >= col, row - col < AB_LD)
    auto at = [&](int row, int col) -> double& { return ab[col * AB_LD + (row - col)]; };
    // two-sided H D H on the symmetric block rows / columns i0 .. i0+L-1, H = I - tau v v^T (v_r in vsh)
    auto two_sided = [&](int i0, int L, double tau) {
        if (tau == 0.0) return;
        double D[4], vc[4];
        const bool rin = r < L;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = gq + 4 * t;
            vc[t] = vsh[c];
            D[t] = (rin && c < L) ? (r >= c ? at(i0 + r, i0 + c) : at(i0 + c, i0 + r)) : 0.0;
        }
        const double vr = vsh[r];
        double pr = (D[0] * vc[0] + D[1] * vc[1]) + (D[2] * vc[2] + D[3] * vc[3]);
        pr += xor16(pr);
        pr += xor32(pr);
        pr *= tau;
        const double K = -0.5 * tau * sum16(pr * vr);
        const double wr = fma(K, vr, pr);
        if (gq == 0) wsh[r] = wr;
        wave_lds_order();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = gq + 4 * t;
            const double wc = wsh[c];
            const double u = fma(-vr, wc, fma(-wr, vc[t], D[t]));
            if (rin && c < L && r >= c) at(i0 + r, i0 + c) = u;
        }
        wave_lds_order();
    };
    for (int s = wave; s + 2 < n; s += SB_WAVES) {
        const int nblk = (n - 2 - s) / SB + 1;
        double tprev = 0.0;
        int Lprev = 0;
        for (int k = 0; k < nblk; ++k) {
            if (s > 0) {   // sweep s - 1 two blocks ahead (or finished)
                while (__hip_atomic_load(&prog[s - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < k + 2)
                    __builtin_amdgcn_s_sleep(1);
            }
            double tau;
            int L;
            if (k == 0) {   // annihilate column s below its subdiagonal
                L = min(SB, n - 1 - s);
                const double x = r < L ? at(s + 1 + r, s) : 0.0;
                const double alpha = __shfl(x, 0, 16);
                const double ss = sum16(r >= 1 ? x * x : 0.0);
                double beta = alpha, scal = 0.0;
                tau = 0.0;
                if (ss > 0.0) {
                    beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
                    tau = (beta - alpha) * rcp2(beta);
                    scal = rcp2(alpha - beta);
                }
                const double v = r == 0 ? 1.0 : (r < L ? x * scal : 0.0);
                if (gq == 0) {
                    vsh[r] = v;
                    if (r < L && tau != 0.0) at(s + 1 + r, s) = r == 0 ? beta : 0.0;
                }
                wave_lds_order();
                two_sided(s + 1, L, tau);
            } else {
                const int R0 = s + 1 + k * SB, C0 = R0 - SB;
                L = min(SB, n - R0);
                // C = A[R0 .., C0 ..] (L x Lprev): C <- C H_{k-1}, then H_k from C's first column, C <- H_k C
                double C[4], vc[4];
                const bool rin = r < L;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int c = gq + 4 * t;
                    vc[t] = vsh[c];
                    C[t] = (rin && c < Lprev) ? at(R0 + r, C0 + c) : 0.0;
                }
                if (tprev != 0.0) {
                    double y = (C[0] * vc[0] + C[1] * vc[1]) + (C[2] * vc[2] + C[3] * vc[3]);
                    y += xor16(y);
                    y += xor32(y);
#pragma unroll
                    for (int t = 0; t < 4; ++t) C[t] = fma(-tprev * y, vc[t], C[t]);
                }
                if (gq == 0) xsh[r] = C[0];   // the first column (c = 0 on the lanes with gq = 0, t = 0)
                wave_lds_order();
                const double x = xsh[r];
                const double alpha = xsh[0];
                const double ss = sum16(r >= 1 && rin ? x * x : 0.0);
                double beta = alpha, scal = 0.0;
                tau = 0.0;
                if (ss > 0.0) {
                    beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
                    tau = (beta - alpha) * rcp2(beta);
                    scal = rcp2(alpha - beta);
                }
                const double vr = r == 0 ? 1.0 : (rin ? x * scal : 0.0);
                if (tau != 0.0) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const double z = sum16(vr * C[t]);
                        C[t] = fma(-tau * z, vr, C[t]);
                    }
                    if (gq == 0) C[0] = r == 0 ? beta : 0.0;
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int c = gq + 4 * t;
                    if (rin && c < Lprev) at(R0 + r, C0 + c) = C[t];
                }
                wave_lds_order();
                if (gq == 0) vsh[r] = vr;
                wave_lds_order();
                two_sided(R0, L, tau);
            }
            if (refl) {   // reflector (s, k) for the back-transformation, at wavefront t = 2 s + k, slot k / 2
                double* rp = refl + (size_t(2 * s + k) * nslot + (k >> 1)) * 17;
                if (gq == 0) rp[r] = vsh[r];
                if (lane == 0) rp[16] = tau;
            }
            tprev = tau;
            Lprev = L;
            wave_lds_order();
            if (lane == 0) __hip_atomic_store(&prog[s], k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (lane == 0) __hip_atomic_store(&prog[s], 1 << 30, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    for (int j = tid; j < n; j += SB_WAVES * 64) {
        d[j] = at(j, j);
        if (j + 1 < n) e[j] = at(j + 1, j);
    }
}

// Clusters of close eigenvalues (|lam_i - lam_{i+1}| <= 1e-3 ||T||, dstein's ORTOL): inverse iteration from
// different start vectors lands in the cluster's invariant subspace, but not orthogonally -- the vectors of each
// cluster are orthonormalised by two passes of modified Gram-Schmidt (in order of decreasing eigenvalue, as
// dstein reorthogonalises against the earlier vectors of a cluster). One workgroup; without clusters it only
// scans the eigenvalues.
__global__ void __launch_bounds__(256) k_cluster_orth(const double* __restrict__ lam, const double* __restrict__ d,
                                                      const double* __restrict__ e, int n, int kk, double* __restrict__ Zt, int ldz) {
    __shared__ double red[4];
    __shared__ double tnorm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double a = 0.0;
    for (int i = tid; i < n; i += 256) a = fmax(a, fabs(d[i]) + (i > 0 ? fabs(e[i - 1]) : 0.0) + (i + 1 < n ? fabs(e[i]) : 0.0));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a = fmax(a, __shfl_xor(a, o, 64));
    if (lane == 0) red[wave] = a;
    __syncthreads();
    if (tid == 0) tnorm = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    const double ortol = 1e-3 * tnorm;
    auto dot = [&](const double* x, const double* y) {
        double s = 0.0;
        for (int i = tid; i < n; i += 256) s = fma(x[i], y[i], s);
        s = sum64(s);
        __syncthreads();
        if (lane == 0) red[wave] = s;
        __syncthreads();
        return (red[0] + red[1]) + (red[2] + red[3]);
    };
    int c0 = 0;
    while (c0 < kk) {
        int c1 = c0 + 1;
        while (c1 < kk && fabs(lam[c1 - 1] - lam[c1]) <= ortol) ++c1;
        for (int j = c0 + 1; j < c1; ++j) {   // cluster [c0, c1): orthonormalise vector j against c0 .. j-1
            double* zj = Zt + size_t(j) * ldz;
            for (int pass = 0; pass < 2; ++pass) {
                for (int i = c0; i < j; ++i) {
                    const double* zi = Zt + size_t(i) * ldz;
                    const double c = dot(zi, zj);
                    for (int k = tid; k < n; k += 256) zj[k] = fma(-c, zi[k], zj[k]);
                    __syncthreads();
                }
                const double nn = sqrt(dot(zj, zj));
                const double inv = nn > 0.0 ? 1.0 / nn : 0.0;
                for (int k = tid; k < n; k += 256) zj[k] *= inv;
                __syncthreads();
            }
        }
        c0 = c1;
    }
}

// Q2 z for the kk eigenvectors z of T (rows of Zt, in place): the stage-2 reflectors in reverse order of
// generation. Sweep s's block k acts on rows s + 1 + 16 k .. +15; the reflectors of one wavefront t = 2 s + k
// act on disjoint rows (consecutive sweeps' blocks of equal t are 2 SB - 1 rows apart) and, whenever an
// earlier-generated reflector has a larger t, the two are disjoint too -- so applying the wavefronts from the
// last to the first, each wavefront's reflectors in any order, is the reverse generation order. The
// reflectors are shared by all vectors: chunks of QC_T wavefronts are staged through LDS by the workgroup;
// each wave carries one vector (LDS), its 4 groups of 16 lanes apply a wavefront's reflectors (one per row
// of 16 lanes: a DPP row sum and one FMA), no barriers inside a chunk.
constexpr int QC_T = 32;
template <int NSLOT>
__global__ void __launch_bounds__(256) k_apply_q2(const double* __restrict__ refl, int n, int kk, int tcount, double* __restrict__ Zt,
                                                  int ldz) {
    __shared__ double rs[QC_T * NSLOT * 17];
    __shared__ double zs[4][SY_MAX];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int q = blockIdx.x * 4 + wave;
    const bool live = q < kk;
    for (int i = lane; i < n; i += 64) zs[wave][i] = live ? Zt[size_t(q) * ldz + i] : 0.0;
    double* z = zs[wave];
    for (int thi = tcount - 1; thi >= 0; thi -= QC_T) {
        const int tlo = max(0, thi - QC_T + 1);
        __syncthreads();
        const int cnt = (thi - tlo + 1) * NSLOT * 17;
        for (int e = tid; e < cnt; e += 256) rs[e] = refl[size_t(tlo) * NSLOT * 17 + e];
        __syncthreads();
        for (int t = thi; t >= tlo; --t) {
            const double* rt = rs + (t - tlo) * NSLOT * 17;
            double zr[(NSLOT + 3) / 4], vr[(NSLOT + 3) / 4], tr[(NSLOT + 3) / 4];
            int row[(NSLOT + 3) / 4];
#pragma unroll
            for (int u = 0; u < (NSLOT + 3) / 4; ++u) {   // the group's reflectors of this wavefront (disjoint rows)
                const int slot = g + 4 * u;
                const int k = 2 * slot + (t & 1), s = (t - k) >> 1;
                const int R0 = s + 1 + SB * k;
                const bool ok = slot < NSLOT && k <= t && R0 + r < n;
                row[u] = ok ? R0 + r : -1;
                vr[u] = ok ? rt[slot * 17 + r] : 0.0;
                tr[u] = ok ? rt[slot * 17 + 16] : 0.0;
                zr[u] = ok ? z[R0 + r] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < (NSLOT + 3) / 4; ++u) {
                const double dot = sum16(vr[u] * zr[u]);
                if (row[u] >= 0) z[row[u]] = fma(-tr[u] * dot, vr[u], zr[u]);
            }
            wave_lds_order();
        }
    }
    wave_lds_order();
    if (live)
        for (int i = lane; i < n; i += 64) Zt[size_t(q) * ldz + i] = z[i];
}

// Q1 Y for 16 vectors per workgroup (rows of Zt): the stage-1 block reflectors H_p = I - V_p T_p V_p^T (rows
// r0_p = 16 (p + 1) ..), applied from the last panel to the first; in row form Y <- Y - ((Y V) T^T) V^T with
// MFMA: G = Y V (16 x 16, K = m over the 4 waves), G2 = G T^T, then the 16 x m update in 16 x 16 tiles.
__global__ void __launch_bounds__(256) k_apply_q1(const double* __restrict__ V, const double* __restrict__ Tp, int n, int npanel, int kk,
                                                  double* __restrict__ Zt, int ldz) {
    __shared__ double ys[SB * SY_MAX], vs[SY_MAX * SB], gp[4][SB * SB], g2[SB * SB], ts[SB * SB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * SB;
    for (int e = tid; e < SB * n; e += 256) {
        const int a = e / n, i = e - a * n;
        ys[a * SY_MAX + i] = (q0 + a < kk) ? Zt[size_t(q0 + a) * ldz + i] : 0.0;
    }
    for (int p = npanel - 1; p >= 0; --p) {
        const int r0 = SB * (p + 1), m = n - r0, KS = (m + 3) / 4;
        __syncthreads();
        for (int e = tid; e < KS * 4 * SB; e += 256) vs[e] = e < m * SB ? V[size_t(p) * SB * n + e] : 0.0;
        ts[tid] = Tp[p * SB * SB + tid];
        __syncthreads();
        {   // G = Y[:, r0..] V (16 x 16)
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int ks = wave; ks < KS; ks += 4) {
                const int k = 4 * ks + (lane >> 4);
                const double av = k < m ? ys[(lane & 15) * SY_MAX + r0 + k] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, vs[k * SB + (lane & 15)], acc, 0, 0, 0);
            }
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) gp[wave][((lane >> 4) + 4 * qq) * SB + (lane & 15)] = acc[qq];
        }
        __syncthreads();
        {   // G2 = G T^T: G2[a][c] = sum_k G[a][k] T[c][k] (T upper: k >= c)
            const int a = tid >> 4, c = tid & 15;
            double s2 = 0.0;
            for (int k = c; k < SB; ++k) {
                const double gak = (gp[0][a * SB + k] + gp[1][a * SB + k]) + (gp[2][a * SB + k] + gp[3][a * SB + k]);
                s2 = fma(gak, ts[c * SB + k], s2);
            }
            g2[a * SB + c] = s2;
        }
        __syncthreads();
        // Y[:, r0 + 16 J ..] -= G2 V_J^T
        const int MT = (m + SB - 1) / SB;
        for (int J = wave; J < MT; J += 4) {
            d4 acc;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int a = (lane >> 4) + 4 * qq, col = SB * J + (lane & 15);
                acc[qq] = col < m ? ys[a * SY_MAX + r0 + col] : 0.0;
            }
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int k = 4 * ks + (lane >> 4);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-g2[(lane & 15) * SB + k], vs[(SB * J + (lane & 15)) * SB + k], acc, 0, 0, 0);
            }
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int a = (lane >> 4) + 4 * qq, col = SB * J + (lane & 15);
                if (col < m) ys[a * SY_MAX + r0 + col] = acc[qq];
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < SB * n; e += 256) {
        const int a = e / n, i = e - a * n;
        if (q0 + a < kk) Zt[size_t(q0 + a) * ldz + i] = ys[a * SY_MAX + i];
    }
}

}  // namespace

// Order limit 256 (XRS_SYEV_MAX lowers it): the 512-thread lower-block kernel runs an order-256 edge in
// 1.31 ms against 2.8 ms of Jacobi sweeps ((x + y).round(128): 22.5 -> 13.8 ms, profiles/r03/sum128_l512_r03s.txt).
// Its first version spilled (the tau = 0 early exit gave the column loop a second latch, and the register
// copies at the merge doubled the live matrix): 3.6 ms; the spilling 1024-thread variant measured 5.8 ms.
bool sym_eig_top_fits(int n, int kk) {
    static const int nmax = std::getenv("XRS_SYEV_MAX") ? std::atoi(std::getenv("XRS_SYEV_MAX")) : 256;
    return n >= 2 && n <= std::min(nmax, SY_MAX) && kk >= 1 && kk <= n;
}

// Two-stage tridiagonalisation A = Q1 Q2 T Q2^T Q1^T (d, e of T; the reflectors in the optional buffers:
// V (n x n), Tp (n / SB x SB x SB), refl (17 x (n - 2) x (n / SB + 1))). Enqueued only.
constexpr int Q2_SLOTS = 9;   // reflectors per wavefront: k / 2 <= (256 / SB) / 2
size_t q2_refl_elems(int n) { return size_t(2 * n) * Q2_SLOTS * 17; }

void sym_tridiag_2stage(xrs_handle_t h, const double* A, int lda, int n, double* d, double* e, double* V, double* Tp, double* refl) {
    XRS_REQUIRE(n >= 2 && n <= SY_MAX, "sym_tridiag_2stage: need 2 <= n <= 256");
    if (refl) XRS_HIP(hipMemsetAsync(refl, 0, q2_refl_elems(n) * 8, h->stream));
    DevBuf W(h, size_t(n) * n * 8), band(h, size_t(SB + 1) * n * 8), Vb(h, V ? 0 : size_t(n) * n * 8), Tb(h, Tp ? 0 : size_t(n / SB + 1) * SB * SB * 8);
    XRS_HIP(hipMemsetAsync(band.d(), 0, size_t(SB + 1) * n * 8, h->stream));
    Sy2sbArgs g{A, lda, n, W.d(), band.d(), V ? V : Vb.d(), Tp ? Tp : Tb.d()};
    hipLaunchKernelGGL(k_sy2sb, dim3(1), dim3(256), 0, h->stream, g);
    check_launch("k_sy2sb");
    hipLaunchKernelGGL(k_sb2st, dim3(1), dim3(SB_WAVES * 64), 0, h->stream, band.d(), n, d, e, refl, Q2_SLOTS);
    check_launch("k_sb2st");
}

void sym_eig_top(xrs_handle_t h, const double* A, int lda, int n, int kk, double* lam, double* S, double* Ut, int ldu, int* status) {
XRS_REQUIRE(n >= 2 && n <= SY_MAX && kk >= 1 && kk <= n, "sym_eig_top: need 2 <= n <= 256 and 1 <= kk <= n");
    DevBuf dbuf(h, size_t(n) * 8), ebuf(h, size_t(n) * 8), tbuf(h, size_t(n) * 8), V(h, size_t(n) * n * 8), lbuf(h, size_t(kk) * 8);
    double* lm = lam ? lam : lbuf.d();
    KernelTimer timer(h, XRS_KFAM_SVD, 4.0 / 3.0 * double(n) * n * n + 4.0 * double(n) * n * kk, 8.0 * double(n) * n * 2);
    static const bool want_stamps = stamps_enabled("syev");
    DevBuf sb(h, want_stamps ? 768 * 8 : 0);
    unsigned long long* stp = want_stamps ? sb.as<unsigned long long>() : nullptr;
    if (stp) XRS_HIP(hipMemsetAsync(stp, 0, 768 * 8, h->stream));
    if (n > 32) {   // two-stage tridiagonalisation, eigenpairs of T, back-transformation Q1 Q2 z
        DevBuf Vp(h, size_t(n) * n * 8), Tp(h, size_t(n / SB + 1) * SB * SB * 8), refl(h, q2_refl_elems(n) * 8);
        sym_tridiag_2stage(h, A, lda, n, dbuf.d(), ebuf.d(), Vp.d(), Tp.d(), refl.d());
        hipLaunchKernelGGL(k_stebz_stein<2>, dim3(kk), dim3(64), 0, h->stream, dbuf.d(), ebuf.d(), n, lm, Ut, ldu, status);
        check_launch("k_stebz_stein");
        hipLaunchKernelGGL(k_cluster_orth, dim3(1), dim3(256), 0, h->stream, lm, dbuf.d(), ebuf.d(), n, kk, Ut, ldu);
        check_launch("k_cluster_orth");
        hipLaunchKernelGGL((k_apply_q2<Q2_SLOTS>), dim3((kk + 3) / 4), dim3(256), 0, h->stream, refl.d(), n, kk, 2 * n, Ut, ldu);
        check_launch("k_apply_q2");
        int npanel = 0;
        while (n - SB * (npanel + 1) >= 2) ++npanel;
        if (npanel > 0) {
            hipLaunchKernelGGL(k_apply_q1, dim3((kk + SB - 1) / SB), dim3(256), 0, h->stream, Vp.d(), Tp.d(), n, npanel, kk, Ut, ldu);
            check_launch("k_apply_q1");
        }
        if (S) {
            hipLaunchKernelGGL(k_sqrt_lam, dim3((kk + 255) / 256), dim3(256), 0, h->stream, lm, kk, S);
            check_launch("k_sqrt_lam");
        }
        return;
    }
    // one-stage (orders <= 32): the register-resident column steps
    if (n <= 64) {
        hipLaunchKernelGGL((k_sytrd<32, 2>), dim3(1), dim3(1024), 0, h->stream, A, lda, n, dbuf.d(), ebuf.d(), tbuf.d(), V.d(), stp);
    } else if (n <= 128) {
        hipLaunchKernelGGL((k_sytrd<32, 4>), dim3(1), dim3(1024), 0, h->stream, A, lda, n, dbuf.d(), ebuf.d(), tbuf.d(), V.d(), stp);
    } else {
        hipLaunchKernelGGL(k_sytrd_l512, dim3(1), dim3(512), 0, h->stream, A, lda, n, dbuf.d(), ebuf.d(), tbuf.d(), V.d());
    }
    check_launch("k_sytrd");
    // the chains' reciprocals: 2 Newton steps after the hardware estimate (one step measured 4.40 vs 4.47 ms
    // per cfg3 round(64) but multiplies the kept sigma's relative error by ~20)
    hipLaunchKernelGGL(k_stebz_stein<2>, dim3(kk), dim3(64), 0, h->stream, dbuf.d(), ebuf.d(), n, lm, Ut, ldu, status);
    check_launch("k_stebz_stein");
    hipLaunchKernelGGL(k_cluster_orth, dim3(1), dim3(256), 0, h->stream, lm, dbuf.d(), ebuf.d(), n, kk, Ut, ldu);
    check_launch("k_cluster_orth");
    if (n <= 64) hipLaunchKernelGGL((k_ormtr<1>), dim3((kk + 3) / 4), dim3(256), 0, h->stream, V.d(), tbuf.d(), n, kk, Ut, ldu);
    else if (n <= 128) hipLaunchKernelGGL((k_ormtr<2>), dim3((kk + 3) / 4), dim3(256), 0, h->stream, V.d(), tbuf.d(), n, kk, Ut, ldu);
    else hipLaunchKernelGGL((k_ormtr<4>), dim3((kk + 3) / 4), dim3(256), 0, h->stream, V.d(), tbuf.d(), n, kk, Ut, ldu);
    check_launch("k_ormtr");
    if (stp) {   // per-phase cycles of the first steps: (b)-wait, reflector, wait, symv, wait, update (+ column)
        std::vector<unsigned long long> hst(768);
        XRS_HIP(hipMemcpyAsync(hst.data(), stp, 768 * 8, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipStreamSynchronize(h->stream));
        for (int w = 0; w < 2; ++w) {
            double ph[6] = {0, 0, 0, 0, 0, 0};
            int steps = 0;
            for (int j = 0; j + 1 < std::min(n - 2, 64); ++j) {
                const unsigned long long* a = hst.data() + 384 * w + 6 * j;
                const unsigned long long nxt = a[6];
                if (!a[0] || !nxt) continue;
                ph[0] += double(a[1] - a[0]); ph[1] += double(a[2] - a[1]); ph[2] += double(a[3] - a[2]);
                ph[3] += double(a[4] - a[3]); ph[4] += double(a[5] - a[4]); ph[5] += double(nxt - a[5]);
                ++steps;
            }
            std::fprintf(stderr, "k_sytrd n=%d thread %d: mean cycles per step over %d: barrier1 %.0f reflector %.0f barrier2 %.0f symv %.0f barrier3 %.0f update %.0f\n",
                         n, w ? 64 : 0, steps, ph[0] / steps, ph[1] / steps, ph[2] / steps, ph[3] / steps, ph[4] / steps, ph[5] / steps);
        }
    }
    if (S) {
        hipLaunchKernelGGL(k_sqrt_lam, dim3((kk + 255) / 256), dim3(256), 0, h->stream, lm, kk, S);
        check_launch("k_sqrt_lam");
    }
}

}  // namespace xrs
