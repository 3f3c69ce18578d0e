// TT hot path on device: move_core (transfer_core sweeps), round (orthogonalise + truncate), <x,y>.
//
// Reference: TTNetwork::move_core (ttNetwork.cpp:582-628) -> TensorNetwork::transfer_core
// (tensorNetwork.cpp:821-909); TTNetwork::round (ttNetwork.cpp:644-665) -> round_edge
// (tensorNetwork.cpp:678-818); <x,y> = value_t(x(i&0)*y(i&0)).
//
// Cores live in HBM for the whole sweep; core k is (r[k], n[k], r[k+1]) row-major. Every matricisation
// used here is a free reshape of that layout, so — unlike the reference, which reshuffles the zipper
// intermediates (27 permutations per <x,y>) — no permutation kernel is needed on the TT path: the GEMM
// transpose flags absorb them.
//
// round(): the left-to-right sweep orthogonalises with CholeskyQR2 (certified) instead of pivoted QR;
// the right-to-left sweep factors each core B = L Q (wide CholeskyQR2) and takes the SVD of the small
// r x r factor L, whose singular values are those of the unfolding (the reference computes them as the
// SVD of C_f^T C_t^T, round_edge :745-779 — identical values because the left core is orthogonal).
// When the factorisation is certified (sigma_min >= c ||B||_F, see linalg.hip), eps < c and
// max_rank >= r, no singular value can be cut, so the SVD is skipped and B = L Q is used directly:
// same represented tensor, same ranks, different (equally valid) orthogonal gauge.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <limits>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#include "tt_common.hpp"

namespace xrs {

namespace ttd {


// reduce_to_maximal_ranks (ttNetwork.cpp:370-402)
std::vector<size_t> maximal_ranks(const TT& t) {
    std::vector<size_t> rk(t.r + 1, t.r + t.d);  // internal ranks r[1..d-1]
    size_t cur = 1;
    for (size_t i = 0; i + 1 < t.d; ++i) {
        cur *= t.n[i];
        if (cur < rk[i]) rk[i] = cur;
        else cur = rk[i];
    }
    cur = 1;
    for (size_t i = 1; i < t.d; ++i) {
        cur *= t.n[t.d - i];
        if (cur < rk[t.d - i - 1]) rk[t.d - i - 1] = cur;
        else cur = rk[t.d - i - 1];
    }
    return rk;
}

bool exceeds_maximal_ranks(const TT& t) {
    const auto mx = maximal_ranks(t);
    for (size_t i = 0; i + 1 < t.d; ++i)
        if (t.r[i + 1] != mx[i]) return true;
    return false;
}

// transfer_core(k -> k+1): posA = last mode -> QC (or QR), posB = 0 -> R * next (tensorNetwork.cpp:842-848, 873)
void transfer_right(TT& t, size_t k, bool rank_reduce) {
    const size_t m = t.rows_left(k), nn = t.r[k + 1], kmax = std::min(m, nn);
    double* Q = t.alloc(m * kmax);
    double* C = t.alloc(kmax * nn);
    size_t rank = kmax;
    if (rank_reduce) rank = qc(t.h, t.core[k], m, nn, Q, C);
    else qr(t.h, t.core[k], m, nn, Q, C);
    const size_t ncols = t.cols_right(k + 1);
    double* nxt = t.alloc(rank * ncols);
    gemm(t.h, nxt, rank, ncols, 1.0, C, nn, false, nn, t.core[k + 1], ncols, false);
    t.release(C);
    t.replace(k, Q);
    t.replace(k + 1, nxt);
    t.r[k + 1] = rank;
}

// transfer_core(k -> k-1): posA = 0 -> CQ (or RQ), posB = last -> prev * R (tensorNetwork.cpp:833-840, 875)
void transfer_left(TT& t, size_t k, bool rank_reduce) {
    const size_t m = t.r[k], nn = t.cols_right(k), kmax = std::min(m, nn);
    double* C = t.alloc(m * kmax);
    double* Q = t.alloc(kmax * nn);
    size_t rank = kmax;
    if (rank_reduce) rank = cq(t.h, t.core[k], m, nn, C, Q);
    else rq(t.h, t.core[k], m, nn, C, Q);
    const size_t prow = t.rows_left(k - 1);
    double* prv = t.alloc(prow * rank);
    gemm(t.h, prv, prow, rank, 1.0, t.core[k - 1], m, false, m, C, rank, false);
    t.release(C);
    t.replace(k, Q);
    t.replace(k - 1, prv);
    t.r[k] = rank;
}

void move_core(TT& t, bool canonicalized, size_t core_pos, size_t pos, bool keep_rank) {
    const size_t d = t.d;
    if (canonicalized) {
        for (size_t k = core_pos; k < pos; ++k) transfer_right(t, k, !keep_rank);
        for (size_t k = core_pos; k > pos; --k) transfer_left(t, k, !keep_rank);
    } else {
        for (size_t k = 0; k < pos; ++k) transfer_right(t, k, !keep_rank);
        for (size_t k = d - 1; k > pos; --k) transfer_left(t, k, !keep_rank);
    }
    while (exceeds_maximal_ranks(t)) {   // ttNetwork.cpp:609-624
        for (size_t k = pos; k > 0; --k) transfer_left(t, k, !keep_rank);
        for (size_t k = 0; k + 1 < d; ++k) transfer_right(t, k, !keep_rank);
        for (size_t k = d - 1; k > pos; --k) transfer_left(t, k, !keep_rank);
    }
}

// left-orthogonalise core k into k+1 (round's canonicalisation sweep, canonicalize_right ->
// transfer_core(allowRankReduction = true), tensorNetwork.cpp:842-848): QC with the reference's rank rule
// |R_kk| < 16 eps R_00 (blasLapackWrapper.cpp:268-272); a certified unfolding keeps its rank without pivoting
void orth_right(TT& t, size_t k) { transfer_right(t, k, true); }

// svd rank cut of calculate_svd (tensor.cpp:1462-1474): max_rank, then first sigma_j <= eps*sigma_0
size_t svd_cut(const std::vector<double>& s, size_t max_rank, double eps) {
    size_t rank = s.size();
    if (max_rank != 0) rank = std::min(rank, max_rank);
    for (size_t j = 1; j < rank; ++j)
        if (s[j] <= eps * s[0]) return j;
    return rank;
}

// T[:, j] *= ratio_j = max(0, S_j - soft) / S_j (0 for S_j == 0): (U S) -> (U S') with the soft threshold
__global__ void k_soft_cols(double* __restrict__ T, const double* __restrict__ S, size_t rows, size_t cols, double soft) {
    for (size_t e = size_t(blockIdx.x) * blockDim.x + threadIdx.x; e < rows * cols; e += size_t(gridDim.x) * blockDim.x) {
        const double s = S[e % cols];
        T[e] = s > 0.0 ? T[e] * (fmax(0.0, s - soft) / s) : 0.0;
    }
}

// truncate the edge between core k-1 and core k (round_edge(k, k-1), core moves to k-1):
// B = core_k (m x nn) = L Q (wide) or Q R (tall), F the triangular factor (g x g, g = min(m, nn) <= 1024),
// F = U S V^T with V from one-sided Jacobi (jacobi_right_vectors: accumulated rotations on the columns of a
// wide L, the rows of a tall R; accurate to u for every singular value);
// the reference's cut (tensor.cpp:1462-1474) on S; core_k <- V_kk^T Q (wide) / V_kk^T (tall),
// core_{k-1} <- core_{k-1} (F V_kk) / (B V_kk) = core_{k-1} (U S)_kk, with max(0, S - soft) for soft > 0
void truncate_edge(TT& t, size_t k, size_t max_rank, double eps, double soft) {
    const size_t m = t.r[k], nn = t.cols_right(k);
    const size_t prow = t.rows_left(k - 1);
    xrs_handle_t h = t.h;
    const bool wide = m <= nn;
    const size_t g = wide ? m : nn;
    XRS_REQUIRE(g <= kHugeMax, "TT round: an edge whose unfoldings both exceed 1024 is not supported");
    double* Q = t.alloc(m * nn);
    double* F = t.alloc(g * g);
    const OrthResult o = orthogonalize(h, t.core[k], m, nn, wide, Q, F);
    if (wide && o.certified && eps < 0.5 * o.cert_ratio && max_rank >= m && !(soft > 0.0)) {
        double* prv = t.alloc(prow * m);   // no singular value can be cut: B = L Q directly
        gemm(h, prv, prow, m, 1.0, t.core[k - 1], m, false, m, F, m, false);
        t.release(F);
        t.replace(k, Q);
        t.replace(k - 1, prv);
        return;
    }
    DevBuf S(h, g * 8), Vt(h, g * g * 8), st(h, 64);
    XRS_HIP(hipMemsetAsync(st.d(), 0, 64, h->stream));
    jacobi_right_vectors(h, F, int(g), wide, S.d(), Vt.d(), st.as<int>(), 60);
    // -2 (a grid-barrier poll of the block kernel timed out) leaves S / Vt invalid: recomputed on the rows of
    // F; other negative statuses are non-convergence warnings, as the reference's dgesdd failure
    // (blasLapackWrapper.cpp:216-224)
    jacobi_settle(h, st.as<int>(), int(g), int(g), [&](int kernel) {
        jacobi_vt(h, F, int(g), false, int(g), int(g), S.d(), Vt.d(), int(g), st.as<int>(), 60, kernel);
    });
    std::vector<double> s(g);
    XRS_HIP(hipMemcpyAsync(s.data(), S.d(), g * 8, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    const size_t kk = svd_cut(s, max_rank, eps);
    double* T = t.alloc(m * kk);
    if (wide) gemm(h, T, m, kk, 1.0, F, g, false, g, Vt.d(), g, true);          // L V_kk = (U S)_kk
    else gemm(h, T, m, kk, 1.0, t.core[k], nn, false, nn, Vt.d(), g, true);     // B V_kk
    if (soft > 0.0) {
        hipLaunchKernelGGL(k_soft_cols, dim3(unsigned(std::min<size_t>((m * kk + 255) / 256, 4096))), dim3(256), 0, h->stream, T, S.d(), m, kk,
                           soft);
        check_launch("k_soft_cols");
    }
    double* cur = t.alloc(kk * nn);
    if (wide) gemm(h, cur, kk, nn, 1.0, Vt.d(), g, false, g, Q, nn, false);     // V_kk^T Q
    else XRS_HIP(hipMemcpyAsync(cur, Vt.d(), kk * nn * 8, hipMemcpyDeviceToDevice, h->stream));
    double* prv = t.alloc(prow * kk);
    gemm(h, prv, prow, kk, 1.0, t.core[k - 1], m, false, m, T, kk, false);
    t.release(T);
    t.release(F);
    t.release(Q);
    t.replace(k, cur);
    t.replace(k - 1, prv);
    t.r[k] = kk;
}

// ---- certified fast path of round() ------------------------------------------------------------
// round() can only change the tensor through a cut: a QC rank drop in the left-to-right sweep
// (|R_kk| < 16 eps R_00, blasLapackWrapper.cpp:268-272) or an SVD cut in round_edge (sigma_j <= eps
// sigma_0 or j >= maxRank, tensor.cpp:1462-1474). When the ranks are within maxRanks and every edge
// unfolding U_k = X_{<k} X_{>=k} is provably well conditioned, neither can happen, and the result is
// the input tensor in right-canonical form (core at 0) with the same ranks -- what one right-to-left
// orthogonalisation sweep produces. Proof obligations:
//   kappa(X_{<k}) <= 1/c_X: Gram G_k = X_{<k}^T X_{<k} built by the left chain G_{k+1} = M^T (G_k M)
//   from the ORIGINAL cores, then a Cholesky of G_k - tau tr(G_k) I succeeding for every k (one batched
//   launch) gives lambda_min(G_k) >= (tau - rounding) tr(G_k) >= tau/4 tr(G_k), c_X = sqrt(tau)/2;
//   kappa(L_k) <= 1/c_L from the certified LQ of core k (orthogonalize);
//   then sigma_min(U)/sigma_max(U) >= c_X c_L > eps (>= 16 eps needed for the QC rule too, since
//   |R_kk| >= sigma_min for any triangular factor).
// Any failed obligation falls back to the reference's two-sweep algorithm, from the failing edge on.

// Gram chains from the current cores (k = 1..d-1, index k):
//   left  G_k = X_{<k}^T X_{<k}:  G_1 = M_0^T M_0, G_{k+1} = M_k^T (G_k M_k)   (M_k: r_k x n_k r_{k+1})
//   right H_k = X_{>=k} X_{>=k}^T: H_{d-1} = M M^T, H_k = M_k (I (x) H_{k+1}) M_k^T
void left_gram_step(TT& t, std::vector<double*>& G, double* T, size_t k, bool do_reduce) {   // G_{k+1} from G_k
    xrs_handle_t h = t.h;
    if (k == 0) {
        gemm_sym(h, G[1], t.r[1], 1.0, t.core[0], t.r[1], true, t.rows_left(0), t.core[0], t.r[1], false);
        if (do_reduce) t.reduce(G[1], t.r[1] * t.r[1]);
        return;
    }
    const size_t a = t.r[k], b = t.r[k + 1], cols = t.cols_right(k);
    gemm(h, T, a, cols, 1.0, G[k], a, false, a, t.core[k], cols, false);
    gemm_sym(h, G[k + 1], b, 1.0, t.core[k], b, true, a * t.n[k], T, b, false);   // M^T (G M): symmetric
    if (do_reduce) t.reduce(G[k + 1], b * b);
}

void right_gram_step(TT& t, std::vector<double*>& H, double* T, size_t k, bool do_reduce) {   // H_k from H_{k+1}
    xrs_handle_t h = t.h;
    const size_t last = t.d - 1;
    if (k == last) {
        const size_t cl = t.cols_right(last);
        gemm_sym(h, H[last], t.r[last], 1.0, t.core[last], cl, false, cl, t.core[last], cl, true);
        if (do_reduce) t.reduce(H[last], t.r[last] * t.r[last]);
        return;
    }
    const size_t a = t.r[k], b = t.r[k + 1], cols = t.cols_right(k);
    gemm(h, T, a * t.n[k], b, 1.0, t.core[k], b, false, b, H[k + 1], b, false);   // M_k(rn x r') H
    gemm_sym(h, H[k], a, 1.0, t.core[k], cols, false, cols, T, cols, true);        // M_k T^T: symmetric
    if (do_reduce) t.reduce(H[k], a * a);
}

// Both chains (G: left Grams, only with `left`; H: right Grams; `store` owns the memory). Unsharded,
// concurrently (left on a side stream, right on the main stream) with their launches interleaved step by
// step. (Both chains' products as one two-entry grid on one stream measured slower: one chain's split-K
// reduce and boundary products no longer overlap the other chain's GEMMs) Sharded, step s of
// both chains shares ONE all-reduce: G_{s+1} and H_{d-1-s} sit side by side in one buffer, the two steps
// forked onto two streams and joined before it.
void gram_chains(TT& t, std::vector<double*>& G, std::vector<double*>& H, std::vector<DevBuf>& store, bool left) {
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    G.assign(d, nullptr);
    H.assign(d, nullptr);
    size_t tmax = 1;
    for (size_t k = 1; k + 1 < d; ++k) tmax = std::max(tmax, t.size(k));
    DevBuf TL(h, tmax * 8), TR(h, tmax * 8);
    if (t.sharded()) {
        for (size_t s = 0; s + 1 < d; ++s) {
            const size_t kl = s + 1, kr = d - 1 - s;
            const size_t nl = left ? t.r[kl] * t.r[kl] : 0, nr = t.r[kr] * t.r[kr];
            store.emplace_back(h, (nl + nr) * 8);
            double* base = store.back().d();
            if (left) G[kl] = base;
            H[kr] = base + nl;
            if (left) {   // the two chains' steps concurrently (left on a side stream), joined before the all-reduce
                StreamFork fork(h);
                fork.side();
                left_gram_step(t, G, TL.d(), s, false);
                fork.main();
                right_gram_step(t, H, TR.d(), kr, false);
                fork.join();
            } else {
                right_gram_step(t, H, TR.d(), kr, false);
            }
            t.reduce(base, nl + nr);
        }
        return;
    }
    for (size_t k = 1; k < d; ++k) {
        if (left) {
            store.emplace_back(h, t.r[k] * t.r[k] * 8);
            G[k] = store.back().d();
        }
        store.emplace_back(h, t.r[k] * t.r[k] * 8);
        H[k] = store.back().d();
    }
    if (!left) {
        for (size_t k = d - 1; k >= 1; --k) right_gram_step(t, H, TR.d(), k);
        return;
    }
    StreamFork fork(h);
    for (size_t s = 0; s + 1 < d; ++s) {
        fork.side();
        left_gram_step(t, G, TL.d(), s);
        fork.main();
        right_gram_step(t, H, TR.d(), d - 1 - s);
    }
    fork.join();
}

// Host-side phase timestamps of round() (XRS_STAMPS=round: one stderr line per round; diagnostics only)
struct HostMarks {
    bool on = stamps_enabled("round");
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    std::string line;
    void mark(const char* what) {
        if (!on) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        char buf[64];
        std::snprintf(buf, sizeof(buf), " %s %.0f", what, us);
        line += buf;
    }
    ~HostMarks();
};
HostMarks* g_marks = nullptr;
HostMarks::~HostMarks() {
    if (g_marks == this) g_marks = nullptr;
    if (on) std::fprintf(stderr, "[round host us]%s\n", line.c_str());
}
#define XRS_MARK(what) do { if (g_marks) g_marks->mark(what); } while (0)


// max |G_i - I| of a batch of square matrices, one workgroup each
__global__ void __launch_bounds__(256) k_dev_identity_many(const DevIdArgs args) {
    const double* G = args.G[blockIdx.x];
    const int n = args.n[blockIdx.x];
    __shared__ double red[4];
    double mx = 0.0;
    for (int e = threadIdx.x + 256 * blockIdx.y; e < n * n; e += 256 * gridDim.y) {
        const double v = fabs(G[e] - ((e / n) == (e % n) ? 1.0 : 0.0));
        mx = (v > mx || v != v) ? v : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double q = __shfl_xor(mx, o, 64);
        mx = (q > mx || q != q) ? q : mx;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = red[0];
        for (int i = 1; i < 4; ++i) m = (red[i] > m || red[i] != red[i]) ? red[i] : m;
        args.out[blockIdx.x * gridDim.y + blockIdx.y] = m;
    }
}

void rl_sweep(TT& t, const size_t* max_ranks, double eps, double cX, size_t from);


// One chain orthogonalisation pass over the current cores: the right Gram chain H_k (and, with
// `certify`, the left chain G_k), ONE batched launch of all Cholesky factorisations -- H_k = L_k L_k^T
// (out of place, into L_k) and, with `certify`, the down-shifted certificates of G_k and H_k (status
// only) -- then every core is transformed independently: C_k = L_k^{-1} M_k (I (x) L_{k+1}),
// C_0 = M_0 (I (x) L_1). In exact arithmetic the C_k (k >= 1) have orthonormal rows and represent the
// same tensor. Nothing is synchronised: the factorisation statuses are copied to pinned host memory
// behind the transforms and judged by chain_check (a failed factorisation only makes C garbage, which
// is then discarded).
// Independent GEMMs; the ones of identical shape go out as one batched launch.

void gemm_grouped(xrs_handle_t h, const std::vector<GemmJob>& jobs) {
    std::vector<bool> done(jobs.size(), false);
    for (size_t i = 0; i < jobs.size(); ++i) {
        if (done[i]) continue;
        const GemmJob& g = jobs[i];
        std::vector<const double*> A, B;
        std::vector<double*> C;
        for (size_t j = i; j < jobs.size(); ++j) {
            const GemmJob& o = jobs[j];
            if (done[j] || o.M != g.M || o.N != g.N || o.K != g.K || o.lda != g.lda || o.ldb != g.ldb || o.ta != g.ta ||
                o.tb != g.tb || o.sym != g.sym || o.alpha != g.alpha || o.tri != g.tri)
                continue;
            done[j] = true;
            A.push_back(o.A);
            B.push_back(o.B);
            C.push_back(o.C);
        }
        if (C.size() == 1 && g.sym) gemm_sym(h, C[0], g.N, g.alpha, A[0], g.lda, g.ta, g.K, B[0], g.ldb, g.tb);
        else if (C.size() == 1) gemm(h, C[0], g.M, g.N, g.alpha, A[0], g.lda, g.ta, g.K, B[0], g.ldb, g.tb, g.tri);
        else gemm_batched(h, int(C.size()), C.data(), g.M, g.N, g.alpha, A.data(), g.lda, g.ta, g.K, B.data(), g.ldb,
                          g.tb, g.sym, g.tri);
    }
}

// ---- Cholesky for 256 < n <= 512 from the n <= 256 kernels (2 x 2 blocks, n1 = 256, n2 = n - 256):
//   W = A + shift*I (shift = shift_rel tr A), L11 = chol(W11), Z11 = L11^{-1}, L21 = W21 Z11^T,
//   L22 = chol(W22 - L21 L21^T); factor jobs also get L = [L11 0; L21 L22] and
//   Z = L^{-1} = [Z11 0; -Z22 L21 Z11, Z22]. Every step is one batched launch over all jobs, so the
//   latency is two 256-Cholesky + two 256-inverses instead of one 512-column sequential sweep
//   (k_potrf32_batched + k_trinv_batched<32>: 1.1 ms per cfg5 pass).
struct BigArgs {
    const double* src[kBigMax];
    double* w11[kBigMax];
    double* w21[kBigMax];
    double* w22[kBigMax];
    double shift[kBigMax];
    int n[kBigMax];
};

__global__ void __launch_bounds__(256) k_split_shift(const BigArgs a) {
    const int j = blockIdx.y, n = a.n[j], n1 = 256, n2 = n - 256;
    const double* A = a.src[j];
    __shared__ double red[4];
    double tr = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) tr += A[size_t(i) * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = tr;
    __syncthreads();
    const double shift = a.shift[j] * (red[0] + red[1] + red[2] + red[3]);
    const size_t total = size_t(n) * n;
    for (size_t e = size_t(blockIdx.x) * 256 + threadIdx.x; e < total; e += size_t(gridDim.x) * 256) {
        const int r = int(e / n), c = int(e - size_t(r) * n);
        const double v = A[e] + (r == c ? shift : 0.0);
        if (r < n1 && c < n1) a.w11[j][size_t(r) * n1 + c] = v;
        else if (r >= n1 && c < n1) a.w21[j][size_t(r - n1) * n1 + c] = v;
        else if (r >= n1 && c >= n1) a.w22[j][size_t(r - n1) * n2 + (c - n1)] = v;
    }
}

struct SubArgs {
    double* y[kBigMax];
    const double* x[kBigMax];
    int count[kBigMax];
};

__global__ void __launch_bounds__(256) k_sub_batched(const SubArgs a) {   // y -= x
    const int j = blockIdx.y;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < a.count[j]; e += gridDim.x * 256) a.y[j][e] -= a.x[j][e];
}

struct AssembleArgs {
    double* out[kBigMax];   // n x n
    const double* b11[kBigMax];
    const double* b21[kBigMax];
    const double* b22[kBigMax];
    int n[kBigMax];
};

__global__ void __launch_bounds__(256) k_assemble_lower(const AssembleArgs a) {   // [B11 0; B21 B22]
    const int j = blockIdx.y, n = a.n[j], n1 = 256, n2 = n - 256;
    const size_t total = size_t(n) * n;
    for (size_t e = size_t(blockIdx.x) * 256 + threadIdx.x; e < total; e += size_t(gridDim.x) * 256) {
        const int r = int(e / n), c = int(e - size_t(r) * n);
        double v = 0.0;
        if (r < n1) v = c < n1 ? a.b11[j][size_t(r) * n1 + c] : 0.0;
        else v = c < n1 ? a.b21[j][size_t(r - n1) * n1 + c] : a.b22[j][size_t(r - n1) * n2 + (c - n1)];
        a.out[j][e] = v;
    }
}


// Enqueues every job; statuses (2 per job: the two diagonal factorisations) go to status[0 .. 2*jobs).
void factor_big(xrs_handle_t h, const std::vector<BigJob>& jobs, int* status, std::vector<DevBuf>& keep) {
    const int nj = int(jobs.size());
    XRS_REQUIRE(nj <= kBigMax, "factor_big: too many jobs");
    constexpr int n1 = 256;
    BigArgs ba{};
    std::vector<double*> w11(nj), w21(nj), w22(nj), d11(nj), d22(nj), z11(nj), pp(nj);
    auto buf = [&](size_t elems) { keep.emplace_back(h, std::max<size_t>(elems, 1) * 8); return keep.back().d(); };
    size_t maxn2 = 0;
    for (int j = 0; j < nj; ++j) {
        const int n = jobs[j].n, n2 = n - n1;
        XRS_REQUIRE(n > n1 && n <= 2 * n1, "factor_big: n out of range");
        w11[j] = buf(size_t(n1) * n1);
        w21[j] = buf(size_t(n2) * n1);
        w22[j] = buf(size_t(n2) * n2);
        d11[j] = buf(dinv_elems(n1));
        d22[j] = buf(dinv_elems(n2));
        z11[j] = buf(size_t(n1) * n1);
        pp[j] = buf(size_t(n2) * n2);
        ba.src[j] = jobs[j].src;
        ba.w11[j] = w11[j];
        ba.w21[j] = w21[j];
        ba.w22[j] = w22[j];
        ba.shift[j] = jobs[j].shift_rel;
        ba.n[j] = n;
        maxn2 = std::max(maxn2, size_t(n2));
    }
    hipLaunchKernelGGL(k_split_shift, dim3(256, nj), dim3(256), 0, h->stream, ba);
    check_launch("k_split_shift");
    auto chol = [&](const std::vector<double*>& W, const std::vector<double*>& D, int first_slot, bool upper_half) {
        for (int b0 = 0; b0 < nj; b0 += kPotrfBatchMax) {
            PotrfBatch pb{};
            const int c = std::min(kPotrfBatchMax, nj - b0);
            for (int i = 0; i < c; ++i) {
                pb.src[i] = nullptr;
                pb.G[i] = W[b0 + i];
                pb.Dinv[i] = D[b0 + i];
                pb.shift[i] = 0.0;
                pb.n[i] = upper_half ? n1 : jobs[b0 + i].n - n1;
            }
            pb.status = status + first_slot + b0;
            potrf_batched(h, pb, c);
        }
    };
    auto inverse = [&](const std::vector<double*>& L, const std::vector<double*>& D, const std::vector<double*>& X,
                       bool upper_half, const std::vector<int>& which) {
        TrinvBatch tb{};
        int c = 0;
        for (int j : which) {
            tb.L[c] = L[j];
            tb.Dinv[c] = D[j];
            tb.X[c] = X[j];
            tb.n[c] = upper_half ? n1 : jobs[j].n - n1;
            ++c;
        }
        if (c) trinv_batched(h, tb, c);
    };
    std::vector<int> all(nj), fac;
    for (int j = 0; j < nj; ++j) {
        all[j] = j;
        if (jobs[j].L) fac.push_back(j);
    }
    chol(w11, d11, 0, true);                     // L11 in w11
    inverse(w11, d11, z11, true, all);           // Z11
    std::vector<GemmJob> g1, g2;
    for (int j = 0; j < nj; ++j) {
        const size_t n2 = size_t(jobs[j].n - n1);
        g1.push_back({n2, size_t(n1), size_t(n1), size_t(n1), size_t(n1), false, true, w21[j], z11[j], w21[j] == nullptr ? nullptr : buf(n2 * n1)});
    }
    // L21 = W21 Z11^T into fresh buffers (GEMM outputs must not alias inputs)
    std::vector<double*> l21(nj);
    for (int j = 0; j < nj; ++j) l21[j] = g1[j].C;
    gemm_grouped(h, g1);
    for (int j = 0; j < nj; ++j) {
        const size_t n2 = size_t(jobs[j].n - n1);
        g2.push_back({n2, n2, size_t(n1), size_t(n1), size_t(n1), false, true, l21[j], l21[j], pp[j], true});
    }
    gemm_grouped(h, g2);                         // P = L21 L21^T (symmetric)
    SubArgs sa{};
    for (int j = 0; j < nj; ++j) {
        sa.y[j] = w22[j];
        sa.x[j] = pp[j];
        sa.count[j] = (jobs[j].n - n1) * (jobs[j].n - n1);
    }
    hipLaunchKernelGGL(k_sub_batched, dim3(64, nj), dim3(256), 0, h->stream, sa);
    check_launch("k_sub_batched");
    chol(w22, d22, nj, false);                   // L22 in w22
    if (fac.empty()) return;
    std::vector<double*> z22(nj, nullptr), tt(nj, nullptr), z21(nj, nullptr);
    for (int j : fac) {
        const size_t n2 = size_t(jobs[j].n - n1);
        z22[j] = buf(n2 * n2);
        tt[j] = buf(n2 * n1);
        z21[j] = buf(n2 * n1);
    }
    inverse(w22, d22, z22, false, fac);          // Z22
    std::vector<GemmJob> g3, g4;
    for (int j : fac) {
        const size_t n2 = size_t(jobs[j].n - n1);
        g3.push_back({n2, size_t(n1), size_t(n1), size_t(n1), size_t(n1), false, false, l21[j], z11[j], tt[j]});
    }
    gemm_grouped(h, g3);                         // T = L21 Z11
    for (int j : fac) {
        const size_t n2 = size_t(jobs[j].n - n1);
        GemmJob g{n2, size_t(n1), n2, n2, size_t(n1), false, false, z22[j], tt[j], z21[j]};
        g.alpha = -1.0;
        g4.push_back(g);
    }
    gemm_grouped(h, g4);                         // Z21 = -Z22 T
    AssembleArgs al{}, az{};
    int c = 0;
    for (int j : fac) {
        al.out[c] = jobs[j].L; al.b11[c] = w11[j]; al.b21[c] = l21[j]; al.b22[c] = w22[j]; al.n[c] = jobs[j].n;
        az.out[c] = jobs[j].Z; az.b11[c] = z11[j]; az.b21[c] = z21[j]; az.b22[c] = z22[j]; az.n[c] = jobs[j].n;
        ++c;
    }
    hipLaunchKernelGGL(k_assemble_lower, dim3(256, c), dim3(256), 0, h->stream, al);
    check_launch("k_assemble_lower");
    hipLaunchKernelGGL(k_assemble_lower, dim3(256, c), dim3(256), 0, h->stream, az);
    check_launch("k_assemble_lower");
}

struct ChainPass {
    std::vector<double*> C;   // new cores (owned by the TT's pool until replaced / released)
    int* status = nullptr;    // pinned host copy of the factorisation statuses
    int count = 0;
    bool certify = false;
};

void chain_pass(TT& t, bool certify, ChainPass& out, int* host_status) {
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    std::vector<double*> G, H;
    std::vector<DevBuf> gram_store, Lf(d), Cs;
    XRS_MARK("pass");
    gram_chains(t, G, H, gram_store, certify);
    open_dot_gate(h);   // a gated async <x,y> runs beside the factorisations and transforms below
    XRS_MARK("chains");
    // edges with r <= 256: one batched register-resident launch; larger (<= 512): factor_big (2 x 2
    // blocks of the same kernels), which also delivers Z = L^{-1}
    std::vector<DevBuf> Z(d);
    for (size_t k = 1; k < d; ++k) Z[k] = DevBuf(h, t.r[k] * t.r[k] * 8);
    size_t dsz = 0;
    for (size_t k = 1; k < d; ++k)
        if (t.r[k] <= 256) dsz += dinv_elems(int(t.r[k]));
    std::vector<double*> dinv(d, nullptr);
    struct Job { const double* src; double* G; double* Dinv; double shift; int n; };
    std::vector<Job> jobs;
    std::vector<BigJob> big, huge;   // huge: r > 512, blocked Cholesky one job at a time
    DevBuf Dv(h, dsz * 8 + 8), Dscr(h, (certify ? 2 * dsz : 1) * 8 + 8);
    size_t off = 0;
    for (size_t k = 1; k < d; ++k) {
        const size_t a = t.r[k];
        Lf[k] = DevBuf(h, a * a * 8);
        if (a > 512) {
            huge.push_back({H[k], 0.0, int(a), Lf[k].d(), Z[k].d()});
            if (certify) {
                huge.push_back({G[k], -kGramShift, int(a), nullptr, nullptr});
                huge.push_back({H[k], -kGramShift, int(a), nullptr, nullptr});
            }
            continue;
        }
        if (a > 256) {
            big.push_back({H[k], 0.0, int(a), Lf[k].d(), Z[k].d()});
            if (certify) {
                big.push_back({G[k], -kGramShift, int(a), nullptr, nullptr});
                big.push_back({H[k], -kGramShift, int(a), nullptr, nullptr});
            }
            continue;
        }
        const size_t de = dinv_elems(int(a));
        dinv[k] = Dv.d() + off;
        jobs.push_back({H[k], Lf[k].d(), dinv[k], 0.0, int(a)});
        if (certify) {   // status-only certificates
            jobs.push_back({G[k], nullptr, Dscr.d() + 2 * off, -kGramShift, int(a)});
            jobs.push_back({H[k], nullptr, Dscr.d() + 2 * off + de, -kGramShift, int(a)});
        }
        off += de;
    }
    const int cnt_small = int(jobs.size());
    int cnt_huge = 0;
    for (const BigJob& j : huge) cnt_huge += chol_full_blocks(size_t(j.n));
    const int cnt = cnt_small + 2 * int(big.size()) + cnt_huge;
    DevBuf st(h, size_t(cnt) * 4 + 64);
    {
        int slot = cnt_small + 2 * int(big.size());
        for (const BigJob& j : huge) {
            chol_full(h, j.src, size_t(j.n), j.shift_rel, j.L, j.Z, st.as<int>() + slot);
            slot += chol_full_blocks(size_t(j.n));
        }
    }
    for (size_t b0 = 0; b0 < big.size(); b0 += kBigMax) {   // chunks of the kernels' argument tables
        const std::vector<BigJob> part(big.begin() + long(b0), big.begin() + long(std::min(big.size(), b0 + kBigMax)));
        factor_big(h, part, st.as<int>() + cnt_small + 2 * b0, Cs);
    }
    for (int b0 = 0; b0 < cnt_small; b0 += kPotrfBatchMax) {
        PotrfBatch pb{};
        const int c = std::min(kPotrfBatchMax, cnt_small - b0);
        for (int i = 0; i < c; ++i) {
            pb.src[i] = jobs[b0 + i].src;
            pb.G[i] = jobs[b0 + i].G;
            pb.Dinv[i] = jobs[b0 + i].Dinv;
            pb.shift[i] = jobs[b0 + i].shift;
            pb.n[i] = jobs[b0 + i].n;
        }
        pb.status = st.as<int>() + b0;
        potrf_batched(h, pb, c);
    }
    XRS_HIP(hipMemcpyAsync(host_status, st.d(), size_t(cnt) * 4, hipMemcpyDeviceToHost, h->stream));
    XRS_MARK("potrf");
    out.status = host_status;
    out.count = cnt;
    out.certify = certify;
    // The d transforms are independent: same-shape GEMMs go out as one batched launch each, all on the
    // main stream (cross-stream event hops cost ~20 us each here; a batch fills the chip as well as
    // concurrent streams do). The left factor is applied as a GEMM with the explicit inverse
    // Z_k = L_k^{-1} (one batched launch); the check below certifies the result either way.
    out.C.assign(d, nullptr);
    std::vector<DevBuf> W(d);
    TrinvBatch tb{};
    int ninv = 0;
    for (size_t k = 0; k < d; ++k) {
        out.C[k] = t.alloc(t.size(k));
        if (k > 0 && k + 1 < d) W[k] = DevBuf(h, t.size(k) * 8);
        if (k > 0 && t.r[k] <= 256) {   // (r > 256: Z came from factor_big)
            tb.L[ninv] = Lf[k].d();
            tb.Dinv[ninv] = dinv[k];
            tb.X[ninv] = Z[k].d();
            tb.n[ninv] = int(t.r[k]);
            ++ninv;
        }
    }
    for (int b0 = 0; b0 < ninv; b0 += kTrinvBatchMax) {
        TrinvBatch part{};
        const int c = std::min(kTrinvBatchMax, ninv - b0);
        for (int i = 0; i < c; ++i) {
            part.L[i] = tb.L[b0 + i];
            part.Dinv[i] = tb.Dinv[b0 + i];
            part.X[i] = tb.X[b0 + i];
            part.n[i] = tb.n[b0 + i];
        }
        trinv_batched(h, part, c);
    }
    // L_k and Z_k of the register-resident kernels (r <= 256) hold exact zeros above the diagonal: their
    // zero K-blocks are skipped (5/8 of the work at r = 256)
    std::vector<GemmJob> right, left;
    for (size_t k = 0; k + 1 < d; ++k) {   // right factors: M_k (I (x) L_{k+1}), (r_k n_k) x r_{k+1} x r_{k+1}
        const size_t b = t.r[k + 1];
        right.push_back({t.rows_left(k), b, b, b, b, false, false, t.core[k], Lf[k + 1].d(), k == 0 ? out.C[k] : W[k].d()});
        right.back().tri = b <= 256 ? kTriB : 0;
    }
    for (size_t k = 1; k < d; ++k) {       // left factors: Z_k (r_k x r_k) times the r_k x (n_k r_{k+1}) unfolding
        const size_t a = t.r[k], cols = t.cols_right(k);
        left.push_back({a, cols, a, a, cols, false, false, Z[k].d(), k + 1 < d ? W[k].d() : t.core[k], out.C[k]});
        left.back().tri = a <= 256 ? kTriA : 0;
    }
    gemm_grouped(h, right);
    gemm_grouped(h, left);
    XRS_MARK("transforms");
}

// True when every factorisation of the pass succeeded (valid after the stream has been synchronised).
bool chain_status_ok(const ChainPass& p) {
    static const bool dbg = std::getenv("XRS_DEBUG_ROUND") != nullptr;
    const int per = p.certify ? 3 : 1;
    for (int i = 0; i < p.count; ++i)
        if (p.status[i] != 0) {
            if (dbg)
                std::fprintf(stderr, "chain_pass: factorisation %d of %d (%d per edge r <= 256, then 2 per r > 256 "
                             "job) failed at column %d\n", i, p.count, per, p.status[i]);
            return false;
        }
    return true;
}

// max_k max |C_k C_k^T - I| over cores 1..d-1 (mode sums completed across ranks when sharded).
// Synchronises the stream (so the pass statuses are readable afterwards).
double chain_check(TT& t, const std::vector<double*>& C) {
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    XRS_MARK("check");
    std::vector<double*> Gr(d, nullptr);
    DevIdArgs da{};
    DevBuf dev(h, d * 16 * 8 + 64);
    int nchk = 0;
    size_t gtot = 0;
    for (size_t k = 1; k < d; ++k) gtot += t.r[k] * t.r[k];
    DevBuf Gall(h, gtot * 8);   // contiguous: one all-reduce for every Gram when sharded
    for (size_t k = 1, off = 0; k < d; off += t.r[k] * t.r[k], ++k) Gr[k] = Gall.d() + off;
    std::vector<GemmJob> grams;
    for (size_t k = 1; k < d; ++k) {
        const size_t a = t.r[k], cols = t.cols_right(k);
        grams.push_back({a, a, cols, cols, cols, false, true, C[k], C[k], Gr[k], true});
    }
    gemm_grouped(h, grams);
    t.reduce(Gall.d(), gtot);   // sharded: complete the mode sums across ranks (no-op otherwise)
    for (size_t k = 1; k < d; ++k) {
        da.G[nchk] = Gr[k];
        da.n[nchk] = int(t.r[k]);
        ++nchk;
    }
    da.out = dev.d();
    constexpr int kSlices = 16;
    hipLaunchKernelGGL(k_dev_identity_many, dim3(nchk, kSlices), dim3(256), 0, h->stream, da);
    check_launch("k_dev_identity_many");
    double* hd = static_cast<double*>(h->host_scratch) + 64;
    XRS_HIP(hipMemcpyAsync(hd, dev.d(), size_t(nchk) * kSlices * 8, hipMemcpyDeviceToHost, h->stream));
    XRS_MARK("enq");
    host_wait(h);
    XRS_MARK("sync");
    double worst = 0.0;
    for (int i = 0; i < nchk * kSlices; ++i) worst = (hd[i] > worst || hd[i] != hd[i]) ? hd[i] : worst;
    return worst;
}

// Chain form of the certified round (no factorisation on a sequential chain): pass 1 certifies both
// chains and transforms the cores; the check confirms right-orthonormality. A chain pass loses about
// kappa^2 u, so an ill-conditioned input (e.g. a square unfolding) can miss the 1e-13 bar: pass 2
// repeats the right chain on the pass-1 cores (now near-orthonormal, so the chain is well conditioned)
// -- CholeskyQR2 applied to the whole train. Only if that also fails does the sequential sweep run.
// One host synchronisation per pass (the check).
bool round_chain(TT& t, const size_t* max_ranks, double eps) {
    const size_t d = t.d;
    static const bool dbg = std::getenv("XRS_DEBUG_ROUND") != nullptr;
    if (d < 2 || d > 65 || (!t.sharded() && exceeds_maximal_ranks(t))) return false;
    for (size_t k = 1; k < d; ++k)
        if (t.r[k] > max_ranks[k - 1] || t.r[k] > kHugeMax) return false;
    const double cX = 0.5 * std::sqrt(kGramShift);
    if (!(eps < 0.25 * cX * cX)) return false;
    // factorisation statuses (<= 3*64 ints) in a region of the pinned scratch no other routine uses
    int* hs = static_cast<int*>(t.h->host_scratch) + 12288;
    HostMarks marks;
    g_marks = marks.on ? &marks : nullptr;
    ChainPass p1;
    chain_pass(t, true, p1, hs);
    double dev = chain_check(t, p1.C);
    if (!chain_status_ok(p1)) {
        for (size_t k = 0; k < d; ++k) t.release(p1.C[k]);
        { g_marks = nullptr; return false; }
    }
    std::vector<double*> C = p1.C;
    if (!(dev <= kOrthTol)) {
        if (dbg) std::fprintf(stderr, "round_chain: pass 1 orthogonality %.3e, second pass\n", dev);
        TT t2 = t;
        t2.core = C.data();
        ChainPass p2;
        chain_pass(t2, false, p2, hs);
        const double dev2 = chain_check(t2, p2.C);
        const bool ok2 = chain_status_ok(p2);
        if (dbg) std::fprintf(stderr, "round_chain: pass 2 orthogonality %.3e (factors %s)\n", dev2, ok2 ? "ok" : "failed");
        if (ok2 && dev2 <= kOrthTol) {
            for (size_t k = 0; k < d; ++k) t.release(C[k]);
            C = p2.C;
            dev = dev2;
        } else {
            for (size_t k = 0; k < d; ++k) t.release(p2.C[k]);
        }
    }
    const bool ok = dev <= kOrthTol;
    if (!ok && t.sharded()) {   // no sharded sequential sweep: report, cores untouched
        for (size_t k = 0; k < d; ++k) t.release(C[k]);
        { g_marks = nullptr; return false; }
    }
    for (size_t k = 0; k < d; ++k) t.replace(k, C[k]);
    if (!ok) rl_sweep(t, max_ranks, eps, cX, d - 1);
    g_marks = nullptr;
    return true;
}

// One right chain pass (CholeskyQR on the whole train) over cores 1..d-1 that are already nearly
// right-orthonormal -- the truncating round's output when its Gram-based cores missed the tolerance:
// same tensor and ranks, orthonormality restored to ~u. False (cores untouched) if the pass failed.
bool reorthonormalize(TT& t) {
    int* hs = static_cast<int*>(t.h->host_scratch) + 12288;
    ChainPass p;
    chain_pass(t, false, p, hs);
    const double dev = chain_check(t, p.C);
    const bool ok = chain_status_ok(p) && dev <= kOrthTol;
    for (size_t k = 0; k < t.d; ++k) {
        if (ok) t.replace(k, p.C[k]);
        else t.release(p.C[k]);
    }
    return ok;
}

// Sequential certified right-to-left CholeskyQR sweep from edge `from` down to 1 (the unfoldings are
// already certified on the left with constant cX); an uncertified LQ hands over to the reference
// algorithm at that edge.
void rl_sweep(TT& t, const size_t* max_ranks, double eps, double cX, size_t from) {
    for (size_t k = from; k >= 1; --k) {
        const size_t m = t.r[k], nn = t.cols_right(k), prow = t.rows_left(k - 1);
        double* Q = t.alloc(m * nn);
        double* L = t.alloc(m * m);
        const OrthResult o = orthogonalize(t.h, t.core[k], m, nn, true, Q, L);
        const double c = o.certified ? cX * o.cert_ratio : 0.0;
        if (!(m <= nn && c > 16.0 * 2.220446049250313e-16 && eps < 0.5 * c)) {
            t.release(Q);
            t.release(L);
            for (size_t j = 0; j < k; ++j) orth_right(t, j);
            for (size_t kk = k; kk >= 1; --kk) truncate_edge(t, kk, max_ranks[kk - 1], eps);
            return;
        }
        double* prv = t.alloc(prow * m);
        gemm(t.h, prv, prow, m, 1.0, t.core[k - 1], m, false, m, L, m, false);
        t.release(L);
        t.replace(k, Q);
        t.replace(k - 1, prv);
    }
}

void round(TT& t, bool canonicalized, size_t core_pos, const size_t* max_ranks, double eps) {
    const size_t d = t.d;
    t.h->last_round_path = XRS_ROUND_CHAIN;
    if (round_chain(t, max_ranks, eps)) return;      // certified, nothing to cut
    t.h->last_round_path = XRS_ROUND_TRUNCATE;
    if (round_truncate(t, max_ranks, eps)) return;   // certified, cuts by maxRank only (tt_trunc.hip)
    static const bool no_general = std::getenv("XRS_NO_GENERAL_ROUND") != nullptr;
    t.h->last_round_path = XRS_ROUND_GENERAL;
    if (!no_general && round_general(t, max_ranks, eps)) return;   // any spectrum, device-resident (tt_trunc.hip)
    t.h->last_round_path = XRS_ROUND_REFERENCE;
    // canonicalize_right (ttNetwork.cpp:638-640, 654)
    const size_t start = canonicalized ? core_pos : 0;
    for (size_t k = start; k + 1 < d; ++k) orth_right(t, k);
    if (!canonicalized)
        ;  // cores 0..d-2 are now left-orthogonal
    // right-to-left truncation (ttNetwork.cpp:656-658)
    for (size_t k = d - 1; k >= 1; --k) truncate_edge(t, k, max_ranks[k - 1], eps);
}

void soft_threshold(TT& t, bool canonicalized, size_t core_pos, const double* taus) {
    const size_t d = t.d;
    t.h->last_round_path = XRS_ROUND_REFERENCE;
    const size_t start = canonicalized ? core_pos : 0;   // canonicalize_right (ttNetwork.cpp:701)
    for (size_t k = start; k + 1 < d; ++k) orth_right(t, k);
    // round_edge(numComponents - i, numComponents - i - 1, max, 0.0, taus[i]) (:703-705): edge i counted
    // from the right end
    for (size_t i = 0; i + 1 < d; ++i) truncate_edge(t, d - 1 - i, std::numeric_limits<size_t>::max(), 0.0, taus[i]);
}

// <x, y> with the zipper run from both ends at once (left environments on a side stream, right ones on
// the main stream) and closed at the middle edge m by sum_ab E_m[a,b] F_m[a,b]: the two chains are
// independent, so the critical path halves and the two streams fill the chip together.
//   left  E_{k+1} (rx_{k+1} x ry_{k+1}) = sum_i X_k[:,i,:]^T E_k Y_k[:,i,:]      (E_0 = 1)
//   right F_k     (rx_k x ry_k)         = sum_i X_k[:,i,:] F_{k+1} Y_k[:,i,:]^T  (F_d = 1)
// Sharded (mode slices): both ends on one stream, the two environments of a step side by side in one
// buffer and completed by ONE all-reduce; the closing sum needs none (E_m, F_m are already global).
double dot_two_ended(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                     const double* const* Y, const TT* shard = nullptr) {
    const size_t m = d / 2;
    size_t emax = 1, tmax = 1;
    for (size_t k = 0; k <= d; ++k) emax = std::max(emax, rx[k] * ry[k]);
    for (size_t k = 0; k < d; ++k) tmax = std::max(tmax, std::max(ry[k] * n[k] * rx[k + 1], rx[k] * n[k] * ry[k + 1]));
    // ping-pong pair buffers [E | F]: E at the front, F right behind the E written in the same step
    DevBuf P0(h, 2 * emax * 8), P1(h, 2 * emax * 8), TL(h, tmax * 8), TR(h, tmax * 8);
    // boundary environments E_0 = F_d = [1]: with rank-1 ends (every TT) the first product of each end is
    // 1 * X_k = X_k exactly, so that GEMM (and the upload of the 1s) is skipped
    const bool unit_l = rx[0] == 1 && ry[0] == 1, unit_r = rx[d] == 1 && ry[d] == 1;
    // <x, x> (the same cores): every environment sum_i X_i^T E X_i / X_i F X_i^T is symmetric, so the
    // second product of each step computes the lower tiles only and mirrors them (gemm_sym: exactly
    // symmetric environments, ~1/4 fewer flops per step)
    bool self = true;
    for (size_t k = 0; k < d && self; ++k) self = X[k] == Y[k] && rx[k + 1] == ry[k + 1];
    auto second = [&](const GemmSpec& g) {
        if (self) gemm_sym(h, g.C, g.M, 1.0, g.A, g.lda, g.ta, g.K, g.B, g.ldb, g.tb);
        else gemm(h, g);
    };
    if (!unit_l || !unit_r) {
        double* ones = static_cast<double*>(h->host_scratch) + 4096;   // (a slot no other routine uses)
        ones[0] = ones[1] = 1.0;
        XRS_HIP(hipMemcpyAsync(P0.d(), &ones[0], 8, hipMemcpyHostToDevice, h->stream));
        XRS_HIP(hipMemcpyAsync(P0.d() + emax, &ones[1], 8, hipMemcpyHostToDevice, h->stream));
    }
    // per step: the left end's products (T = E^T X_k, E' = T^T Y_k) and the right end's (T = X_k F,
    // F' = T Y_k^T); the first product of an end is skipped at a unit boundary (T = X_k)
    struct EndStep {
        bool on = false, first = false;
        GemmSpec g1{}, g2{};
    };
    const size_t steps = std::max(m, d - m);
    auto plan = [&](size_t s, double* E, double* F, double* nb, EndStep& L, EndStep& R, size_t& ne) {
        L = EndStep{};
        R = EndStep{};
        ne = 0;
        if (s < m) {
            const size_t k = s, a = rx[k], b = ry[k], nk = n[k], a2 = rx[k + 1], b2 = ry[k + 1];
            L.on = true;
            L.first = !(s == 0 && unit_l);
            const double* T = L.first ? TL.d() : X[k];
            L.g1 = GemmSpec{E, X[k], TL.d(), b, nk * a2, a, b, nk * a2, true, false};          // E^T X_k: b x (nk a2)
            L.g2 = GemmSpec{T, Y[k], nb, a2, b2, b * nk, a2, b2, true, false};                 // ((b nk) x a2)^T Y_k
            ne = a2 * b2;
        }
        if (s < d - m) {
            const size_t k = d - 1 - s, a = rx[k], b = ry[k], nk = n[k], a2 = rx[k + 1], b2 = ry[k + 1];
            R.on = true;
            R.first = !(s == 0 && unit_r);
            const double* T = R.first ? TR.d() : X[k];
            R.g1 = GemmSpec{X[k], F, TR.d(), a * nk, b2, a2, a2, b2, false, false};            // X_k F: (a nk) x b2
            R.g2 = GemmSpec{T, Y[k], nb + (shard ? ne : emax), a, b, nk * b2, nk * b2, nk * b2, false, true};   // T Y_k^T
        }
    };
    // the left end on a side stream beside the right end on the main stream (one stream when sharded)
    double *E = P0.d(), *F = P0.d() + emax;
    double* nextbuf = P1.d();
    double* curbuf = P0.d();
    {
        StreamFork fork(h);
        for (size_t s = 0; s < steps; ++s) {   // launches interleaved step by step (see gram_chains)
            EndStep L, R;
            size_t ne;
            plan(s, E, F, nextbuf, L, R, ne);
            if (L.on) {
                if (!shard) fork.side();
                if (L.first) gemm(h, L.g1);
                second(L.g2);
            }
            if (R.on) {
                if (!shard) fork.main();
                if (R.first) gemm(h, R.g1);
                second(R.g2);
            }
            // one all-reduce for both ends. The left end is idle only in the last step of an odd order
            // (d - m = m + 1): E then stays in the other buffer, untouched by this step's F.
            if (shard) shard->reduce(nextbuf, ne + (R.on ? R.g2.M * R.g2.N : 0));
            if (L.on) E = L.g2.C;
            if (R.on) F = R.g2.C;
            std::swap(curbuf, nextbuf);
        }
        fork.join();
    }
    return reduce_to_host(h, 1, E, F, rx[m] * ry[m]);
}

double dot(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y, const TT* shard = nullptr) {
    size_t emax = 1, tmax = 1;
    for (size_t k = 0; k < d; ++k) {
        emax = std::max(emax, rx[k + 1] * ry[k + 1]);
        tmax = std::max(tmax, ry[k] * n[k] * rx[k + 1]);
    }
    if (d >= 4) return dot_two_ended(h, d, n, rx, X, ry, Y, shard);
    DevBuf E0(h, emax * 8), E1(h, emax * 8), T(h, tmax * 8);
    const double one = 1.0;
    XRS_HIP(hipMemcpyAsync(E0.d(), &one, 8, hipMemcpyHostToDevice, h->stream));
    double* E = E0.d();
    double* En = E1.d();
    for (size_t k = 0; k < d; ++k) {
        const size_t a = rx[k], b = ry[k], nk = n[k], a2 = rx[k + 1], b2 = ry[k + 1];
        // T (b x nk a2) = E^T (b x a) * X_k (a x nk a2)
        gemm(h, T.d(), b, nk * a2, 1.0, E, b, true, a, X[k], nk * a2, false);
        // E' (a2 x b2) = T^T as ((b nk) x a2)^T * Y_k ((b nk) x b2)
        gemm(h, En, a2, b2, 1.0, T.d(), a2, true, b * nk, Y[k], b2, false);
        if (shard) shard->reduce(En, a2 * b2);   // sum over all ranks' mode slices
        std::swap(E, En);
    }
    double* hs = static_cast<double*>(h->host_scratch);
    XRS_HIP(hipMemcpyAsync(hs, E, 8, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    return hs[0];
}

}  // namespace ttd

// Asynchronous <x, y> (xrs_tt_dot_async). The caller's thread only forks (records ev_dot on the main
// stream; the child's two streams -- side streams 1 and 2 -- wait for it) and posts the TT descriptors to
// a persistent worker thread, which enqueues the ordinary two-ended zipper on the child handle and
// synchronises it. The caller meanwhile enqueues its next work (x.round) on the main stream, so both
// run on the device together and the ~25 launches of the product cost the caller no host time.
// Releases of the parent's blocks wait for the worker to finish (fence_readers): the round's
// replacement of x's cores never recycles a block the product still reads.
class DotWorker {
   public:
    explicit DotWorker(xrs_handle_t parent) : child_(create_child_handle(parent)), th_([this] { run(); }) {}
    ~DotWorker() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
            state_.store(kPosted, std::memory_order_release);
            gate_.store(1, std::memory_order_release);
        }
        cv_.notify_all();
        th_.join();
        (void)xrs_destroy(child_);
    }
    xrs_handle_t child() const { return child_; }
    // gated: the worker enqueues only once open_gate() has been called (with gate_ev: the child's streams
    // first wait for that event)
    void post(size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
              const double* const* Y, bool gated) {
        gate_ev_ = nullptr;
        gate_.store(gated ? 0 : 1, std::memory_order_release);
        d_ = d;
        n_.assign(n, n + d);
        rx_.assign(rx, rx + d + 1);
        ry_.assign(ry, ry + d + 1);
        X_.assign(X, X + d);
        Y_.assign(Y, Y + d);
        err_code_ = 0;
        {
            std::lock_guard<std::mutex> g(m_);
            state_.store(kPosted, std::memory_order_release);
        }
        cv_.notify_all();
    }
    void open_gate(hipEvent_t ev) {
        if (gate_.load(std::memory_order_acquire) != 0) return;
        gate_ev_ = ev;
        {
            std::lock_guard<std::mutex> g(m_);
            gate_.store(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    bool gate_closed() const { return gate_.load(std::memory_order_acquire) == 0; }
    // blocks until the posted product has finished (device included)
    void wait_done() {
        open_gate(nullptr);
        for (int i = 0; i < (1 << 16) && state_.load(std::memory_order_acquire) != kDone; ++i) __builtin_ia32_pause();
        if (state_.load(std::memory_order_acquire) != kDone) {
            std::unique_lock<std::mutex> g(m_);
            cv_.wait(g, [&] { return state_.load(std::memory_order_acquire) == kDone; });
        }
    }
    double take() {
        wait_done();
        state_.store(kIdle, std::memory_order_release);
        if (err_code_ != 0) throw Error{err_code_, err_msg_};
        return value_;
    }

   private:
    static constexpr int kIdle = 0, kPosted = 1, kDone = 2;
    void run() {
        (void)hipSetDevice(child_->device);
        for (;;) {
            // spin briefly (the next product usually follows within a step), then sleep
            for (int i = 0; i < (1 << 18) && state_.load(std::memory_order_acquire) != kPosted; ++i) __builtin_ia32_pause();
            if (state_.load(std::memory_order_acquire) != kPosted) {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return state_.load(std::memory_order_acquire) == kPosted; });
            }
            if (quit_) return;
            for (int i = 0; i < (1 << 18) && gate_.load(std::memory_order_acquire) == 0; ++i) __builtin_ia32_pause();
            if (gate_.load(std::memory_order_acquire) == 0) {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gate_.load(std::memory_order_acquire) != 0 || quit_; });
            }
            if (quit_) return;
            try {
                if (gate_ev_ != nullptr) {
                    XRS_HIP(hipStreamWaitEvent(child_->stream, gate_ev_, 0));
                    XRS_HIP(hipStreamWaitEvent(child_->side_stream[0], gate_ev_, 0));
                }
                value_ = ttd::dot(child_, d_, n_.data(), rx_.data(), X_.data(), ry_.data(), Y_.data());
            } catch (const Error& e) {
                err_code_ = e.code;
                err_msg_ = e.msg;
            } catch (const std::exception& e) {
                err_code_ = XRS_EINVAL;
                err_msg_ = e.what();
            }
            {
                std::lock_guard<std::mutex> g(m_);
                state_.store(kDone, std::memory_order_release);
            }
            cv_.notify_all();
        }
    }
    xrs_handle_t child_;
    size_t d_ = 0;
    std::vector<size_t> n_, rx_, ry_;
    std::vector<const double*> X_, Y_;
    double value_ = 0.0;
    int err_code_ = 0;
    std::string err_msg_;
    bool quit_ = false;
    std::atomic<int> state_{kIdle};
    std::atomic<int> gate_{1};
    hipEvent_t gate_ev_ = nullptr;
    std::mutex m_;
    std::condition_variable cv_;
    std::thread th_;   // (last: started after every other member is constructed)
};

void dot_async(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
               const double* const* Y) {
    XRS_REQUIRE(!h->dot_pending, "an asynchronous inner product is already in flight on this handle");
    if (h->dot_worker == nullptr) h->dot_worker = new DotWorker(h);
    xrs_handle_t c = h->dot_worker->child();
    c->prof_mask = h->prof_mask;   // (the parent's profiler collects the child's records at prof_end)
    // Gate (default; XRS_DOT_GATE=0: start at once): the product starts behind the Gram chains of the next
    // round on this handle (open_dot_gate, called by chain_pass), so that it fills the round's
    // factorisation phase -- one batched Cholesky launch on a few CUs -- instead of halving the chains'
    // share of the chip. Anything that waits for the product opens the gate first (open_dot_gate: at the
    // handle's current stream point). Gated, that event is the product's only dependency: it lies after
    // this call in the handle's stream order, so no fork event is recorded here (3 HIP calls, ~15 us of
    // host time at the head of every step).
    static const bool gate = [] {
        const char* e = std::getenv("XRS_DOT_GATE");
        return !(e && e[0] == '0');
    }();
    if (!gate) {
        XRS_HIP(hipEventRecord(h->ev_dot, h->stream));
        XRS_HIP(hipStreamWaitEvent(c->stream, h->ev_dot, 0));
        XRS_HIP(hipStreamWaitEvent(c->side_stream[0], h->ev_dot, 0));
    }
    h->dot_worker->post(d, n, rx, X, ry, Y, gate);
    h->dot_pending = true;
    h->reader_pending = true;
}

void open_dot_gate(xrs_handle_t h) {
    if (!h->dot_pending || h->dot_worker == nullptr || !h->dot_worker->gate_closed()) return;
    XRS_HIP(hipEventRecord(h->ev_dot_join, h->stream));
    h->dot_worker->open_gate(h->ev_dot_join);
}

double dot_wait(xrs_handle_t h) {
    XRS_REQUIRE(h->dot_pending, "no asynchronous inner product in flight on this handle");
    open_dot_gate(h);   // (no round opened it: the product starts behind the handle's current point)
    h->dot_pending = false;
    h->reader_pending = false;
    return h->dot_worker->take();
}

xrs_handle_t dot_child(xrs_handle_t h) { return h->dot_worker ? h->dot_worker->child() : nullptr; }

namespace ttd {

void check_tt(size_t d, const size_t* n, const size_t* r, double* const* cores) {
    XRS_REQUIRE(d >= 1, "TT must have at least one component");
    XRS_REQUIRE(n && r && cores, "null TT description");
    XRS_REQUIRE(r[0] == 1 && r[d] == 1, "boundary ranks must be 1");
    for (size_t k = 0; k < d; ++k) {
        XRS_REQUIRE(n[k] > 0 && r[k + 1] > 0, "dimensions and ranks must be positive");
        XRS_REQUIRE(cores[k] != nullptr, "null core");
    }
}

}  // namespace ttd

using namespace ttd;

void wait_dot_done(xrs_handle_t h) {
    if (!h->dot_pending || h->dot_worker == nullptr) return;
    open_dot_gate(h);
    h->dot_worker->wait_done();
}

void destroy_dot_worker(xrs_handle_t h) {
    if (h->dot_worker == nullptr) return;
    if (h->dot_pending) {
        try {
            open_dot_gate(h);
            (void)h->dot_worker->take();
        } catch (...) {
        }
        h->dot_pending = false;
    }
    delete h->dot_worker;
    h->dot_worker = nullptr;
}

namespace tt {
void move_core(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
               size_t pos, bool keep_rank) {
    check_tt(d, n, r, cores);
    TT t{h, d, n, r, cores};
    xrs::move_core(t, canonicalized, core_pos, pos, keep_rank);
}
void round(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
           const size_t* max_ranks, double eps) {
    check_tt(d, n, r, cores);
    TT t{h, d, n, r, cores};
    xrs::round(t, canonicalized, core_pos, max_ranks, eps);
}
double dot(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y) {
    return xrs::dot(h, d, n, rx, X, ry, Y);
}
void soft_threshold(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
                    const double* taus) {
    check_tt(d, n, r, cores);
    TT t{h, d, n, r, cores};
    xrs::soft_threshold(t, canonicalized, core_pos, taus);
}
}  // namespace tt

}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_tt_move_core(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, int canonicalized,
                     size_t core_position, size_t position, int keep_rank) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        check_tt(d, n, r, cores);
        XRS_REQUIRE(position < d, "Illegal core-position");
        XRS_REQUIRE(!canonicalized || core_position < d, "Illegal current core position");
        TT t{h, d, n, r, cores};
        move_core(t, canonicalized != 0, core_position, position, keep_rank != 0);
    });
}

int xrs_tt_round(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, int canonicalized,
                 size_t core_position, const size_t* max_ranks, double eps) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        check_tt(d, n, r, cores);
        XRS_REQUIRE(eps < 1.0 && eps >= 0.0, "_eps must be smaller than one.");
        for (size_t k = 0; k + 1 < d; ++k)
            XRS_REQUIRE(max_ranks[k] > 0, "Trying to round a TTTensor to rank 0 is not possible.");
        XRS_REQUIRE(!canonicalized || core_position < d, "Illegal current core position");
        TT t{h, d, n, r, cores};
        round(t, canonicalized != 0, core_position, max_ranks, eps);
    });
}

int xrs_tt_soft_threshold(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, int canonicalized,
                          size_t core_position, const double* taus) {
    return guarded([&] {
        XRS_REQUIRE(h && (d < 2 || taus), "null argument");
        check_tt(d, n, r, cores);
        XRS_REQUIRE(!canonicalized || core_position < d, "Illegal current core position");
        for (size_t k = 0; k + 1 < d; ++k) XRS_REQUIRE(taus[k] >= 0.0, "soft threshold must not be negative");
        TT t{h, d, n, r, cores};
        soft_threshold(t, canonicalized != 0, core_position, taus);
    });
}

int xrs_tt_round_sharded(xrs_handle_t h, size_t d, const size_t* n_local, size_t* r, double** cores,
                         const size_t* max_ranks, double eps, xrs_allreduce_fn allreduce, void* ctx, int* certified) {
    return guarded([&] {
        XRS_REQUIRE(h && certified, "null argument");
        XRS_REQUIRE(d >= 2 && n_local && r && cores, "null TT description");
        XRS_REQUIRE(r[0] == 1 && r[d] == 1, "boundary ranks must be 1");
        XRS_REQUIRE(eps < 1.0 && eps >= 0.0, "_eps must be smaller than one.");
        for (size_t k = 0; k + 1 < d; ++k)
            XRS_REQUIRE(max_ranks[k] > 0, "Trying to round a TTTensor to rank 0 is not possible.");
        TT t{h, d, n_local, r, cores};
        t.shard_mode = true;
        t.ar = allreduce;   // null: one rank
        t.ar_ctx = ctx;
        // no cut possible: the chain round; ranks to cut: the certified truncation (the ranks' order is not
        // known here: tall right edges and left structural excess report uncertified; see xrs_tt_round_sharded_ex)
        *certified = (round_chain(t, max_ranks, eps) || round_truncate(t, max_ranks, eps)) ? 1 : 0;
    });
}

int xrs_tt_round_sharded_ex(xrs_handle_t h, size_t d, const size_t* n_local, size_t* r, double** cores,
                            const size_t* max_ranks, double eps, int world, int rank, xrs_allreduce_fn allreduce,
                            void* ctx, int* path) {
    return guarded([&] {
        XRS_REQUIRE(h && path, "null argument");
        XRS_REQUIRE(d >= 2 && n_local && r && cores && max_ranks, "null TT description");
        XRS_REQUIRE(r[0] == 1 && r[d] == 1, "boundary ranks must be 1");
        XRS_REQUIRE(world >= 1 && rank >= 0 && rank < world, "world / rank out of range");
        XRS_REQUIRE(size_t(world) * d <= 2040, "world * d above 2040");
        XRS_REQUIRE(eps < 1.0 && eps >= 0.0, "_eps must be smaller than one.");
        for (size_t k = 0; k + 1 < d; ++k)
            XRS_REQUIRE(max_ranks[k] > 0, "Trying to round a TTTensor to rank 0 is not possible.");
        TT t{h, d, n_local, r, cores};
        t.shard_mode = true;
        t.ar = allreduce;   // null: one rank
        t.ar_ctx = ctx;
        t.world = world;
        t.rank = rank;
        static const bool no_general = std::getenv("XRS_NO_GENERAL_ROUND") != nullptr;
        *path = 0;
        if (round_chain(t, max_ranks, eps)) *path = XRS_ROUND_CHAIN;
        else if (round_truncate(t, max_ranks, eps)) *path = XRS_ROUND_TRUNCATE;
        else if (!no_general && round_general(t, max_ranks, eps)) *path = XRS_ROUND_GENERAL;
        if (*path) h->last_round_path = *path;
    });
}

int xrs_tt_dot_sharded(xrs_handle_t h, double* result, size_t d, const size_t* n_local, const size_t* rx,
                       const double* const* X, const size_t* ry, const double* const* Y, xrs_allreduce_fn allreduce,
                       void* ctx) {
    return guarded([&] {
        XRS_REQUIRE(h && result, "null argument");
        XRS_REQUIRE(d >= 1 && n_local && rx && ry && X && Y, "null TT description");
        check_tt(d, n_local, rx, const_cast<double* const*>(X));
        check_tt(d, n_local, ry, const_cast<double* const*>(Y));
        TT t{h, d, n_local, const_cast<size_t*>(rx), const_cast<double**>(X)};
        t.shard_mode = true;
        t.ar = allreduce;   // null: one rank
        t.ar_ctx = ctx;
        *result = dot(h, d, n_local, rx, X, ry, Y, &t);
    });
}

int xrs_tt_last_round_path(xrs_handle_t h) { return h ? h->last_round_path : -1; }

int xrs_tt_dot(xrs_handle_t h, double* result, size_t d, const size_t* n, const size_t* rx, const double* const* X,
               const size_t* ry, const double* const* Y) {
    return guarded([&] {
        XRS_REQUIRE(h && result, "null argument");
        check_tt(d, n, rx, const_cast<double* const*>(X));
        check_tt(d, n, ry, const_cast<double* const*>(Y));
        *result = dot(h, d, n, rx, X, ry, Y);
    });
}

int xrs_tt_dot_async(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X,
                     const size_t* ry, const double* const* Y) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        check_tt(d, n, rx, const_cast<double* const*>(X));
        check_tt(d, n, ry, const_cast<double* const*>(Y));
        XRS_REQUIRE(d >= 2, "the asynchronous inner product needs at least two components");
        dot_async(h, d, n, rx, X, ry, Y);
    });
}

int xrs_tt_dot_wait(xrs_handle_t h, double* result) {
    return guarded([&] {
        XRS_REQUIRE(h && result, "null argument");
        *result = dot_wait(h);
    });
}

}  // extern "C"
