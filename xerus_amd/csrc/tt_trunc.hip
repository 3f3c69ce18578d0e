// Certified truncating TT round: TTNetwork::round (ttNetwork.cpp:644-665) when ranks are cut.
//
// The reference: canonicalize_right (pivoted-QR sweep left to right, rank rule |R_kk| < 16 eps R_00),
// then right to left round_edge per edge (tensorNetwork.cpp:678-818): SVD of the edge's r x r factor,
// cut at maxRank then at the first sigma_j <= eps sigma_0 (tensor.cpp:1462-1474), core k <- Vt, core
// k-1 <- core k-1 * U S. Here, for a TT whose unfoldings are provably well conditioned:
//  1. structural rank excess at the left end (r_{k+1} > n_0 ... n_k, e.g. after x + y) is removed by
//     the reference's own QC steps (exact rank rule), then one left chain pass gives the left-canonical
//     cores: G_{k+1} = M_k^T (G_k (x) I) M_k, G_k = L_k L_k^T, A_k = (L_k^T (x) I) M_k L_{k+1}^{-T}, with
//     a status-only Cholesky of G_k - tau tr(G_k) I per edge certifying that no QC rank drop happens;
//  2. the right-to-left sweep runs on the device without host synchronisation: per edge the Gram P of
//     the edge matrix B (r x N: P = B B^T, or B^T B when r > N), its Cholesky factor L (plus the
//     certificate chol(P - tau tr(P) I): sigma_min(B) >= sqrt(tau/2) ||B||_F > eps sigma_0, so the eps
//     rule cannot cut and the rank is min(r, N, maxRank) -- known on the host in advance), the right
//     singular vectors of L (or L^T) by one-sided Jacobi in LDS (svd.hip), and three GEMMs:
//        wide (B = L Q, L = U S V^T): core_k <- S_kk^{-1} U_kk^T B,  core_{k-1} <- core_{k-1} (U S)_kk
//        tall (B = Q L^T):            core_k <- Vt_kk,               core_{k-1} <- core_{k-1} (B Vt_kk^T)
//     (the Jacobi runs on the columns of L in both cases: U of L in the wide, Vt of L^T in the tall case);
//  3. one host synchronisation reads every status (factorisations, Jacobi convergence) and the
//     orthonormality of the left-canonical and of the final right-canonical cores. Any failure discards
//     the new cores and the caller runs the reference's algorithm (tt.hip: orth_right + truncate_edge).
// Same ranks and the same singular values as the reference; the kept subspaces and hence the
// represented tensor agree up to rounding (the SVD gauge of the cores may differ, as for every SVD).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "tt_common.hpp"

namespace xrs {
namespace ttd {

namespace {

constexpr double kTruncOrthTol = 1e-12;    // max |C C^T - I| of a canonical core; above it: one chain pass
constexpr double kTruncAcceptTol = 1e-8;   // above it the sweep is rejected (reference algorithm instead)

// Host-side record of everything enqueued; buffers are released once the sweep is judged.
struct Sweep {
    TT& t;
    std::vector<DevBuf> keep;
    std::vector<double*> owned;   // pool blocks that become cores on success (released on failure)
    explicit Sweep(TT& tt) : t(tt) {}
    double* buf(size_t elems) {
        keep.emplace_back(t.h, std::max<size_t>(elems, 1) * 8);
        return keep.back().d();
    }
    double* core(size_t elems) {
        double* p = t.alloc(elems);
        owned.push_back(p);
        return p;
    }
    void drop(double* p) {   // a core block that is no longer needed
        auto it = std::find(owned.begin(), owned.end(), p);
        if (it != owned.end()) {
            owned.erase(it);
            t.release(p);
        }
    }
    void discard() {
        for (double* p : owned) t.release(p);
        owned.clear();
    }
};

// one or more Cholesky factorisations of an n x n symmetric matrix in a single launch (n <= 512; larger
// ones blocked, one job at a time):
// the factor L (lower, out of place) and its inverse Z = L^{-1}, plus status-only certificates
// chol(A - tau tr(A) I). Statuses go to status[0..count).
struct CholJob {
    const double* A;
    int n;
    double* L;   // null: certificate only
    double* Z;
    double shift = 0.0;   // relative diagonal shift (factor jobs; certificates always -kGramShift)
};

void chol_jobs(Sweep& sw, const std::vector<CholJob>& jobs, int* status) {
    xrs_handle_t h = sw.t.h;
    std::vector<BigJob> big;
    std::vector<int> big_slot;
    PotrfBatch pb{};
    TrinvBatch tb{};
    int ns = 0, ninv = 0;
    std::vector<int> huge;
    for (size_t i = 0; i < jobs.size(); ++i) {
        const CholJob& j = jobs[i];
        if (j.n > 512) {   // blocked, one job at a time (ranks above the batched kernels)
            huge.push_back(int(i));
            continue;
        }
        if (j.n > 256) {
            big.push_back({j.A, j.L ? j.shift : -kGramShift, j.n, j.L, j.Z});
            big_slot.push_back(int(i));
            continue;
        }
        XRS_REQUIRE(ns < kPotrfBatchMax, "chol_jobs: batch too large");
        double* dinv = j.L ? sw.buf(dinv_elems(j.n)) : sw.buf(dinv_elems(j.n));
        pb.src[ns] = j.A;
        pb.G[ns] = j.L;
        pb.Dinv[ns] = dinv;
        pb.shift[ns] = j.L ? j.shift : -kGramShift;
        pb.n[ns] = j.n;
        ++ns;
        if (j.L && j.Z) {
            tb.L[ninv] = j.L;
            tb.Dinv[ninv] = dinv;
            tb.X[ninv] = j.Z;
            tb.n[ninv] = j.n;
            ++ninv;
        }
    }
    // statuses: the small jobs first in job order is not needed -- keep one slot per small job, then two
    // per big job (factor_big's two diagonal blocks); the caller only tests all-zero
    if (ns) {
        pb.status = status;
        potrf_batched(h, pb, ns);
    }
    if (ninv) trinv_batched(h, tb, ninv);
    if (!big.empty()) {
        std::vector<DevBuf> keep;
        factor_big(h, big, status + ns, keep);
        for (auto& k : keep) sw.keep.push_back(std::move(k));
    }
    int slot = ns + 2 * int(big.size());
    for (int i : huge) {
        const CholJob& j = jobs[size_t(i)];
        chol_full(h, j.A, size_t(j.n), j.L ? j.shift : -kGramShift, j.L, j.Z, status + slot);
        slot += chol_full_blocks(size_t(j.n));
    }
}

int chol_status_count(const std::vector<CholJob>& jobs) {
    int c = 0;
    for (const CholJob& j : jobs) c += j.n > 512 ? chol_full_blocks(size_t(j.n)) : (j.n > 256 ? 2 : 1);
    return c;
}

// max |X X^T - I| (rows, `rows` = true) or max |X^T X - I| of a list of matrices -> dev[0..count*16);
// the Grams sit in one buffer, completed across ranks by ONE all-reduce when sharded
void orth_devs(Sweep& sw, const std::vector<const double*>& X, const std::vector<size_t>& m, const std::vector<size_t>& n,
               bool rows, double* dev) {
    xrs_handle_t h = sw.t.h;
    const size_t cnt = X.size();
    size_t total = 0;
    for (size_t i = 0; i < cnt; ++i) total += (rows ? m[i] : n[i]) * (rows ? m[i] : n[i]);
    double* all = sw.buf(total);
    std::vector<GemmJob> grams;
    DevIdArgs da{};
    size_t off = 0;
    for (size_t i = 0; i < cnt; ++i) {
        const size_t g = rows ? m[i] : n[i];
        double* G = all + off;
        off += g * g;
        if (rows) grams.push_back({g, g, n[i], n[i], n[i], false, true, X[i], X[i], G, true});
        else grams.push_back({g, g, m[i], g, g, true, false, X[i], X[i], G, true});
        da.G[i] = G;
        da.n[i] = int(g);
    }
    gemm_grouped(h, grams);
    sw.t.reduce(all, total);
    da.out = dev;
    hipLaunchKernelGGL(k_dev_identity_many, dim3(unsigned(cnt), 16), dim3(256), 0, h->stream, da);
    check_launch("k_dev_identity_many");
}

// wide edge, B = L Q with the left singular vectors of L as the rows of Ut (Jacobi on the columns of L):
// M = S^{-1} Ut[:kk] (new core = M B = Vt_kk Q) and T = Ut[:kk]^T S (= U S, core_{k-1} <- core_{k-1} T)
__global__ void __launch_bounds__(256) k_edge_factors(const double* __restrict__ Ut, const double* __restrict__ S, int r, int kk,
                                                      double* __restrict__ M, double* __restrict__ T, int s_is_lam) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < kk * r; e += gridDim.x * 256) {
        const int i = e / r, j = e - i * r;
        // (s_is_lam: S holds the eigenvalues of P = B B^T, sigma = sqrt(max(lambda, 0)) -- k_sqrt_lam's value)
        const double u = Ut[size_t(i) * r + j], s = s_is_lam ? sqrt(fmax(S[i], 0.0)) : S[i];
        M[e] = s > 0.0 ? u / s : 0.0;
        T[size_t(j) * kk + i] = u * s;
    }
}

// One left chain pass over the cores `src` (ranks t.r): G_{k+1} = M_k^T (G_k (x) I) M_k, G_k = L_k L_k^T
// (+ the status-only certificate of G_k - tau tr(G_k) I with `certify`), Z_k = L_k^{-1}, and the
// left-canonical cores A_k = (L_k^T (x) I) M_k Z_{k+1}^T (A_{d-1} = (L^T (x) I) M_{d-1}).
// shift: relative diagonal shift of the factorisations (the general round's shifted CholeskyQR3 over the
// train); Gout / Zout (optional): the Grams G_k and inverses Z_k = L_k^{-1} of this pass (k = 1..d-1)
void left_pass(Sweep& sw, TT& t0, double* const* src, bool certify, std::vector<double*>& A, int* status, int& nst,
               double shift = 0.0, std::vector<double*>* Gout = nullptr, std::vector<double*>* Zout = nullptr) {
    TT t = t0;
    t.core = const_cast<double**>(src);
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    std::vector<double*> G(d, nullptr);
    size_t tmax = 1;
    for (size_t k = 1; k + 1 < d; ++k) tmax = std::max(tmax, t.size(k));
    double* T = sw.buf(tmax);
    for (size_t k = 1; k < d; ++k) G[k] = sw.buf(t.r[k] * t.r[k]);
    for (size_t k = 0; k + 1 < d; ++k) left_gram_step(t, G, T, k, true);   // (sharded: + one all-reduce per step)
    open_dot_gate(h);   // a gated async <x,y> runs beside the factorisations below
    std::vector<double*> Lf(d, nullptr), Zf(d, nullptr);
    std::vector<CholJob> jobs;
    for (size_t k = 1; k < d; ++k) {
        const int a = int(t.r[k]);
        Lf[k] = sw.buf(size_t(a) * a);
        Zf[k] = sw.buf(size_t(a) * a);
        jobs.push_back({G[k], a, Lf[k], Zf[k], shift});
        if (certify) jobs.push_back({G[k], a, nullptr, nullptr});
    }
    for (size_t b0 = 0; b0 < jobs.size(); b0 += 40) {   // (potrf_batched / trinv tables hold 48 / 64)
        const std::vector<CholJob> part(jobs.begin() + long(b0), jobs.begin() + long(std::min(jobs.size(), b0 + 40)));
        chol_jobs(sw, part, status + nst);
        nst += chol_status_count(part);
    }
    A.assign(d, nullptr);
    std::vector<double*> W(d, nullptr);
    std::vector<GemmJob> lefts, rights;
    for (size_t k = 0; k < d; ++k) {
        A[k] = sw.core(t.size(k));
        if (k == 0) continue;
        const size_t a = t.r[k], cols = t.cols_right(k);
        W[k] = (k + 1 < d) ? sw.buf(t.size(k)) : A[k];
        lefts.push_back({a, cols, a, a, cols, true, false, Lf[k], t.core[k], W[k]});
    }
    for (size_t k = 0; k + 1 < d; ++k) {
        const size_t b = t.r[k + 1];
        rights.push_back({t.rows_left(k), b, b, b, b, false, true, k == 0 ? t.core[0] : W[k], Zf[k + 1], A[k]});
    }
    gemm_grouped(h, lefts);
    gemm_grouped(h, rights);
    if (Gout) *Gout = G;
    if (Zout) *Zout = Zf;
}

}  // namespace

// Global mode sizes and this rank's first slice per mode (sharded: one all-reduce of a world x d table
// with this rank's slice counts in its row, one host synchronisation; world unknown: the sums only).
ShardLayout shard_layout(TT& t) {
    const size_t d = t.d;
    ShardLayout lay;
    if (t.layout_cached) {
        lay.ng = t.layout_ng;
        lay.off = t.layout_off;
        lay.known = t.layout_known;
        return lay;
    }
    lay.ng.assign(t.n, t.n + d);
    lay.off.assign(d, 0);
    lay.known = !t.sharded();
    if (!t.sharded()) return lay;
    xrs_handle_t h = t.h;
    const size_t w = t.world > 0 ? size_t(t.world) : 1, me = t.world > 0 ? size_t(t.rank) : 0;
    XRS_REQUIRE(w * d <= 2040 && me < w, "shard_layout: world / rank out of range");
    // (pinned scratch: doubles 4100 .. 6140, a region no other routine uses -- 2048.. the check points'
    // deviations, 4096 dot_two_ended's unit environments, 6144.. the status words)
    double* hn = static_cast<double*>(h->host_scratch) + 4100;
    for (size_t i = 0; i < w * d; ++i) hn[i] = 0.0;
    for (size_t k = 0; k < d; ++k) hn[me * d + k] = double(t.n[k]);
    DevBuf tab(h, w * d * 8);
    XRS_HIP(hipMemcpyAsync(tab.d(), hn, w * d * 8, hipMemcpyHostToDevice, h->stream));
    t.reduce(tab.d(), w * d);
    XRS_HIP(hipMemcpyAsync(hn, tab.d(), w * d * 8, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    for (size_t k = 0; k < d; ++k) {
        size_t s = 0, o = 0;
        for (size_t q = 0; q < w; ++q) {
            const size_t c = size_t(hn[q * d + k] + 0.5);
            s += c;
            if (q < me) o += c;
        }
        lay.ng[k] = s;
        lay.off[k] = o;
    }
    // an emulated communicator (rank 0 of identical slices) sums a zero-padded core to nranks x rank 0's
    // block, not the TT's core: the layout counts as unknown, so the steps that need a gathered core (tall
    // right edges, left structural excess) report uncertified instead of factorising a wrong matrix
    lay.known = t.world > 0 && !(t.ar == &xrs_comm_allreduce && comm_is_emulated(t.ar_ctx));
    t.layout_cached = true;
    t.layout_ng = lay.ng;
    t.layout_off = lay.off;
    t.layout_known = lay.known;
    return lay;
}

// Full core (a, ng, b) on every rank from this rank's slices (a, nl, b) at mode offset `off`: zeros
// elsewhere, completed by one all-reduce (each entry has exactly one non-zero contribution: exact).
void gather_core(TT& t, const double* local, size_t a, size_t nl, size_t ng, size_t b, size_t off, double* full) {
    xrs_handle_t h = t.h;
    XRS_HIP(hipMemsetAsync(full, 0, a * ng * b * 8, h->stream));
    if (nl && a && b)
        XRS_HIP(hipMemcpy2DAsync(full + off * b, ng * b * 8, local, nl * b * 8, nl * b * 8, a, hipMemcpyDeviceToDevice, h->stream));
    t.reduce(full, a * ng * b);
}

// This rank's slices (a, nl, b) of a full core (a, ng, b).
void slice_core(TT& t, const double* full, size_t a, size_t ng, size_t b, size_t off, size_t nl, double* local) {
    if (!(nl && a && b)) return;
    XRS_HIP(hipMemcpy2DAsync(local, nl * b * 8, full + off * b, ng * b * 8, nl * b * 8, a, hipMemcpyDeviceToDevice, t.h->stream));
}

// transfer_right (QC of core k, R into core k + 1) of a sharded TT: the left unfolding's rows are the
// ranks' mode blocks, so core k is gathered (small: a structural excess r_{k+1} > r_k n_k bounds it by
// r_{k+1}^2), factorised identically on every rank (deterministic kernels, same rank decision) and sliced.
void transfer_right_sharded(TT& t, size_t k, const ShardLayout& lay) {
    XRS_REQUIRE(lay.known, "transfer_right_sharded: rank layout unknown");
    const size_t a = t.r[k], nl = t.n[k], ng = lay.ng[k], b = t.r[k + 1];
    const size_t m = a * ng, kmax = std::min(m, b);
    double* full = t.alloc(m * b);
    gather_core(t, t.core[k], a, nl, ng, b, lay.off[k], full);
    double* Q = t.alloc(m * kmax);
    double* C = t.alloc(kmax * b);
    const size_t rank = qc(t.h, full, m, b, Q, C);
    t.release(full);
    double* Ql = t.alloc(a * nl * rank);
    slice_core(t, Q, a, ng, rank, lay.off[k], nl, Ql);
    const size_t ncols = t.cols_right(k + 1);
    double* nxt = t.alloc(rank * ncols);
    gemm(t.h, nxt, rank, ncols, 1.0, C, b, false, b, t.core[k + 1], ncols, false);
    t.release(C);
    t.release(Q);
    t.replace(k, Ql);
    t.replace(k + 1, nxt);
    t.r[k + 1] = rank;
}

// 1a of both rounds: structural excess (a wide left unfolding, r_{k+1} > r_k n_k, e.g. the boundary edges
// of x + y) removed by the reference's own QC steps (exact rank rule, host syncs). Sharded with an unknown
// layout: left in place (the left Gram is then singular, the certificate fails, the caller gathers).
void remove_left_excess(TT& t, const ShardLayout& lay) {
    for (size_t k = 0; k + 1 < t.d; ++k) {
        if (!(t.r[k + 1] > t.r[k] * lay.ng[k])) continue;
        if (!t.sharded()) transfer_right(t, k, true);
        else if (lay.known) transfer_right_sharded(t, k, lay);
    }
}

bool round_truncate(TT& t, const size_t* max_ranks, double eps) {
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    static const bool dbg = std::getenv("XRS_DEBUG_ROUND") != nullptr;
    if (d < 2 || d > 64) return false;
    const double cX = 0.5 * std::sqrt(kGramShift);
    if (!(eps < 0.25 * cX * cX)) return false;
    for (size_t k = 1; k < d; ++k)
        if (t.r[k] > kHugeMax) return false;

    // global mode sizes and this rank's slice offsets (sharded: one all-reduce + host sync)
    const ShardLayout lay = shard_layout(t);
    const std::vector<size_t>& ng = lay.ng;
    // 1a. structural excess (a wide left unfolding, r_{k+1} > r_k n_k, e.g. the boundary edges of x + y):
    //     the reference's own QC steps there (exact rank rule, host syncs; sharded: on the gathered core)
    remove_left_excess(t, lay);

    Sweep sw(t);
    // statuses: factorisations from 0 up, Jacobi convergence at kJacobiSlot + edge
    constexpr int kStatusWords = 1024, kJacobiSlot = 768;
    DevBuf st(h, kStatusWords * 4), devb(h, 64 * 16 * 8);
    int* status = st.as<int>();
    int nst = 0;
    XRS_HIP(hipMemsetAsync(status, 0, kStatusWords * 4, h->stream));

    // 1b. left chain pass (certified), and a second one on its output when a single CholeskyQR pass over
    //     the train left the cores short of orthonormal (kappa^2 u > tol: CholeskyQR2 on the whole train)
    int* hs = static_cast<int*>(h->host_scratch) + 13312;
    double* hd = static_cast<double*>(h->host_scratch) + 2048;
    std::vector<double*> A;
    left_pass(sw, t, t.core, true, A, status, nst);
    double worst = 0.0;
    for (int pass = 1;; ++pass) {
        {
            std::vector<const double*> X;
            std::vector<size_t> m, n;
            for (size_t k = 0; k + 1 < d; ++k) {
                X.push_back(A[k]);
                m.push_back(t.rows_left(k));
                n.push_back(t.r[k + 1]);
            }
            orth_devs(sw, X, m, n, false, devb.d());
        }
        // check point (one host sync): the factorisations and the left-canonical form
        const int nchk = int(d - 1) * 16;
        XRS_HIP(hipMemcpyAsync(hs, status, size_t(nst) * 4, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipMemcpyAsync(hd, devb.d(), size_t(nchk) * 8, hipMemcpyDeviceToHost, h->stream));
        host_wait(h);
        bool ok = true;
        for (int i = 0; i < nst; ++i) ok = ok && hs[i] == 0;
        worst = 0.0;
        for (int i = 0; i < nchk; ++i) worst = (hd[i] > worst || hd[i] != hd[i]) ? hd[i] : worst;
        if (dbg) std::fprintf(stderr, "round_truncate: left pass %d %s, orthogonality %.3e\n", pass,
                              ok ? "certified" : "NOT certified", worst);
        if (!ok) {
            sw.discard();
            return false;
        }
        if (worst <= kTruncOrthTol) break;
        if (pass == 2) {
            sw.discard();
            return false;
        }
        std::vector<double*> A1 = A;
        nst = 0;
        XRS_HIP(hipMemsetAsync(status, 0, kStatusWords * 4, h->stream));
        left_pass(sw, t, A1.data(), false, A, status, nst);
        for (double* p : A1) sw.drop(p);
    }

    // 2. right-to-left truncation sweep, device resident; new ranks decided on the host in advance
    std::vector<size_t> rr(t.r, t.r + d + 1);   // ranks as the sweep goes
    nst = 0;
    XRS_HIP(hipMemsetAsync(status, 0, kStatusWords * 4, h->stream));
    std::vector<int*> jst;   // Jacobi statuses
    // certificates of the eigensolver edges on side stream 0 (off the sweep's critical path), when this
    // handle owns its streams and is not inside a fork
    const bool cert_side = !h->borrowed_streams && h->stream == h->own_stream && h->side_stream[0] && h->prof_mask == 0;
    bool side_used = false;
    struct : PotrfBatch { int count = 0; } pending_cert{};
    auto flush_certs = [&]() {
        if (pending_cert.count == 0) return;
        pending_cert.status = status + nst;
        XRS_HIP(hipEventRecord(h->ev_fork, h->stream));
        XRS_HIP(hipStreamWaitEvent(h->side_stream[0], h->ev_fork, 0));
        side_used = true;
        StreamSwap on_side(h, h->side_stream[0]);   // (restores h->stream on scope exit, also on a throw)
        potrf_batched(h, pending_cert, pending_cert.count);
        nst += pending_cert.count;
        pending_cert.count = 0;
    };
    for (size_t k = d - 1; k >= 1; --k) {
        const size_t r = rr[k], N = t.n[k] * rr[k + 1], Ng = ng[k] * rr[k + 1];   // local / global columns
        const size_t kk = std::min({r, Ng, max_ranks[k - 1]});
        const bool wide = r <= Ng;
        // sharded tall edge: the N x N Gram spans the ranks' column blocks -- the core (r x Ng, small: Ng < r)
        // is gathered and the edge runs replicated on every rank (deterministic kernels: identical results)
        const bool tall_gather = !wide && t.sharded();
        if (tall_gather && !lay.known) {
            if (dbg) std::fprintf(stderr, "round_truncate: sharded tall edge %zu, rank layout unknown -> not certified\n", k);
            if (side_used) {   // the side stream may still read this sweep's buffers
                XRS_HIP(hipEventRecord(h->ev_join[0], h->side_stream[0]));
                XRS_HIP(hipStreamWaitEvent(h->stream, h->ev_join[0], 0));
            }
            sw.discard();
            return false;
        }
        const size_t Nw = tall_gather ? Ng : N;   // columns of the edge matrix as factorised here
        const size_t g = wide ? r : Nw;
        double* B = A[k];
        if (tall_gather) {
            B = sw.buf(r * Nw);
            gather_core(t, A[k], r, t.n[k], ng[k], rr[k + 1], lay.off[k], B);
        }
        double* P = sw.buf(g * g);
        if (wide) gemm_sym(h, P, g, 1.0, B, N, false, N, B, N, true);
        else gemm_sym(h, P, g, 1.0, B, Nw, true, r, B, Nw, false);
        if (wide) t.reduce(P, g * g);   // sharded: sum over the mode slices
        // the kept subspace: P's kk dominant eigenvectors. The certificate chol(P - tau tr(P) I) bounds
        // kappa(P) <= 4 / tau, so P's eigenvectors are accurate to u kappa-free relative gaps and no eps cut
        // can fire (kk is known): up to 256 by the tridiagonal eigensolver (syev.hip, ~10x faster than the
        // Jacobi sweeps), above it (or XRS_TRUNC_JACOBI=1) by one-sided Jacobi on the rows of L^T, i.e. on
        // the columns of the Cholesky factor (Drmac-Veselic: far fewer sweeps than the factor's rows)
        static const bool force_jacobi = std::getenv("XRS_TRUNC_JACOBI") != nullptr;
        const bool use_eig = !force_jacobi && sym_eig_top_fits(int(g), int(kk));
        double* L = use_eig ? nullptr : sw.buf(g * g);
        double* Z = (!use_eig && g > 256) ? sw.buf(g * g) : nullptr;   // (factor_big always builds L^{-1})
        if (use_eig && cert_side) {
            // the eigensolver does not need the factor: the status-only certificates run on a side stream
            // beside it (their statuses are read after the one join before the final check), batched: edges
            // d-1 .. 2 in one launch forked behind edge 2's P, edge 1 on its own (a fork per edge left a
            // ~7 us gap before every tridiagonalisation: the event record on the main stream)
            const int slot = pending_cert.count;
            XRS_REQUIRE(slot < kPotrfBatchMax, "round_truncate: too many certificates");
            pending_cert.src[slot] = P;
            pending_cert.G[slot] = nullptr;
            pending_cert.Dinv[slot] = sw.buf(dinv_elems(int(g)));
            pending_cert.shift[slot] = -kGramShift;
            pending_cert.n[slot] = int(g);
            pending_cert.count = slot + 1;
            if (k <= 2 || slot + 1 == kPotrfBatchMax) flush_certs();
        } else {
            std::vector<CholJob> cj{{P, int(g), nullptr, nullptr}};
            if (!use_eig) cj.insert(cj.begin(), CholJob{P, int(g), L, Z});
            chol_jobs(sw, cj, status + nst);
            nst += chol_status_count(cj);
        }
        double* S = sw.buf(g);
        double* Vt = (wide || tall_gather) ? sw.buf(g * g) : sw.core(g * g);
        int* js = status + kJacobiSlot + int(jst.size());
        if (use_eig) sym_eig_top(h, P, int(g), int(g), int(kk), S, nullptr, Vt, int(g), js);   // (S <- lambda)
        else jacobi_vt(h, L, int(g), true, int(g), int(g), S, Vt, int(g), js);
        jst.push_back(js);
        double* Tk = sw.buf(r * kk);
        double* newk;
        if (wide) {   // Vt holds U_L^T (P = B B^T = L L^T, B = L Q, L = U S V^T)
            double* M = sw.buf(kk * r);
            hipLaunchKernelGGL(k_edge_factors, dim3(unsigned(std::min<size_t>((kk * r + 255) / 256, 512))), dim3(256), 0,
                               h->stream, Vt, S, int(r), int(kk), M, Tk, int(use_eig));
            check_launch("k_edge_factors");
            newk = sw.core(kk * N);
            gemm(h, newk, kk, N, 1.0, M, r, false, r, B, N, false);               // S^{-1} U^T B = Vt_B[:kk]
        } else {      // Vt holds the right singular vectors of L^T = those of B (B = Q L^T)
            if (tall_gather) {   // this rank's columns (mode slices) of the first kk rows
                newk = sw.core(kk * N);
                slice_core(t, Vt, kk, ng[k], rr[k + 1], lay.off[k], t.n[k], newk);
            } else {
                newk = Vt;                                                        // first kk rows
            }
            gemm(h, Tk, r, kk, 1.0, B, Nw, false, Nw, Vt, Nw, true);              // U S = B Vt_kk^T
        }
        const size_t prow = t.rows_left(k - 1);   // = rr[k-1] * n[k-1] (left ranks unchanged so far)
        double* prevk = sw.core(prow * kk);
        gemm(h, prevk, prow, kk, 1.0, A[k - 1], r, false, r, Tk, kk, false);
        sw.drop(A[k]);
        sw.drop(A[k - 1]);
        A[k] = newk;
        A[k - 1] = prevk;
        rr[k] = kk;
    }
    flush_certs();
    if (side_used) {   // join: the side stream's certificates before the statuses are read
        XRS_HIP(hipEventRecord(h->ev_join[0], h->side_stream[0]));
        XRS_HIP(hipStreamWaitEvent(h->stream, h->ev_join[0], 0));
    }
    // right-orthonormality of the new cores 1..d-1
    {
        std::vector<const double*> X;
        std::vector<size_t> m, n;
        for (size_t k = 1; k < d; ++k) {
            X.push_back(A[k]);
            m.push_back(rr[k]);
            n.push_back(t.n[k] * rr[k + 1]);   // (local columns; the Grams are all-reduced)
        }
        orth_devs(sw, X, m, n, true, devb.d());
    }
    const int nchk2 = int(d - 1) * 16;
    XRS_HIP(hipMemcpyAsync(hs, status, size_t(kStatusWords) * 4, hipMemcpyDeviceToHost, h->stream));
    XRS_HIP(hipMemcpyAsync(hd, devb.d(), size_t(nchk2) * 8, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    bool ok = true;
    for (int i = 0; i < nst; ++i) ok = ok && hs[i] == 0;
    int max_sweeps = 0;
    for (size_t i = 0; i < jst.size(); ++i) {
        const int s = hs[kJacobiSlot + int(i)];
        ok = ok && s >= 0;
        max_sweeps = std::max(max_sweeps, s);
    }
    worst = 0.0;
    for (int i = 0; i < nchk2; ++i) worst = (hd[i] > worst || hd[i] != hd[i]) ? hd[i] : worst;
    if (dbg) std::fprintf(stderr, "round_truncate: sweep %s, max Jacobi sweeps %d, orthogonality %.3e\n",
                          ok ? "certified" : "NOT certified", max_sweeps, worst);
    if (!ok || !(worst <= kTruncAcceptTol)) {
        sw.discard();
        return false;
    }
    for (size_t k = 0; k < d; ++k) t.replace(k, A[k]);
    sw.owned.clear();
    for (size_t k = 1; k < d; ++k) t.r[k] = rr[k];
    // the new cores S^-1 U^T B carry kappa(B_kk)^2 u of non-orthogonality: one chain pass if that is
    // above the canonical-form tolerance (the represented tensor and the ranks are final already)
    if (worst > kTruncOrthTol) {
        const bool re = reorthonormalize(t);
        if (dbg) std::fprintf(stderr, "round_truncate: re-orthonormalised (%s)\n", re ? "ok" : "failed");
    }
    return true;
}

// ================================================================================================
// General truncating round (any spectrum, maxRank and eps cuts): the reference's two sweeps
// (ttNetwork.cpp:644-665) with every factorisation enqueued and no host synchronisation per edge.
//  1. left to right (canonicalize_right): core_k = Q_k R_k by shifted CholeskyQR3 (Fukaya et al. 2020;
//     backward stable for kappa < 1/u), core_{k+1} <- R_k core_{k+1}. The reference's QC drops a rank only
//     when a pivoted |R_jj| < 16 u R_00 (blasLapackWrapper.cpp:268-272); every R_jj of any triangular
//     factor is >= sigma_min, and sigma_min >= 1 / ||R^{-1}||_F, so a device certificate
//     1 / ||R^{-1}||_F > 32 u ||A||_F proves that no rank drops (else the round falls back);
//  2. right to left (round_edge, tensorNetwork.cpp:678-818): B = core_k (r x N) = L Q by the same
//     factorisation (wide), the right singular vectors and values of L by one-sided Jacobi on its rows
//     (svd.hip; singular values to u ||B|| absolute, so eps cuts far below sqrt(u) are decided on
//     accurate values), the cut of calculate_svd (tensor.cpp:1462-1474) evaluated ON THE DEVICE
//     (k_cut_rows), core_k <- V_kk^T Q, core_{k-1} <- core_{k-1} L V_kk (= U S). Ranks are not
//     known on the host until the end: the sweep keeps the uncut sizes with zero rows / columns beyond
//     the device-side rank, and the cores are compacted once after the single synchronisation.
// Tall edges (r > N: structural excess at the right end, e.g. x + y) use B = Q R and the right singular
// vectors of R. Certificates that fail (rank drop possible, Cholesky breakdown, Jacobi not converged,
// non-orthonormal result) discard the new cores; the caller then runs the reference's sequential sweep.
namespace {

constexpr double kUnit = 1.1102230246251565e-16;   // 2^-53

// flag = 1 unless 1 / ||W||_F > c ||A||_F, W = R^{-1}, ||A||_F^2 = trG[0] (potrf's trace output)
__global__ void __launch_bounds__(256) k_rank_cert(const double* __restrict__ W, int n, const double* __restrict__ trG, double c,
                                                   int* __restrict__ flag) {
    __shared__ double red[4];
    double s = 0.0;
    for (int e = threadIdx.x; e < n * n; e += 256) s = fma(W[e], W[e], s);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double w2 = (red[0] + red[1]) + (red[2] + red[3]);
        // 1 / ||W|| > c ||A||  <=>  c^2 ||W||^2 ||A||^2 < 1  (NaN -> flagged)
        flag[0] = (c * c * w2 * trG[0] < 1.0) ? 0 : 1;
    }
}

// rank cut of calculate_svd on the device: kk = min(r, max_rank), then the first j >= 1 with
// S_j <= eps S_0 (tensor.cpp:1462-1474). Every workgroup recomputes it (S is r <= 1024 doubles).
__device__ int device_cut(const double* __restrict__ S, int r, long max_rank, double eps) {
    __shared__ int best;
    if (threadIdx.x == 0) best = int(std::min<long>(r, max_rank));
    __syncthreads();
    const double thr = eps * S[0];
    for (int j = 1 + int(threadIdx.x); j < r; j += int(blockDim.x))
        if (S[j] <= thr) atomicMin(&best, j);
    __syncthreads();
    return best;
}

// V (g x g): right singular vectors of the edge factor as rows (S descending); rows >= kk zeroed in place
__global__ void __launch_bounds__(256) k_cut_rows(double* __restrict__ Vt, const double* __restrict__ S, int g, long max_rank, double eps,
                                                  int* __restrict__ kk_out) {
    const int kk = device_cut(S, g, max_rank, eps);
    if (blockIdx.x == 0 && threadIdx.x == 0) kk_out[0] = kk;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < g * g; e += gridDim.x * 256)
        if (e / g >= kk) Vt[e] = 0.0;
}

// X[i][i] += v (n x n)
__global__ void k_add_identity(double* __restrict__ X, int n, double v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) X[size_t(i) * n + i] += v;
}

// Tall edges of the general round: after the cut of edge k + 1 the columns (i, b) of core_k with b >= the
// device rank *kk (the padded ones) are exactly zero, so the Gram X^T X has exactly zero rows / columns
// there. fill: those diagonal entries become the largest diagonal entry (the Cholesky factors the two
// blocks independently and Q keeps zero columns there); fill = false: the final factor's padded diagonal
// back to zero (R's padded rows / columns are then exactly zero: singular values 0, cut by the rank rule).
__global__ void __launch_bounds__(256) k_pad_diag(double* __restrict__ G, int N, int b, const int* __restrict__ kk, bool fill) {
    __shared__ double red[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int keep = *kk;
    double v = 0.0;
    if (fill) {
        for (int p = t; p < N; p += 256) v = fmax(v, G[size_t(p) * N + p]);
        for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
        if (lane == 0) red[w] = v;
        __syncthreads();
        v = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
        if (!(v > 0.0)) v = 1.0;
    }
    for (int p = t; p < N; p += 256)
        if (p % b >= keep) G[size_t(p) * N + p] = v;
}

// flag = 1 unless 1 / ||W||_F > c ||X||_F with ||X||_F^2 = trace(G) (G: n x n Gram of the unfolding)
__global__ void __launch_bounds__(256) k_rank_cert_gram(const double* __restrict__ W, const double* __restrict__ G, int n, double c,
                                                        int* __restrict__ flag) {
    __shared__ double red[8];
    double s = 0.0, tr = 0.0;
    for (int e = threadIdx.x; e < n * n; e += 256) s = fma(W[e], W[e], s);
    for (int i = threadIdx.x; i < n; i += 256) tr += G[size_t(i) * n + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        tr += __shfl_xor(tr, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = s;
        red[4 + (threadIdx.x >> 6)] = tr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double w2 = (red[0] + red[1]) + (red[2] + red[3]), t2 = (red[4] + red[5]) + (red[6] + red[7]);
        flag[0] = (c * c * w2 * t2 < 1.0) ? 0 : 1;
    }
}

unsigned grid_for(size_t elems) { return unsigned(std::min<size_t>(std::max<size_t>((elems + 255) / 256, 1), 256)); }

// Shifted CholeskyQR3, enqueued: tall A (m x n, m >= n) = Q R (RL = R, upper, n x n), or wide A (m x n,
// m <= n) = L Q (RL = L, lower, m x m). st[0..3) potrf statuses; trG[0] = ||A||_F^2; with Rinv, the
// explicit inverse of the triangular factor (tall: R^{-1} transposed, i.e. L3^{-1} L2^{-1} L1^{-1} --
// same Frobenius norm). N = min(m, n) <= 512. pad_kk (tall only): the columns p with p % pad_b >= *pad_kk are
// known to be zero (k_pad_diag). reduce (sharded): the Grams are sums over the ranks' blocks of the long
// dimension, all-reduced; Mg = its global length (the shift must be the same on every rank).
void scqr3(Sweep& sw, const double* A, size_t m, size_t n, bool wide, double* Q, double* RL, int* st, double* trG, double* Rinv,
           const int* pad_kk = nullptr, int pad_b = 1, bool reduce = false, size_t Mg = 0) {
    xrs_handle_t h = sw.t.h;
    const size_t N = wide ? m : n, M = wide ? n : m;
    const int Ni = int(N);
    double* G = sw.buf(N * N);
    double* L[3] = {sw.buf(N * N), sw.buf(N * N), sw.buf(N * N)};
    double* Dv[3] = {sw.buf(dinv_elems(Ni)), sw.buf(dinv_elems(Ni)), sw.buf(dinv_elems(Ni))};
    double* X1 = sw.buf(m * n);
    double* X2 = sw.buf(m * n);
    double* info = sw.buf(4);
    const double s_rel = 11.0 * (double(Mg ? Mg : M) * N + double(N) * (N + 1)) * kUnit;
    const double* cur = A;
    double* outs[3] = {X1, X2, Q};
    for (int p = 0; p < 3; ++p) {
        if (wide) gemm_sym(h, L[p], N, 1.0, cur, n, false, M, cur, n, true);   // X X^T
        else gemm_sym(h, L[p], N, 1.0, cur, n, true, M, cur, n, false);        // X^T X
        if (reduce) sw.t.reduce(L[p], N * N);
        if (pad_kk && !wide) {
            hipLaunchKernelGGL(k_pad_diag, dim3(1), dim3(256), 0, h->stream, L[p], Ni, pad_b, pad_kk, true);
            check_launch("k_pad_diag");
        }
        potrf(h, L[p], Ni, p == 0 ? s_rel : 0.0, Dv[p], st + p, p == 0 ? info : nullptr);
        trsm(h, wide, L[p], Dv[p], Ni, cur, n, outs[p], n, int(M));           // tall: X L^{-T}, wide: L^{-1} X
        cur = outs[p];
    }
    if (trG) XRS_HIP(hipMemcpyAsync(trG, info, 8, hipMemcpyDeviceToDevice, h->stream));
    // RL = L1 L2 L3 (wide) / R = L3^T L2^T L1^T (tall); potrf leaves the upper triangles zero
    if (wide) {
        gemm(h, G, N, N, 1.0, L[0], N, false, N, L[1], N, false);
        gemm(h, RL, N, N, 1.0, G, N, false, N, L[2], N, false);
    } else {
        gemm(h, G, N, N, 1.0, L[2], N, true, N, L[1], N, true);
        gemm(h, RL, N, N, 1.0, G, N, false, N, L[0], N, true);
        if (pad_kk) {
            hipLaunchKernelGGL(k_pad_diag, dim3(1), dim3(256), 0, h->stream, RL, Ni, pad_b, pad_kk, false);
            check_launch("k_pad_diag");
        }
    }
    if (Rinv) {   // L3^{-1} L2^{-1} L1^{-1} from the identity by three column TRSMs
        double* I0 = sw.buf(N * N);
        double* I1 = sw.buf(N * N);
        XRS_HIP(hipMemsetAsync(I0, 0, N * N * 8, h->stream));
        hipLaunchKernelGGL(k_add_identity, dim3(grid_for(N)), dim3(256), 0, h->stream, I0, Ni, 1.0);
        check_launch("k_add_identity");
        trsm(h, true, L[0], Dv[0], Ni, I0, N, I1, N, Ni);
        trsm(h, true, L[1], Dv[1], Ni, I1, N, I0, N, Ni);
        trsm(h, true, L[2], Dv[2], Ni, I0, N, Rinv, N, Ni);
    }
}

}  // namespace

// xerus::EPSILON, the default eps of round(maxRanks): an eps above it may cut an edge arbitrarily deep
constexpr double kDefaultEps = 8 * 2.220446049250313e-16;

bool round_general(TT& t, const size_t* max_ranks, double eps) {
    const size_t d = t.d;
    xrs_handle_t h = t.h;
    static const bool dbg = std::getenv("XRS_DEBUG_ROUND") != nullptr;
    if (d < 2 || d > 64) return false;
    for (size_t k = 1; k < d; ++k)
        if (t.r[k] > size_t(kSmallMax)) return false;

    // global mode sizes / this rank's slice offsets (sharded: one all-reduce + host sync); structural excess
    // at the left end (r_{k+1} > r_k n_k): the reference's own QC steps (as round_truncate)
    const ShardLayout lay = shard_layout(t);
    const std::vector<size_t>& ng = lay.ng;
    const bool sharded = t.sharded();
    remove_left_excess(t, lay);

    Sweep sw(t);
    constexpr int kSlots = 2048;
    DevBuf stb(h, kSlots * 4), devb(h, 64 * 16 * 8);
    int* st = stb.as<int>();
    XRS_HIP(hipMemsetAsync(st, 0, kSlots * 4, h->stream));
    int nst = 0;
    const int kJac = 1536, kRank = 1792;   // Jacobi sweep counts; device ranks

    std::vector<double*> A(t.core, t.core + d);   // current cores (originals untouched)
    std::vector<size_t> rr(t.r, t.r + d + 1);
    int* hs = static_cast<int*>(h->host_scratch) + 12288;

    // 1a. left to right as shifted CholeskyQR3 over the whole train: three chain passes (Gram chain
    //     G_{k+1} = M_k^T (G_k (x) I) M_k, ONE batched Cholesky launch of G_k + s tr(G_k) I (first pass) /
    //     G_k, grouped transforms A_k = (L_k^T (x) I) M_k L_{k+1}^{-T}) -- the left-orthonormal train
    //     without a sequential factorisation chain. Per edge R_k = L3^T L2^T L1^T, R_k^{-1} = Z1^T Z2^T Z3^T
    //     gives the rank certificate; the orthonormality of the result is checked. One synchronisation.
    bool chain_ok = false;
    {
        size_t mmax = 1, rmax = 1;
        for (size_t k = 0; k < d; ++k) {
            mmax = std::max(mmax, rr[k] * ng[k]);
            rmax = std::max(rmax, rr[k + 1]);
        }
        const double s_rel = 11.0 * kUnit * (double(mmax) * double(d) + double(rmax) * double(rmax + 1));
        std::vector<double*> A1, A2, A3, G1, Z1, Z2, Z3;
        int cst = 0;
        left_pass(sw, t, t.core, false, A1, st, cst, s_rel, &G1, &Z1);
        left_pass(sw, t, A1.data(), false, A2, st, cst, 0.0, nullptr, &Z2);
        left_pass(sw, t, A2.data(), false, A3, st, cst, 0.0, nullptr, &Z3);
        for (double* p : A1) sw.drop(p);
        for (double* p : A2) sw.drop(p);
        // W_k = Z3 Z2 Z1 (= (R_k^{-1})^T), batched over the edges
        std::vector<GemmJob> j1, j2;
        std::vector<double*> W1(d, nullptr), W(d, nullptr);
        for (size_t k = 1; k < d; ++k) {
            const size_t a = rr[k];
            W1[k] = sw.buf(a * a);
            W[k] = sw.buf(a * a);
            j1.push_back({a, a, a, a, a, false, false, Z2[k], Z1[k], W1[k]});
            j2.push_back({a, a, a, a, a, false, false, Z3[k], W1[k], W[k]});
        }
        gemm_grouped(h, j1);
        gemm_grouped(h, j2);
        const int crank = cst;
        for (size_t k = 1; k < d; ++k) {
            hipLaunchKernelGGL(k_rank_cert_gram, dim3(1), dim3(256), 0, h->stream, W[k], G1[k], int(rr[k]), 32.0 * kUnit, st + cst);
            check_launch("k_rank_cert_gram");
            ++cst;
        }
        {
            std::vector<const double*> X;
            std::vector<size_t> m, n;
            for (size_t k = 0; k + 1 < d; ++k) {
                X.push_back(A3[k]);
                m.push_back(rr[k] * t.n[k]);
                n.push_back(rr[k + 1]);
            }
            orth_devs(sw, X, m, n, false, devb.d());
        }
        double* hd = static_cast<double*>(h->host_scratch) + 2048;
        const int nchk = int(d - 1) * 16;
        XRS_HIP(hipMemcpyAsync(hs, st, size_t(cst) * 4, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipMemcpyAsync(hd, devb.d(), size_t(nchk) * 8, hipMemcpyDeviceToHost, h->stream));
        host_wait(h);
        chain_ok = true;
        int first_bad = -1;
        for (int i = 0; i < cst; ++i)
            if (hs[i] != 0) {
                chain_ok = false;
                first_bad = i;
                break;
            }
        double worst = 0.0;
        for (int i = 0; i < nchk; ++i) worst = (hd[i] > worst || hd[i] != hd[i]) ? hd[i] : worst;
        chain_ok = chain_ok && worst <= kTruncOrthTol;
        if (dbg)
            std::fprintf(stderr, "round_general: chain left sweep %s (first bad slot %d of %d, rank certificates from %d), orthogonality %.3e\n",
                         chain_ok ? "certified" : "NOT certified", first_bad, cst, crank, worst);
        if (chain_ok) {
            A = A3;
        } else {
            for (double* p : A3) sw.drop(p);
        }
        XRS_HIP(hipMemsetAsync(st, 0, size_t(cst) * 4, h->stream));
    }

    // 1b. otherwise core by core: A_k = Q_k, next = R_k core_{k+1}, each by shifted CholeskyQR3
    for (size_t k = 0; !chain_ok && k + 1 < d; ++k) {
        const size_t m = rr[k] * t.n[k], b = rr[k + 1];
        if (rr[k] * ng[k] < b) {   // (sharded with an unknown layout: the excess could not be removed)
            sw.discard();
            return false;
        }
        double* Q = sw.core(m * b);
        double* R = sw.buf(b * b);
        double* Rinv = sw.buf(b * b);
        double* trG = sw.buf(1);
        scqr3(sw, A[k], m, b, false, Q, R, st + nst, trG, Rinv, nullptr, 1, sharded, rr[k] * ng[k]);
        nst += 3;
        hipLaunchKernelGGL(k_rank_cert, dim3(1), dim3(256), 0, h->stream, Rinv, int(b), trG, 32.0 * kUnit, st + nst);
        check_launch("k_rank_cert");
        ++nst;
        const size_t cols = t.n[k + 1] * rr[k + 2];
        double* nxt = sw.core(b * cols);
        gemm(h, nxt, b, cols, 1.0, R, b, false, b, A[k + 1], cols, false);
        sw.drop(A[k]);   // (an intermediate core of this sweep; the originals are not owned)
        A[k] = Q;
        A[k + 1] = nxt;
    }
    open_dot_gate(h);

    // 2. right to left, uncut (padded) sizes: g[k] = working rank of edge k
    std::vector<size_t> g(rr);
    std::vector<int> jac;
    int nsync = 0;
    for (size_t k = d - 1; k >= 1; --k) {
        // After the cut of edge k + 1 to its device rank kk, core_k keeps n_k (g_{k+1} - kk) zero columns. If
        // r_k > n_k kk, its unfolding has rank < r_k: a wide Gram B B^T would be exactly singular (tall ones
        // are masked, k_pad_diag). When the cut can go that deep (an eps cut, or maxRank n_k < r_k), read kk
        // (one synchronisation) and compact core_k to its kk right columns; core_{k+1}'s first kk rows
        // already hold the kept rows.
        if (k + 1 < d && g[k] > ng[k] && (eps > kDefaultEps || max_ranks[k] * ng[k] < g[k])) {
            int* kh = hs + kSlots - 1;
            XRS_HIP(hipMemcpyAsync(kh, st + kRank + int(k + 1), 4, hipMemcpyDeviceToHost, h->stream));
            host_wait(h);
            ++nsync;
            const size_t v = size_t(*kh);
            if (*kh >= 1 && v < g[k + 1] && v * ng[k] < g[k]) {
                const size_t rows = g[k] * t.n[k], gb = g[k + 1];
                double* Cc = sw.core(rows * v);
                XRS_HIP(hipMemcpy2DAsync(Cc, v * 8, A[k], gb * 8, v * 8, rows, hipMemcpyDeviceToDevice, h->stream));
                sw.drop(A[k]);
                A[k] = Cc;
                g[k + 1] = v;
            }
        }
        const size_t r = g[k], N = t.n[k] * g[k + 1], Ng = ng[k] * g[k + 1];   // local / global columns
        const bool wide = r <= Ng;
        // sharded tall edge: gathered (r x Ng, Ng < r) and factorised replicated (as round_truncate)
        const bool tall_gather = !wide && sharded;
        if (tall_gather && !lay.known) {
            if (dbg) std::fprintf(stderr, "round_general: sharded tall edge %zu, rank layout unknown -> not certified\n", k);
            sw.discard();
            return false;
        }
        const size_t Nw = tall_gather ? Ng : N;
        const size_t gg = wide ? r : Nw;
        double* B = A[k];
        if (tall_gather) {
            B = sw.buf(r * Nw);
            gather_core(t, A[k], r, t.n[k], ng[k], g[k + 1], lay.off[k], B);
        }
        double* Qf = sw.buf(r * Nw);
        double* F = sw.buf(gg * gg);
        // (tall edge after a cut of edge k + 1: its padded zero columns, k_pad_diag)
        const int* pad = (!wide && k + 1 < d) ? st + kRank + int(k + 1) : nullptr;
        scqr3(sw, B, r, Nw, wide, Qf, F, st + nst, nullptr, nullptr, pad, int(g[k + 1]), wide && sharded, Ng);
        nst += 3;
        double* S = sw.buf(gg);
        double* V = sw.buf(gg * gg);
        int* js = st + kJac + int(jac.size());
        // right singular vectors of the triangular factor by one-sided Jacobi (svd.hip jacobi_right_vectors:
        // wide L through its columns with the rotations accumulated, tall R through its rows): accurate to u
        // whatever the singular value (no division by S), so the new core V_kk^T Q has orthonormal rows to
        // ~u even after eps cuts far below sqrt(u)
        static const bool no_early = std::getenv("XRS_JACOBI_NO_EARLY") != nullptr;
        jacobi_right_vectors(h, F, int(gg), wide, S, V, js, 40, !no_early);
        jac.push_back(int(k));
        hipLaunchKernelGGL(k_cut_rows, dim3(grid_for(gg * gg)), dim3(256), 0, h->stream, V, S, int(gg),
                           long(std::min<size_t>(max_ranks[k - 1], size_t(1) << 40)), eps, st + kRank + int(k));
        check_launch("k_cut_rows");   // V rows >= kk zeroed: V_kk^T
        const size_t prow = g[k - 1] * t.n[k - 1];
        double* prevk = sw.core(prow * gg);
        double* newk = sw.core(gg * N);
        double* T = sw.buf(r * gg);
        if (wide) {   // B = L Q, L = U S V^T: core_k <- V_kk^T Q, core_{k-1} <- core_{k-1} (L V_kk) = (U S)_kk
            gemm(h, newk, gg, N, 1.0, V, gg, false, gg, Qf, N, false);
            gemm(h, T, r, gg, 1.0, F, gg, false, gg, V, gg, true);
        } else {      // B = Q R, R = U S V^T: core_k <- V_kk^T, core_{k-1} <- core_{k-1} (B V_kk)
            if (tall_gather) slice_core(t, V, gg, ng[k], g[k + 1], lay.off[k], t.n[k], newk);   // this rank's columns
            else XRS_HIP(hipMemcpyAsync(newk, V, gg * N * 8, hipMemcpyDeviceToDevice, h->stream));
            gemm(h, T, r, gg, 1.0, B, Nw, false, Nw, V, Nw, true);
        }
        gemm(h, prevk, prow, gg, 1.0, A[k - 1], r, false, r, T, gg, false);
        sw.drop(A[k]);
        sw.drop(A[k - 1]);
        A[k] = newk;
        A[k - 1] = prevk;
        g[k] = gg;
    }

    // 3. the synchronisation: statuses, Jacobi sweeps, device ranks
    XRS_HIP(hipMemcpyAsync(hs, st, size_t(kSlots) * 4, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    bool ok = true;
    int bad = -1;
    for (int i = 0; i < nst; ++i)
        if (hs[i] != 0) {
            ok = false;
            bad = i;
            break;
        }
    int max_sweeps = 0;
    for (size_t i = 0; i < jac.size(); ++i) {
        ok = ok && hs[kJac + int(i)] >= 0;
        max_sweeps = std::max(max_sweeps, hs[kJac + int(i)]);
    }
    std::vector<size_t> kk(d + 1, 1);
    for (size_t k = 1; k < d; ++k) {
        const int v = hs[kRank + int(k)];
        ok = ok && v >= 1 && size_t(v) <= g[k];
        kk[k] = size_t(std::max(v, 1));
    }
    if (dbg) {
        std::fprintf(stderr, "round_general: %s (first failing status slot %d), max Jacobi sweeps %d, %d rank read-backs; per edge:",
                     ok ? "certified" : "NOT certified", bad, max_sweeps, nsync);
        for (size_t i = 0; i < jac.size(); ++i) std::fprintf(stderr, " %d:%d", jac[i], hs[kJac + int(i)]);
        std::fprintf(stderr, "\n");
    }
    if (!ok) {
        sw.discard();
        return false;
    }
    // 4. compaction to the device ranks: core_k[:kk_k, :, :kk_{k+1}]
    std::vector<double*> C(d, nullptr);
    for (size_t k = 0; k < d; ++k) {
        const size_t a = kk[k], n = t.n[k], b = kk[k + 1], ga = g[k], gb = g[k + 1];
        if (a == ga && b == gb) {
            C[k] = A[k];
            continue;
        }
        C[k] = sw.core(a * n * b);
        // rows (i, j) of the (ga n) x gb matrix with i < a, first b columns
        XRS_HIP(hipMemcpy2DAsync(C[k], b * 8, A[k], gb * 8, b * 8, a * n, hipMemcpyDeviceToDevice, h->stream));
        sw.drop(A[k]);
    }
    // right-orthonormality of cores 1..d-1 (S^{-1} U^T B carries kappa(B_kk) u of deviation)
    {
        std::vector<const double*> X;
        std::vector<size_t> m, n;
        for (size_t k = 1; k < d; ++k) {
            X.push_back(C[k]);
            m.push_back(kk[k]);
            n.push_back(t.n[k] * kk[k + 1]);
        }
        orth_devs(sw, X, m, n, true, devb.d());
    }
    double* hd = static_cast<double*>(h->host_scratch) + 2048;
    const int nchk = int(d - 1) * 16;
    XRS_HIP(hipMemcpyAsync(hd, devb.d(), size_t(nchk) * 8, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    double worst = 0.0;
    for (int i = 0; i < nchk; ++i) worst = (hd[i] > worst || hd[i] != hd[i]) ? hd[i] : worst;
    if (dbg) std::fprintf(stderr, "round_general: right orthogonality %.3e\n", worst);
    if (!(worst <= kTruncAcceptTol)) {
        sw.discard();
        return false;
    }
    for (size_t k = 0; k < d; ++k) t.replace(k, C[k]);
    sw.owned.clear();
    for (size_t k = 1; k < d; ++k) t.r[k] = kk[k];
    if (worst > kTruncOrthTol) {
        const bool re = reorthonormalize(t);
        if (dbg) std::fprintf(stderr, "round_general: re-orthonormalised (%s)\n", re ? "ok" : "failed");
    }
    return true;
}

}  // namespace ttd
}  // namespace xrs
