// Internal interface of the TT drivers (tt.hip: move_core, certified chain round, <x,y>; tt_trunc.hip:
// the certified truncating round). Not part of the C-ABI.
#pragma once
#include <vector>

#include "smallla.hpp"

namespace xrs {
// start a gated asynchronous inner product of the handle behind its current stream point (tt.hip)
void open_dot_gate(xrs_handle_t h);

namespace ttd {

struct TT {
    xrs_handle_t h;
    size_t d;
    const size_t* n;
    size_t* r;      // d + 1 ranks, r[0] = r[d] = 1
    double** core;

    size_t rows_left(size_t k) const { return r[k] * n[k]; }      // (r_k n_k) x r_{k+1}
    size_t cols_right(size_t k) const { return n[k] * r[k + 1]; }  // r_k x (n_k r_{k+1})
    size_t size(size_t k) const { return r[k] * n[k] * r[k + 1]; }

    double* alloc(size_t elems) { return static_cast<double*>(h->pool->alloc(std::max<size_t>(elems, 1) * 8)); }
    void release(double* p) {
        if (!p) return;
        fence_readers(h);   // an in-flight async inner product may still read the block
        h->pool->release(p);
    }
    void replace(size_t k, double* p) { release(core[k]); core[k] = p; }

    // Mode-sharded TT (xrs_tt_*_sharded): n[] are this rank's slice counts and every sum over the
    // mode index is completed by an all-reduce across ranks; null for a whole TT on one device.
    // shard_mode without a hook: a single rank (the local sums are the global ones, no synchronisation)
    bool shard_mode = false;
    xrs_allreduce_fn ar = nullptr;
    void* ar_ctx = nullptr;
    // the ranks' layout (xrs_tt_round_sharded_ex): world > 0 when known; each rank holds a contiguous block
    // of every mode, blocks in rank order. Unknown (0): cores whose unfolding spans the ranks' blocks
    // (tall right edges, structural-excess QC steps) cannot be gathered and the round reports uncertified
    int world = 0;
    int rank = 0;
    // shard_layout's result, computed once per TT (its all-reduce and host wait are paid once per round even
    // when the certified truncation falls through to the general round)
    bool layout_cached = false;
    std::vector<size_t> layout_ng, layout_off;
    bool layout_known = false;
    bool sharded() const { return shard_mode; }
    void reduce(double* buf, size_t count) const {
        if (!ar) return;
        // the built-in RCCL hook is stream-ordered; any other hook sees a synchronised stream
        if (ar != &xrs_comm_allreduce) XRS_HIP(hipStreamSynchronize(h->stream));
        const int rc = ar(ar_ctx, buf, count);
        XRS_REQUIRE(rc == 0, "all-reduce callback failed");
    }
};

// Mode layout of a sharded TT (tt_trunc.hip): global mode sizes ng, this rank's first slice off per mode;
// known = false when the ranks' order is unknown (world 0) -- then off is meaningless.
struct ShardLayout {
    std::vector<size_t> ng, off;
    bool known = true;
};
ShardLayout shard_layout(TT& t);
void gather_core(TT& t, const double* local, size_t a, size_t nl, size_t ng, size_t b, size_t off, double* full);
void slice_core(TT& t, const double* full, size_t a, size_t ng, size_t b, size_t off, size_t nl, double* local);
void transfer_right_sharded(TT& t, size_t k, const ShardLayout& lay);
void remove_left_excess(TT& t, const ShardLayout& lay);

// reduce_to_maximal_ranks (ttNetwork.cpp:370-402) of the internal ranks; true if any rank exceeds it
std::vector<size_t> maximal_ranks(const TT& t);
bool exceeds_maximal_ranks(const TT& t);

// relative downward shift of the certifying Cholesky factorisations (see tt.hip, round_chain)
constexpr double kGramShift = 1e-11;
constexpr double kOrthTol = 1e-13;   // max |C_k C_k^T - I| accepted for the right-canonical cores

// Gram chains (k = 1..d-1): left G_{k+1} = M_k^T (G_k M_k), right H_k = M_k (I (x) H_{k+1}) M_k^T
void left_gram_step(TT& t, std::vector<double*>& G, double* T, size_t k, bool do_reduce = true);
void right_gram_step(TT& t, std::vector<double*>& H, double* T, size_t k, bool do_reduce = true);
void gram_chains(TT& t, std::vector<double*>& G, std::vector<double*>& H, std::vector<DevBuf>& store, bool left = true);

struct DevIdArgs {
    const double* G[64];
    int n[64];
    double* out;
};
// max |G_i - I| of a batch of square matrices; out[i * gridDim.y + slice]
__global__ void k_dev_identity_many(const DevIdArgs args);

// Independent GEMMs; the ones of identical shape go out as one batched launch.
struct GemmJob {
    size_t M, N, K, lda, ldb;
    bool ta, tb;
    const double* A;
    const double* B;
    double* C;
    bool sym = false;   // result known symmetric (M == N): lower tiles only, mirrored
    double alpha = 1.0;
    int tri = 0;        // triangular operands (kTriA / kTriB, gemm): zero K-blocks skipped
};
void gemm_grouped(xrs_handle_t h, const std::vector<GemmJob>& jobs);

// Cholesky (+ explicit inverse) of 256 < n <= 512 matrices from the n <= 256 kernels (2 x 2 blocks)
constexpr int kBigMax = 64;
// largest rank of the certified chain / truncating rounds (blocked Cholesky above 512, the 1024-column
// register tiling of the block Jacobi SVD)
constexpr size_t kHugeMax = 1024;
struct BigJob {
    const double* src;
    double shift_rel;
    int n;
    double* L;   // factor jobs: full L and Z = L^{-1} (n x n); certificates: both null
    double* Z;
};
void factor_big(xrs_handle_t h, const std::vector<BigJob>& jobs, int* status, std::vector<DevBuf>& keep);

// the reference's two-sweep algorithm pieces (sequential, host-synchronising)
void transfer_right(TT& t, size_t k, bool rank_reduce);   // transfer_core(k -> k+1): QC (or QR) + R * next
void orth_right(TT& t, size_t k);
size_t svd_cut(const std::vector<double>& s, size_t max_rank, double eps);
// round_edge (tensorNetwork.cpp:678-818) of the edge k-1 | k, core moving to k-1; soft > 0 replaces the
// kept singular values by max(0, sigma - soft) (round_edge's _softThreshold, :766 / :788)
void truncate_edge(TT& t, size_t k, size_t max_rank, double eps, double soft = 0.0);
// TTNetwork::soft_threshold (ttNetwork.cpp:688-713): canonicalize_right, then round_edge(maxRank = inf,
// eps = 0, soft = taus[i]) over the edges right to left, taus[0] at the last edge (the reference's order)
void soft_threshold(TT& t, bool canonicalized, size_t core_pos, const double* taus);

// one right chain pass restoring right-orthonormality of nearly orthonormal cores (tt.hip)
bool reorthonormalize(TT& t);

// certified truncating round (tt_trunc.hip): left-canonical chain pass + device-resident right-to-left
// truncation sweep with one host synchronisation; false (cores untouched) when a certificate fails
bool round_truncate(TT& t, const size_t* max_ranks, double eps);

// general truncating round (tt_trunc.hip): any spectrum, maxRank and eps cuts, shifted CholeskyQR3 +
// Jacobi SVD per edge, enqueued with device-side rank cuts and one synchronisation; false (cores
// untouched) when a certificate fails (possible QC rank drop, breakdown, non-orthonormal result)
bool round_general(TT& t, const size_t* max_ranks, double eps);

}  // namespace ttd
}  // namespace xrs
