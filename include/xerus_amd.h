/*
 * xerus_amd.h — C-ABI of the MI355X-native xerus hot path (dense contraction + TT rounding).
 *
 * The reference (xerus v3.0.1, /root/reference) has no plugin registry; its narrowest internal
 * boundary is the free-function namespace xerus::blasWrapper over raw row-major double*
 * (include/xerus/blasLapackWrapper.h:37-146) plus the Tensor-level reshuffle/contract
 * (include/xerus/tensor.h:56-66). Every entry point below replaces one of those and cites it.
 *
 * Conventions (identical to the reference unless stated):
 *   - element type double (include/xerus/basic.h:44), all matrices ROW-MAJOR, dims are size_t;
 *   - every data pointer is a DEVICE pointer (allocated with xrs_malloc or any hipMalloc'd memory
 *     of the handle's device); host<->device traffic happens only in xrs_upload/xrs_download and
 *     in the few functions that return a scalar (documented per function);
 *   - work is enqueued on the handle's stream; functions that must return a host value
 *     (rank, norm) synchronise that stream;
 *   - return value: 0 = ok, < 0 = argument error (reference: XERUS_REQUIRE -> generic_error,
 *     misc/check.h:60-65), > 0 = numerical failure (reference: LAPACK info != 0,
 *     blasLapackWrapper.cpp:263,290,409). xrs_last_error() returns the message of the last
 *     failure on the calling host thread.
 *   - the library never frees caller buffers (SURVEY §8(b) "Ownership"). Functions that must
 *     allocate because the rank is data dependent (QC/CQ, TT round) write into caller-provided
 *     buffers sized for the maximal rank min(m,n) and return the rank.
 *   - one handle per host thread (a stream + a caching device allocator); no global mutable state
 *     besides the thread-local error string.
 */
#ifndef XERUS_AMD_H
#define XERUS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct xrs_handle_s* xrs_handle_t;

#define XRS_OK 0
#define XRS_EINVAL (-1)      /* illegal argument (reference: REQUIRE failure)           */
#define XRS_ENOMEM (-2)      /* device allocation failed                                */
#define XRS_EHIP (-3)        /* HIP runtime error                                       */
#define XRS_ENUMERIC 1       /* numerical failure (reference: LAPACK info != 0)          */

/* ---------------------------------------------------------------- runtime */
/** Create a handle on device `device` with its own non-blocking stream. */
int xrs_create(xrs_handle_t* handle, int device);
int xrs_destroy(xrs_handle_t handle);
/** Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). NULL = own stream. */
int xrs_set_stream(xrs_handle_t handle, void* hip_stream);
void* xrs_get_stream(xrs_handle_t handle);
int xrs_synchronize(xrs_handle_t handle);
const char* xrs_last_error(void);
const char* xrs_version(void);

/** Stream-ordered caching allocator of the handle (blocks are reused, never hipFree'd in flight). */
int xrs_malloc(xrs_handle_t handle, void** ptr, size_t bytes);
int xrs_free(xrs_handle_t handle, void* ptr);
/** Bytes currently held by the handle's pool (in use + cached). */
size_t xrs_pool_bytes(xrs_handle_t handle);
int xrs_upload(xrs_handle_t handle, double* dst_dev, const double* src_host, size_t n);
int xrs_download(xrs_handle_t handle, double* dst_host, const double* src_dev, size_t n);
int xrs_memset_zero(xrs_handle_t handle, double* dst_dev, size_t n);
int xrs_copy(xrs_handle_t handle, double* dst_dev, const double* src_dev, size_t n);

/* ---------------------------------------------------------------- level 1 (blasLapackWrapper.h:42-48) */
/** *result = ||x||_2   (replaces blasWrapper::two_norm, blasLapackWrapper.cpp:88-98). Synchronises. */
int xrs_nrm2(xrs_handle_t handle, double* result, const double* x, size_t n);
/** *result = x^T y     (replaces blasWrapper::dot_product, blasLapackWrapper.cpp:101-110). Synchronises. */
int xrs_dot(xrs_handle_t handle, double* result, const double* x, const double* y, size_t n);
/** *result = ||x||_1   (replaces blasWrapper::one_norm, blasLapackWrapper.cpp:76-86). Synchronises. */
int xrs_asum(xrs_handle_t handle, double* result, const double* x, size_t n);
/** x *= alpha          (replaces misc::scale / Tensor::apply_factor, misc/basicArraySupport.h:60-70). */
int xrs_scal(xrs_handle_t handle, double* x, double alpha, size_t n);
/** y += alpha*x        (replaces misc::add_scaled, misc/basicArraySupport.h:90-110). */
int xrs_axpy(xrs_handle_t handle, double* y, double alpha, const double* x, size_t n);
/** X[i,:] *= s[i], X is m x n (replaces the diag(S)*dense product of round_edge,
 *  sparseTimesFullContraction.cpp:66-96 dispatched from tensorNetwork.cpp:769). */
int xrs_scale_rows(xrs_handle_t handle, double* X, const double* s, size_t m, size_t n);

/* ---------------------------------------------------------------- level 3 (blasLapackWrapper.h:61-85) */
/** C = alpha * op(A) * op(B), beta = 0, row-major, ldc = N.
 *  Replaces blasWrapper::matrix_matrix_product (blasLapackWrapper.cpp:149-195) with the same
 *  argument order: M = _leftDim, N = _rightDim, K = _middleDim, lda = transA ? M : K in the inline
 *  overload (blasLapackWrapper.h:74-85). The reference delegates M==1 / N==1 to GEMV and K==1 to
 *  GER (:161-166); here every shape goes through the MFMA kernel family (results equal within
 *  rounding). C must not alias A or B. */
int xrs_gemm(xrs_handle_t handle, double* C, size_t M, size_t N, double alpha,
             const double* A, size_t lda, int transA, size_t K,
             const double* B, size_t ldb, int transB);

/** Extension (no reference counterpart): `count` independent same-shape GEMMs
 *  C[i] = alpha * op(A[i]) * op(B[i]) in one launch per 32 entries. A, B, C: host arrays of device
 *  pointers; shapes and flags as in xrs_gemm. Used for the independent per-core products of a TT round. */
int xrs_gemm_batched(xrs_handle_t handle, size_t count, double* const* C, size_t M, size_t N, double alpha,
                     const double* const* A, size_t lda, int transA, size_t K,
                     const double* const* B, size_t ldb, int transB);

/** Extension (no reference counterpart): C (N x N) = alpha * op(A) * op(B) for a product the caller
 *  knows to be symmetric (a Gram A^T A, or M^T G M with G symmetric). Only the tiles on or below the
 *  diagonal are computed; the result is written exactly symmetric. Flags and ld as in xrs_gemm (M = N). */
int xrs_gemm_sym(xrs_handle_t handle, double* C, size_t N, double alpha,
                 const double* A, size_t lda, int transA, size_t K,
                 const double* B, size_t ldb, int transB);

/** fp32 form of xrs_gemm on the fp32 matrix cores (v_mfma_f32_16x16x4_f32, 157.3 TF/s peak): C = alpha *
 *  op(A) * op(B), float operands and result, row-major, ldc = N; argument order, ld rules and aliasing as
 *  xrs_gemm. The reduced-precision variant of blasWrapper::matrix_matrix_product (blasLapackWrapper.cpp:
 *  149-195, whose cblas_dgemm :177-191 computes in value_t = double): relative error ~1e-7 * sum|a b| per
 *  element. Deterministic (fixed split-K slice order). No reference counterpart at this precision. */
int xrs_gemm_f32(xrs_handle_t handle, float* C, size_t M, size_t N, float alpha,
                 const float* A, size_t lda, int transA, size_t K,
                 const float* B, size_t ldb, int transB);

/* ---------------------------------------------------------------- permutation (tensor.h:65) */
/** out = reshuffle(in, shuffle): out[...] with mode i of `in` moved to position shuffle[i]
 *  (indexedTensor_tensor_evaluate.cpp:55-143; shuffle[i] = NEW position of OLD mode i, :80-82).
 *  Bit-exact. `dims` are the dims of `in`. out must not alias in. */
int xrs_permute(xrs_handle_t handle, double* out, const double* in, size_t ndim,
                const size_t* dims, const size_t* shuffle);

/* ---------------------------------------------------------------- factorisations (blasLapackWrapper.h:90-135) */
/** Rank-revealing A = Q*C for an m x n matrix (replaces blasWrapper::qc, blasLapackWrapper.cpp:235-305).
 *  Q: m x rank, orthonormal columns; C: rank x n. Rank rule of the reference (:268-272):
 *  the first k with |R_kk| < 16*DBL_EPSILON*R_00 of the column-pivoted QR (dgeqp3 sign convention).
 *  Q must hold m*min(m,n) doubles, C min(m,n)*n; on return they are packed with leading dims
 *  rank and n. *rank is written on the host. Synchronises. */
int xrs_qc(xrs_handle_t handle, double* Q, double* C, size_t* rank, const double* A, size_t m, size_t n);
/** A = C*Q, C: m x rank, Q: rank x n orthonormal rows (replaces blasWrapper::cq, :308-371;
 *  pivoting over the rows of A as the reference's col-major dgeqp3 on A^T). Synchronises. */
int xrs_cq(xrs_handle_t handle, double* C, double* Q, size_t* rank, const double* A, size_t m, size_t n);
/** Unpivoted A = Q*R, Q: m x min(m,n), R: min(m,n) x n (replaces blasWrapper::qr, :374-431). */
int xrs_qr(xrs_handle_t handle, double* Q, double* R, const double* A, size_t m, size_t n);
/** Unpivoted A = R*Q, R: m x min(m,n), Q: min(m,n) x n (replaces blasWrapper::rq, :445-498). */
int xrs_rq(xrs_handle_t handle, double* R, double* Q, const double* A, size_t m, size_t n);
/** Thin SVD A = U*diag(S)*Vt, U: m x k, S: k, Vt: k x n, k = min(m,n), S descending
 *  (replaces blasWrapper::svd / dgesdd 'S', blasLapackWrapper.cpp:201-232). */
int xrs_svd(xrs_handle_t handle, double* U, double* S, double* Vt, const double* A, size_t m, size_t n);
/** Solve A X = B, A m x n, B m x p, X n x p (replaces blasWrapper::solve, blasLapackWrapper.cpp:540-640):
 *  the reference's dispatch (m != n: least squares; not symmetric: general; symmetric with a positive
 *  diagonal: Cholesky, falling back to the general path). Cholesky is blocked (any n); the general and
 *  least-squares paths are the solve of xrs_solve_least_squares. Synchronises. */
int xrs_solve(xrs_handle_t handle, double* X, const double* A, size_t m, size_t n, const double* B, size_t p);
/** Minimum-norm least-squares solution of A X = B (replaces blasWrapper::solve_least_squares / dgelsd,
 *  blasLapackWrapper.cpp:647-721): X = V S^+ U^T B, singular values <= EPSILON * sigma_max dropped
 *  (min(m, n) <= 512); above, a shifted-CholeskyQR3 QR / LQ solve for full-rank A (rank-deficient A of
 *  that size: XRS_ENUMERIC). */
int xrs_solve_least_squares(xrs_handle_t handle, double* X, const double* A, size_t m, size_t n, const double* B, size_t p);
/** Singular values and right singular vectors of the rows of A (p x q, p <= q <= 1024; kernel 1: p <= 512) by one-sided
 *  Jacobi -- the SVD step of the truncating TT round (TTNetwork::round's per-edge svd,
 *  ttNetwork.cpp:644-665, without U). S: p descending; Vt: p x q, orthonormal rows for S > 0.
 *  kernel: 0 auto, 1 one workgroup, 2 multi-workgroup blocks (p > 16). *sweeps (host): Jacobi
 *  sweeps used, -1 not converged, -2 grid-barrier timeout. Synchronises. */
int xrs_svd_rows_vt(xrs_handle_t handle, double* S, double* Vt, int* sweeps, const double* A, size_t p, size_t q, int kernel);
/** Householder tridiagonalisation of a symmetric n x n matrix A (lower triangle read, 2 <= n <= 256) in one
 *  register-resident workgroup; d (n) and e (n - 1) of T = Q^T A Q. The first stage of the truncating round's eigensolver (dsytrd's role,
 *  tensor.cpp:1424-1489 via the certified edge Gram); exposed for its tests. Synchronises. */
int xrs_sym_tridiag(xrs_handle_t handle, double* d, double* e, const double* A, size_t n);
/** Eigenpairs of the kk largest eigenvalues of a symmetric n x n matrix A (lower triangle read, 2 <= n <= 256,
 *  1 <= kk <= n): the certified truncating round's replacement of the per-edge SVD when the edge Gram is
 *  certified well conditioned (no reference counterpart: the reference always runs dgesdd, tensor.cpp:1424-1489).
 *  Householder tridiagonalisation, multisection + inverse iteration, back-transformation. lam: kk descending;
 *  Ut: kk x n, row i = the eigenvector of lam[i]. *status (host): 0, or -1 when a multisection did not
 *  converge. Synchronises. */
int xrs_sym_eig_top(xrs_handle_t handle, double* lam, double* Ut, int* status, const double* A, size_t n, size_t kk);

/* ---------------------------------------------------------------- TT hot path (ttNetwork.cpp) */
/* A TT of order d is passed as d device core pointers; core k has dims (r[k], n[k], r[k+1]),
 * r[0] = r[d] = 1 (ttNetwork.cpp:57-108, 457-460). Functions that change ranks allocate NEW cores
 * from the handle's pool, write their pointers into `cores` and free the old ones with xrs_free
 * (the caller owns the result and releases it with xrs_free). */

/** Left-to-right / right-to-left orthogonalisation moving the core to `position`
 *  (TTNetwork::move_core, ttNetwork.cpp:582-628, transfer_core tensorNetwork.cpp:821-909).
 *  `canonicalized`/`core_position` describe the input state as in the reference (:588-607). */
int xrs_tt_move_core(xrs_handle_t handle, size_t d, const size_t* n, size_t* r, double** cores,
                     int canonicalized, size_t core_position, size_t position, int keep_rank);
/** TTNetwork::round(maxRanks, eps) (ttNetwork.cpp:644-665): canonicalise right, then truncate
 *  every edge right-to-left keeping at most max_ranks[k] singular values and cutting
 *  sigma_j <= eps*sigma_0 (tensor.cpp:1463-1474). On return the core is at position 0. */
int xrs_tt_round(xrs_handle_t handle, size_t d, const size_t* n, size_t* r, double** cores,
                 int canonicalized, size_t core_position, const size_t* max_ranks, double eps);
/** TTNetwork::soft_threshold (ttNetwork.cpp:688-713): left-to-right QC sweep (canonicalize_right), then
 *  right to left per edge the SVD with no rank cut beyond exact zeros (maxRank = inf, eps = 0) whose
 *  singular values become max(0, sigma - tau) (round_edge's _softThreshold, tensorNetwork.cpp:766,788).
 *  taus: d-1 thresholds, taus[0] for the LAST edge (the reference's loop order). Core ends at 0. */
int xrs_tt_soft_threshold(xrs_handle_t handle, size_t d, const size_t* n, size_t* r, double** cores,
                          int canonicalized, size_t core_position, const double* taus);
/** Entrywise (Hadamard) product of two TTs of equal mode sizes (entrywise_product, ttNetwork.cpp:1275-1309,
 *  core by core as perform_component_product, :1209-1272): out[k] = (ra[k] rb[k], ext[k], ra[k+1] rb[k+1])
 *  with out[k][(a,b), i, (a',b')] = A[k][a, i, a'] B[k][b, i, b'] (fused rank a major, b minor), alpha
 *  multiplied into out[0]. ext[k] = n_k for TTTensor cores, n_k m_k for TTOperator cores. Output cores come
 *  from the handle's pool (release with xrs_free); no canonicalisation (the reference then moves the core
 *  to A's core position when both inputs are canonical). */
int xrs_tt_entrywise_product(xrs_handle_t handle, size_t d, const size_t* ext, const size_t* ra, const double* const* A,
                             const size_t* rb, const double* const* B, double alpha, double** out);
/** TTOperator application, the core-wise contraction of a TTStack (ttStack.cpp:197-309, built by
 *  TTNetwork<true>::specialized_contraction_f, ttNetwork.cpp:886-967). Operator A: cores
 *  (ra[k], n[k], m[k], ra[k+1]). With p == NULL, B is a TTTensor with cores (rb[k], m[k], rb[k+1]) and
 *  out[k] = (ra[k] rb[k], n[k], ra[k+1] rb[k+1]) holds sum_j A[a,i,j,a'] B[b,j,b'] (y = A x); with
 *  transpose_a the row mode is contracted instead (x^T A: B cores (rb[k], n[k], rb[k+1]), out modes m[k]).
 *  With p != NULL, B is an operator with cores (rb[k], m[k], p[k], rb[k+1]) and out[k] is the operator
 *  core (ra rb, n, p, ra' rb') of A B. Fused ranks (a, b), the operator's index major. The output cores
 *  are allocated from the handle's pool (release with xrs_free). No canonicalisation: the reference
 *  then moves the core to the operator's core position (ttStack.cpp:163-166), xrs_tt_move_core. */
int xrs_tt_operator_apply(xrs_handle_t handle, size_t d, const size_t* n, const size_t* m, const size_t* p, const size_t* ra,
                          const double* const* A, const size_t* rb, const double* const* B, int transpose_a, double** out);
/** Which algorithm the handle's last xrs_tt_round used: XRS_ROUND_CHAIN (certified, no cut possible:
 *  Gram chains + batched factorisations), XRS_ROUND_TRUNCATE (certified truncation: left chain pass +
 *  device-resident right-to-left SVD sweep), XRS_ROUND_GENERAL (any spectrum and eps: shifted
 *  CholeskyQR3 sweep + Jacobi SVDs with device-side rank cuts, one synchronisation), XRS_ROUND_REFERENCE (the reference's sequential
 *  QC + round_edge sweeps); 0 before the first round. Diagnostics for tests and benchmarks. */
#define XRS_ROUND_CHAIN 1
#define XRS_ROUND_TRUNCATE 2
#define XRS_ROUND_REFERENCE 3
#define XRS_ROUND_GENERAL 4
int xrs_tt_last_round_path(xrs_handle_t handle);
/** <x,y> of two TTs with equal mode sizes (value_t(x(i&0)*y(i&0)), ttNetwork.cpp:782-789 path,
 *  SURVEY §3.4) as a left-to-right zipper without permutations. *result on host. Synchronises. */
int xrs_tt_dot(xrs_handle_t handle, double* result, size_t d, const size_t* n,
               const size_t* rx, const double* const* xcores,
               const size_t* ry, const double* const* ycores);

/** Asynchronous <x,y> (same algorithm and result as xrs_tt_dot): enqueued on the handle's side streams
 *  1 and 2 from the main stream's current point, NOT joined into the main stream, so work enqueued next
 *  (e.g. xrs_tt_round of x) runs beside it. Until xrs_tt_dot_wait, the cores may be read and released
 *  (releases through this handle -- xrs_free, a round replacing cores -- wait for the inner product
 *  first) but not written in place. One in flight per handle. No counterpart in the reference (whose
 *  value_t(x(i&0)*y(i&0)) is synchronous); xrs_tt_dot_wait returns what xrs_tt_dot would have. */
int xrs_tt_dot_async(xrs_handle_t handle, size_t d, const size_t* n,
                     const size_t* rx, const double* const* xcores,
                     const size_t* ry, const double* const* ycores);
/** Waits for the handle's asynchronous inner product; *result on host. */
int xrs_tt_dot_wait(xrs_handle_t handle, double* result);
/** <x,y> on fp32 MFMA tiles (v_mfma_f32_16x16x4_f32): the two-ended zipper of xrs_tt_dot with the fp64
 *  cores rounded to fp32 as they are loaded, fp32 environments renormalised by powers of two every step,
 *  the closing sum in fp64. A reduced-precision side path (|error| ~1e-7 ||x|| ||y||), NOT a replacement
 *  for value_t(x(i&0)*y(i&0)) (ttNetwork.cpp:782-789), which xrs_tt_dot restates in fp64. d >= 2.
 *  *result on host. Synchronises. */
int xrs_tt_dot_f32(xrs_handle_t handle, double* result, size_t d, const size_t* n,
                   const size_t* rx, const double* const* xcores,
                   const size_t* ry, const double* const* ycores);

/** All-reduce (element-wise sum over all ranks) of `count` doubles at the device pointer `buf`, in place.
 *  Called by the sharded TT entry points with the handle's stream synchronised; returns 0 on success.
 *  The Python layer (xerus_amd.dist) binds it to torch.distributed (RCCL over xGMI on MI355X).
 *  A NULL hook means one rank: the local sums are final and no synchronisation happens. */
typedef int (*xrs_allreduce_fn)(void* ctx, double* buf, size_t count);
/** All-gather: every rank contributes `count` doubles at `send`; `recv` (world * count doubles, device)
 *  receives them in rank order. Same calling convention as xrs_allreduce_fn. */
typedef int (*xrs_allgather_fn)(void* ctx, const double* send, double* recv, size_t count);

/** RCCL communicator (no reference counterpart: xerus is single-process). xrs_comm_allreduce is an
 *  xrs_allreduce_fn taking an xrs_comm_t as ctx: it enqueues an in-place fp64 sum ncclAllReduce on the
 *  handle's stream and returns at once; the sharded TT drivers recognise it and skip the host stream
 *  synchronisation other hooks need (no host round trip per collective). One rank calls
 *  xrs_comm_unique_id (128 bytes), the caller distributes the id, every rank calls xrs_comm_create.
 *  RCCL is loaded at run time; the calls fail with a status if it is absent. */
typedef struct xrs_comm_s* xrs_comm_t;
int xrs_comm_unique_id(void* id128_out);
int xrs_comm_create(xrs_handle_t handle, int nranks, int rank, const void* id128, xrs_comm_t* comm_out);
int xrs_comm_destroy(xrs_comm_t comm);
size_t xrs_comm_calls(xrs_comm_t comm);
int xrs_comm_allreduce(void* comm, double* buf, size_t count);
/** Emulated communicator for per-rank timing on one GPU (no RCCL): rank 0 of `nranks` ranks that hold
 *  IDENTICAL mode slices, i.e. the sharding of the TT whose every mode is the local one repeated nranks
 *  times. xrs_comm_allreduce on it enqueues buf *= nranks (exactly that TT's sum over ranks) on the handle's
 *  stream; all-gather is refused. A diagnostic: the sharded round then runs a real rank's kernels, with
 *  collectives of zero cost (tools/cfg5_rank_probe.py). Limitation: a core gathered through
 *  it (a zero-padded block all-reduced) would be nranks x rank 0's block, not the TT's core, so the steps
 *  that gather -- tall right edges, left structural-excess QC -- treat the layout as unknown and the round
 *  reports uncertified (path 0) instead. */
int xrs_comm_emulate(xrs_handle_t handle, int nranks, xrs_comm_t* comm_out);
/** xrs_allgather_fn of the communicator: ncclAllGather (fp64) enqueued on the handle's stream. */
int xrs_comm_allgather(void* comm, const double* send, double* recv, size_t count);

/** Full cores of a mode-sharded TT on every rank (the fallback of a sharded round whose certificate
 *  fails): the ranks' slices (mode blocks of xerus_amd.dist.mode_partition) of all components go out in
 *  ONE all-gather of padded blocks and are scattered into new cores (r[k], n_global[k], r[k+1]) from the
 *  handle's pool (release with xrs_free). Device to device; synchronises. */
int xrs_tt_gather_sharded(xrs_handle_t handle, size_t d, const size_t* n_global, int world, int rank, const size_t* r,
                          const double* const* local_cores, double** full_cores_out, xrs_allgather_fn allgather, void* ctx);
/** This rank's mode slices of full cores into new pool buffers (local_out[k]: (r[k], m_k, r[k+1])). */
int xrs_tt_shard(xrs_handle_t handle, size_t d, const size_t* n_global, int world, int rank, const size_t* r,
                 const double* const* full_cores, double** local_out);

/** Mode-sharded TT round (no reference counterpart: xerus is single-process).
 *  Each rank holds, for every component k, the mode slices of its own subset (n_local[k] of them) as
 *  an (r_k, n_local[k], r_{k+1}) row-major device array. The Gram chains are sums over the mode index,
 *  completed by one all-reduce per chain step (both chains' r x r Grams together) and one for all
 *  orthogonality Grams: d + 0 all-reduces per pass; the per-core transforms are local.
 *  *certified = 1: rounded in place (right-canonical, core at 0, ranks unchanged: no cut possible);
 *  *certified = 0: certificate failed, cores untouched (gather and use xrs_tt_round). */
int xrs_tt_round_sharded(xrs_handle_t handle, size_t d, const size_t* n_local, size_t* r, double** cores,
                         const size_t* max_ranks, double eps, xrs_allreduce_fn allreduce, void* ctx, int* certified);

/** Mode-sharded TT round for every input: the ranks' layout is given (world ranks, this one is
 *  `rank`; every rank holds a contiguous block of each mode, blocks in rank order -- the layout of
 *  xerus_amd.dist.mode_partition or any other), so besides the chain round and the certified truncation
 *  (xrs_tt_round_sharded) it also runs the sharded general round (any spectrum and eps: shifted
 *  CholeskyQR3 + Jacobi SVDs with device-side rank cuts, ttNetwork.cpp:644-665 semantics). Cores whose
 *  unfolding spans the ranks' blocks -- tall right edges (r_k > n_k r_{k+1}, e.g. after x + y) and the
 *  structural-excess QC steps at the left end -- are gathered by one all-reduce of a zero-padded core
 *  (small: bounded by r^2) and factorised replicated. *path = XRS_ROUND_CHAIN / _TRUNCATE / _GENERAL on
 *  success, 0 if every certificate failed (then the left-end QC steps may have been applied: the cores
 *  represent the same tensor; gather and use xrs_tt_round). world * d <= 2040. */
int xrs_tt_round_sharded_ex(xrs_handle_t handle, size_t d, const size_t* n_local, size_t* r, double** cores,
                            const size_t* max_ranks, double eps, int world, int rank, xrs_allreduce_fn allreduce,
                            void* ctx, int* path);

/** <x,y> of two TTs mode-sharded identically (two-ended zipper: one all-reduce per step for both
 *  environments, ceil(d/2) in all for d >= 4; one per component below). */
int xrs_tt_dot_sharded(xrs_handle_t handle, double* result, size_t d, const size_t* n_local, const size_t* rx,
                       const double* const* X, const size_t* ry, const double* const* Y, xrs_allreduce_fn allreduce,
                       void* ctx);

/* ---------------------------------------------------------------- profiling */
/** Kernel-duration instrumentation: while enabled, every launch of a kernel whose family id is in
 *  `family_mask` is bracketed by HIP events on the handle's stream. */
#define XRS_KFAM_GEMM 1u
#define XRS_KFAM_PERMUTE 2u
#define XRS_KFAM_QR 4u
#define XRS_KFAM_SVD 8u
#define XRS_KFAM_ELEMWISE 16u
#define XRS_KFAM_SPLITK 32u   /* the fp64 GEMMs' separate split-K reduce launches (k_splitk_reduce*) */
int xrs_prof_begin(xrs_handle_t handle, uint32_t family_mask);
/** Stops instrumentation, synchronises and returns (launches, total kernel milliseconds,
 *  algorithmic flops, algorithmic bytes) of the instrumented launches. */
int xrs_prof_end(xrs_handle_t handle, size_t* launches, double* total_ms, double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif /* XERUS_AMD_H */
