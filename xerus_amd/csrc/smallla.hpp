// Launch wrappers of the small dense kernels (smallla.hip) and the factorisation drivers (linalg.cpp).
#pragma once
#include <functional>
#include <vector>

#include "elementwise.hpp"

namespace xrs {

constexpr int kSmallMax = 512;  // largest n handled by the single-workgroup kernels

// G (n x n) := L with G + shift_rel*trace(G)*I = L L^T (lower, upper zeroed); Dinv: n x 32 inverses of the
// diagonal blocks. *status_dev = 0 on success, else 1 + first failing column; info_dev[0] = trace(G)
// (may be null). Enqueued only.
void potrf(xrs_handle_t h, double* G, int n, double shift_rel, double* Dinv, int* status_dev, double* info_dev = nullptr);
// Batch of independent Cholesky factorisations (n <= 256 each), one workgroup per matrix, each with its
// own relative diagonal shift; status[i] as for potrf. Dinv[i] needs ceil(n_i/16)*256 doubles.
constexpr int kPotrfBatchMax = 48;
struct PotrfBatch {
    // entry i factors src[i] (nullptr: G[i] in place) into G[i]; G[i] == nullptr (n <= 256 only): the
    // factor is not stored (certificates: only the status is wanted)
    const double* src[kPotrfBatchMax];
    double* G[kPotrfBatchMax];
    double* Dinv[kPotrfBatchMax];
    double shift[kPotrfBatchMax];
    int n[kPotrfBatchMax];
    int slot[kPotrfBatchMax];   // entry i writes status[slot[i]] (set by potrf_batched; callers leave it)
    int* status;
};
void potrf_batched(xrs_handle_t h, const PotrfBatch& b, int count);
// doubles needed for the Dinv output of potrf / potrf_batched for an n x n matrix
size_t dinv_elems(int n);
// Batch of explicit inverses X_i = L_i^{-1} of lower-triangular factors from potrf / potrf_batched
// (Dinv_i their diagonal-block inverses); X_i is n_i x n_i, upper triangle zero. One launch per Dinv layout.
constexpr int kTrinvBatchMax = 64;
struct TrinvBatch {
    const double* L[kTrinvBatchMax];
    const double* Dinv[kTrinvBatchMax];
    double* X[kTrinvBatchMax];
    int n[kTrinvBatchMax];
};
void trinv_batched(xrs_handle_t h, const TrinvBatch& b, int count);
// X = L^{-1} Y. cols=false: the RHS vectors are the nvec rows of Y (ld ldy); cols=true: the nvec columns.
void trsm(xrs_handle_t h, bool cols, const double* L, const double* Dinv, int n, const double* Y, size_t ldy, double* X,
          size_t ldx, int nvec);
// Exact dgeqp3/dgeqrf + dorgqr emulation on A (m x n row-major). pivot=false -> unpivoted Householder QR.
// abs_r00: use |R_00| in the rank rule (when the caller already knows the reference's R_00 is positive).
// Q: m x min(m,n) (ld min(m,n)), C: rank x n (C rows beyond rank untouched). Returns the rank (synchronises).
size_t qrcp(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* C, bool pivot, bool abs_r00,
            bool rank_rule);
// One-sided Jacobi SVD of the rows of W (p x q, p <= q): U (p x p), S (p), Vt (p x q), S descending.
void jacobi_svd_rows(xrs_handle_t h, const double* W, int p, int q, double* U, double* S, double* Vt);

// Right singular vectors of W (p x q, p <= min(q, 512); W[i][k] at W[i*ldw + k], or W[k*ldw + i] with
// trans) by one-sided Jacobi on its rows (svd.hip): S (p) descending, Vt (p x q, row stride ldvt)
// orthonormal rows, W = U S Vt with U S = W Vt^T. *status_dev = sweeps used, -1 if not converged in
// max_sweeps, -2 if the block kernel's grid barrier timed out. kernel: 0 auto (p >= 32: the
// multi-workgroup block kernel, else one workgroup with W in LDS when p (q + 1) <= 18432 doubles),
// 1 one workgroup, 2 blocks. stamps (block kernel, diagnostics): status_dev[4..8] receive thread 0's
// cycles per cross-round phase (dot, rotation, update, barrier) and its rotation count -- status_dev
// must then hold 9 ints. Enqueued only.
void jacobi_vt(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* S, double* Vt, int ldvt,
               int* status_dev, int max_sweeps = 40, int kernel = 0, bool stamps = false, bool early = false);
bool jacobi_vt_fits_lds(int p, int q);
// Full SVD of the rows of W (p x q, p <= q, 32 ceil(q/32) + p <= 1024) by the block Jacobi kernel with
// the rotations accumulated (svd.hip): W = U diag(S) Vt, U p x p orthogonal (row stride ldu), S
// descending, Vt p x q (orthonormal rows for S > 0). Status as jacobi_vt. Enqueued only.
// Eigenpairs of the kk largest eigenvalues of a symmetric n x n matrix A (lower triangle read, 2 <= n <= 256):
// Householder tridiagonalisation (one workgroup, register-resident), multisection + inverse iteration per
// eigenvalue, back-transformation (syev.hip). lam (kk, optional) descending, S = sqrt(max(lam, 0))
// (optional), Ut rows = the eigenvectors (kk x n, row stride ldu). *status_dev set to -1 if a
// multisection did not converge (left untouched otherwise). Enqueued only.
bool sym_eig_top_fits(int n, int kk);   // the truncating round's policy (n <= 256 unless XRS_SYEV_MAX lowers it)
void sym_eig_top(xrs_handle_t h, const double* A, int lda, int n, int kk, double* lam, double* S, double* Ut, int ldu, int* status_dev);
// Householder tridiagonalisation (syev.hip's k_sytrd): d (n), e (n - 1) of T = Q^T A Q
void sym_tridiag(xrs_handle_t h, const double* A, int lda, int n, double* d, double* e);
// Square SVD (2 <= n <= 128) through the bidiagonal and its Golub-Kahan tridiagonal (syev.hip), certified a
// posteriori (residual and orthogonality <= 6e-15): false -> the outputs are invalid, recompute. diag
// (optional, 4): relative residual, max |U^T U - I|, max |Vt Vt^T - I|, multisection status. Synchronises.
// svd_bidiag_mode: XRS_SVD_BIDIAG (0 off, 1 on with the Jacobi fallback (default), 2 strict: failure throws).
int svd_bidiag_mode();
bool svd_bidiag(xrs_handle_t h, const double* A, int n, double* U, double* S, double* Vt, double* diag = nullptr);
bool jacobi_usv_fits(int p, int q);
void jacobi_usv(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* U, int ldu, double* S, double* Vt, int ldvt,
                int* status_dev, int max_sweeps = 40, bool early = false);
// Right singular vectors (rows of Vt, g x g) and S of a triangular g x g factor F: lower (L of B = L Q) by
// accumulated rotations on the rows of F^T, upper (R of B = Q R) on the rows of F. Enqueued only.
// early: the block kernel's early stop (svd.hip kEarlyCos2: no confirming sweep after one whose rotations
// were all below |cos| 1e-7) -- the truncation sweeps (tt_trunc.hip round_general)
void jacobi_right_vectors(xrs_handle_t h, const double* F, int g, bool lower, double* S, double* Vt, int* status_dev,
                          int max_sweeps = 40, bool early = false);

// Reads a Jacobi status word (synchronises) and returns it. -2 (a grid-barrier poll of the block kernel timed
// out) means the outputs are invalid, not a convergence failure: rerun(kernel) recomputes them (kernel 1 = one
// workgroup where p <= 512, else the block kernel once more); a second -2 throws. Other negative statuses are
// non-convergence warnings, as the reference's dgesdd failure (blasLapackWrapper.cpp:216-224).
int jacobi_settle(xrs_handle_t h, int* status_dev, int p, int q, const std::function<void(int kernel)>& rerun);

struct OrthResult {
    bool certified;   // sigma_min(A) >= cert_ratio * ||A||_F proven (Cholesky of the shifted Gram succeeded)
    double cert_ratio;
    bool robust;      // the shifted CholeskyQR3 / Householder path was needed
};

// Tall A (m x n, m >= n): A = Q R, Q m x n orthonormal columns, R n x n upper triangular.
// Wide B (m x n, m <= n) with wide=true: B = L Q, L m x m lower, Q m x n orthonormal rows.
OrthResult orthogonalize(xrs_handle_t h, const double* A, size_t m, size_t n, bool wide, double* Q, double* RL);

// Reference-semantics factorisations (blasLapackWrapper.cpp:235-498); device buffers as in xerus_amd.h.
size_t qc(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* C);
size_t cq(xrs_handle_t h, const double* A, size_t m, size_t n, double* C, double* Q);
void qr(xrs_handle_t h, const double* A, size_t m, size_t n, double* Q, double* R);
void rq(xrs_handle_t h, const double* A, size_t m, size_t n, double* R, double* Q);
void svd(xrs_handle_t h, const double* A, size_t m, size_t n, double* U, double* S, double* Vt);

// dense solves (solve.hip): blasWrapper::solve / solve_least_squares semantics; chol_blocked / chol_solve:
// SPD factorisation of any size (L lower, Z the diagonal-block inverses) and the two triangular sweeps
void solve_dense(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p);
void svd_solve(xrs_handle_t h, double* X, const double* A, size_t m, size_t n, const double* B, size_t p);
bool chol_blocked(xrs_handle_t h, const double* A, size_t n, double* L, std::vector<DevBuf>& Z);
void chol_solve(xrs_handle_t h, const double* L, const std::vector<DevBuf>& Z, size_t n, const double* B, size_t p, double* X);
// Cholesky of A + shift_rel tr(A) I for any n, enqueued only: status[0 .. chol_full_blocks(n)) (all zero on
// success), optional L (lower) and Z = L^{-1} (n x n each)
int chol_full_blocks(size_t n);
void chol_full(xrs_handle_t h, const double* A, size_t n, double shift_rel, double* L, double* Z, int* status);

// helpers
void transpose(xrs_handle_t h, double* out, const double* in, size_t rows, size_t cols);
int read_status(xrs_handle_t h, const int* status_dev, int count, int* host_out);

}  // namespace xrs
