// Internal entry points shared between the kernel translation units and the TT drivers.
#pragma once
#include <algorithm>

#include "runtime.hpp"

namespace xrs {

// level 1 / elementwise (elementwise.hip)
// partial: >= 1024 doubles of device scratch for the block sums (null: the handle's dev_scratch)
void reduce_to_device(xrs_handle_t h, int mode, const double* x, const double* y, size_t n, double* out_dev,
                      double* partial = nullptr);
double reduce_to_host(xrs_handle_t h, int mode, const double* x, const double* y, size_t n);
void scal(xrs_handle_t h, double* x, double alpha, size_t n);
void axpy(xrs_handle_t h, double* y, double alpha, const double* x, size_t n);
void scale_rows(xrs_handle_t h, double* X, const double* s, size_t m, size_t n);
void scale_cols(xrs_handle_t h, double* X, const double* s, size_t m, size_t n);
void diag_sum(xrs_handle_t h, double* out, const double* X, size_t P, size_t m);
void offset_add(xrs_handle_t h, double* out, const size_t* out_dims, const double* in, const size_t* in_dims, size_t nd,
                const size_t* offsets, double alpha);
void strided_eval(xrs_handle_t h, double* out, const double* in, size_t nd, const size_t* out_dims, const size_t* in_strides,
                  size_t nt, const size_t* tr_dims, const size_t* tr_strides, size_t base);

// gemm.hip
// tri: operands known triangular with EXACT zeros outside the triangle, whose zero K-blocks are skipped:
// bit 0 = op(A) lower (A[m][k] = 0 for k > m), bit 1 = op(B) lower (B[k][n] = 0 for k < n)
constexpr int kTriA = 1, kTriB = 2;
void gemm(xrs_handle_t h, double* C, size_t M, size_t N, double alpha, const double* A, size_t lda, bool ta, size_t K,
          const double* B, size_t ldb, bool tb, int tri = 0);
// Batch of same-shape GEMMs C[i] = alpha op(A[i]) op(B[i]) in one launch per kGemmBatchMax entries
constexpr int kGemmBatchMax = 32;
void gemm_batched(xrs_handle_t h, int count, double* const* C, size_t M, size_t N, double alpha, const double* const* A,
                  size_t lda, bool ta, size_t K, const double* const* B, size_t ldb, bool tb, bool sym = false,
                  int tri = 0);
// C (N x N) = alpha op(A) op(B) for a product KNOWN to be symmetric (Grams, M^T G M with G symmetric):
// only the lower tiles are computed and mirrored, so C is exactly symmetric
void gemm_sym(xrs_handle_t h, double* C, size_t N, double alpha, const double* A, size_t lda, bool ta, size_t K,
              const double* B, size_t ldb, bool tb);

// One GEMM C = op(A) op(B) (alpha 1) as a value (planned ahead of its launch).
struct GemmSpec {
    const double* A;
    const double* B;
    double* C;
    size_t M, N, K, lda, ldb;
    bool ta, tb;
};
inline void gemm(xrs_handle_t h, const GemmSpec& g) {
    gemm(h, g.C, g.M, g.N, 1.0, g.A, g.lda, g.ta, g.K, g.B, g.ldb, g.tb);
}

// permute.hip
void permute(xrs_handle_t h, double* out, const double* in, size_t ndim, const size_t* dims, const size_t* shuffle);

}  // namespace xrs
