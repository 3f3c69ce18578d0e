// TTOperator application: the core-wise contraction of a TTStack (ttStack.cpp:197-309; the stack is
// built by TTNetwork<true>::specialized_contraction_f, ttNetwork.cpp:886-967).
//
//   operator x vector:   C[(a,b), i, (a',b')]    = sum_j A[a, i, j, a'] X[b, j, b']
//   operator x operator: C[(a,b), i, k, (a',b')] = sum_j A[a, i, j, a'] B[b, j, k, b']
//   transposed (x^T A):  C[(a,b), j, (a',b')]    = sum_i A[a, i, j, a'] X[b, i, b']   (x(i&0) * A(i/2, j/2))
//
// The fused rank index is (a, b), the operator's rank major: the order in which the stack's nodes are
// contracted (the operator's node first) and then reshuffled (ttStack.cpp:216-228, 241-296).
// One pass writes every output element exactly once (8 B per element, the HBM bound); the operands'
// cores are small and stay cache-resident. The contraction index is short (the mode size), so this is
// streaming work, not a GEMM.
#include "runtime.hpp"
#include "tt_common.hpp"

namespace xrs {
namespace {

struct OpCoreArgs {
    const double* A;
    const double* B;
    double* C;
    int ra, ra2, rb, rb2;    // ranks of A's and B's cores (left, right)
    int n, m, p;             // output mode (A's row or column mode), contracted mode, B's second mode (1: vector)
    int trans;               // 0: contract A's column mode with B; 1: contract A's row mode (x^T A)
    int na, ma;              // A's mode sizes (rows, columns)
};

// one thread per output element, the right fused rank index (a', b') fastest: coalesced stores and
// coalesced reads of B along b'
__global__ void __launch_bounds__(256) k_op_core(const OpCoreArgs g, size_t total) {
    const size_t idx = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (idx >= total) return;
    size_t t = idx;
    const int b2 = int(t % g.rb2); t /= g.rb2;
    const int a2 = int(t % g.ra2); t /= g.ra2;
    const int k = int(t % g.p);    t /= g.p;
    const int i = int(t % g.n);    t /= g.n;
    const int b = int(t % g.rb);   t /= g.rb;
    const int a = int(t);
    // A[a, r, c, a'] with (r, c) = (i, j) or (j, i)
    const size_t a_row = size_t(a) * g.na;
    double acc = 0.0;
    for (int j = 0; j < g.m; ++j) {
        const int r = g.trans ? j : i, c = g.trans ? i : j;
        const double av = g.A[((a_row + r) * g.ma + c) * g.ra2 + a2];
        const double bv = g.B[((size_t(b) * g.m + j) * g.p + k) * g.rb2 + b2];
        acc = fma(av, bv, acc);
    }
    g.C[idx] = acc;
}

// entrywise (Hadamard) product core: C[(a,b), i, (a',b')] = alpha A[a, i, a'] B[b, i, b'] with i over the
// external modes of the core (n, or n m for an operator core); one thread per output element, (a', b')
// fastest (coalesced stores and reads of B), HBM-bound on the 8 B written per element
__global__ void __launch_bounds__(256) k_entrywise_core(const double* __restrict__ A, const double* __restrict__ B,
                                                        double* __restrict__ C, int ra, int ra2, int rb, int rb2, int ext,
                                                        double alpha, size_t total) {
    const size_t idx = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (idx >= total) return;
    size_t t = idx;
    const int b2 = int(t % rb2); t /= rb2;
    const int a2 = int(t % ra2); t /= ra2;
    const int i = int(t % ext);  t /= ext;
    const int b = int(t % rb);   t /= rb;
    const int a = int(t);
    C[idx] = alpha * A[(size_t(a) * ext + i) * ra2 + a2] * B[(size_t(b) * ext + i) * rb2 + b2];
}

}  // namespace
}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_tt_entrywise_product(xrs_handle_t h, size_t d, const size_t* ext, const size_t* ra, const double* const* A,
                             const size_t* rb, const double* const* B, double alpha, double** out) {
    return guarded([&] {
        XRS_REQUIRE(h && ext && ra && rb && A && B && out, "null argument");
        XRS_REQUIRE(d >= 1, "TT must have at least one component");
        XRS_REQUIRE(ra[0] == 1 && ra[d] == 1 && rb[0] == 1 && rb[d] == 1, "boundary ranks must be 1");
        for (size_t k = 0; k < d; ++k) {
            XRS_REQUIRE(ext[k] > 0 && ra[k + 1] > 0 && rb[k + 1] > 0, "dimensions and ranks must be positive");
            XRS_REQUIRE(A[k] && B[k], "null core");
            XRS_REQUIRE(ra[k] * rb[k] < (1u << 31) && ra[k + 1] * rb[k + 1] < (1u << 31) && ext[k] < (1u << 31),
                        "product rank or mode too large");
        }
        std::vector<double*> made(d, nullptr);
        try {
            for (size_t k = 0; k < d; ++k) {
                const size_t total = ra[k] * rb[k] * ext[k] * ra[k + 1] * rb[k + 1];
                made[k] = static_cast<double*>(h->pool->alloc(total * 8));
                KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(total), 8.0 * double(total));
                hipLaunchKernelGGL(k_entrywise_core, dim3(unsigned((total + 255) / 256)), dim3(256), 0, h->stream, A[k], B[k], made[k],
                                   int(ra[k]), int(ra[k + 1]), int(rb[k]), int(rb[k + 1]), int(ext[k]), k == 0 ? alpha : 1.0, total);
                check_launch("k_entrywise_core");
            }
        } catch (...) {
            for (double* q : made)
                if (q) h->pool->release(q);
            throw;
        }
        for (size_t k = 0; k < d; ++k) out[k] = made[k];
    });
}

int xrs_tt_operator_apply(xrs_handle_t h, size_t d, const size_t* n, const size_t* m, const size_t* p, const size_t* ra,
                          const double* const* A, const size_t* rb, const double* const* B, int transpose_a, double** out) {
    return guarded([&] {
        XRS_REQUIRE(h && n && m && ra && rb && A && B && out, "null argument");
        XRS_REQUIRE(d >= 1, "TT must have at least one component");
        XRS_REQUIRE(ra[0] == 1 && ra[d] == 1 && rb[0] == 1 && rb[d] == 1, "boundary ranks must be 1");
        XRS_REQUIRE(!(transpose_a && p), "the transposed application takes a TTTensor");
        for (size_t k = 0; k < d; ++k) {
            XRS_REQUIRE(n[k] > 0 && m[k] > 0 && ra[k + 1] > 0 && rb[k + 1] > 0 && (!p || p[k] > 0), "dimensions and ranks must be positive");
            XRS_REQUIRE(A[k] && B[k], "null core");
        }
        std::vector<double*> made(d, nullptr);
        try {
            for (size_t k = 0; k < d; ++k) {
                OpCoreArgs g{};
                g.A = A[k];
                g.B = B[k];
                g.ra = int(ra[k]);
                g.ra2 = int(ra[k + 1]);
                g.rb = int(rb[k]);
                g.rb2 = int(rb[k + 1]);
                g.na = int(n[k]);
                g.ma = int(m[k]);
                g.trans = transpose_a;
                g.n = transpose_a ? int(m[k]) : int(n[k]);   // the free mode of A
                g.m = transpose_a ? int(n[k]) : int(m[k]);   // the contracted one
                g.p = p ? int(p[k]) : 1;
                const size_t total = size_t(g.ra) * g.rb * g.n * g.p * size_t(g.ra2) * g.rb2;
                made[k] = static_cast<double*>(h->pool->alloc(total * 8));
                g.C = made[k];
                KernelTimer timer(h, XRS_KFAM_ELEMWISE, 2.0 * double(total) * g.m, 8.0 * double(total));
                hipLaunchKernelGGL(k_op_core, dim3(unsigned((total + 255) / 256)), dim3(256), 0, h->stream, g, total);
                check_launch("k_op_core");
            }
        } catch (...) {
            for (double* q : made)
                if (q) h->pool->release(q);
            throw;
        }
        for (size_t k = 0; k < d; ++k) out[k] = made[k];
    });
}

}  // extern "C"
