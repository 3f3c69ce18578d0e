// fp32 GEMM on the CDNA4 fp32 matrix cores (sgemm.hip): the reduced-precision contraction path.
#pragma once
#include <cstddef>

#include "runtime.hpp"

namespace xrs {

// Optional per-launch extras of sgemm. A "max word" is kMaxLanes device words (float bits of non-negative
// values) whose maximum is the value: producers atomicMax into lane (workgroup id % kMaxLanes), so no single
// word takes more than a few arrivals per launch.
//   sa / sb : max words of operand A / B; the operand is multiplied by the power of two 2^-e that brings the
//             max into [0.5, 1) as it is staged (exact);
//   amax    : max word that receives max|C| (one atomicMax per workgroup; the caller zeroes it first);
//   cmax_a / cmax_b : kCmaxSlots device words (zeroed by the caller) that receive max|A| / max|B| of an fp64
//             operand as read, one slot per workgroup (blockIdx modulo kCmaxSlots); the fp32 zipper checks
//             every core's max against its safe range after the run (dot32.hip).
constexpr int kMaxLanes = 16;
constexpr int kCmaxSlots = 1024;
struct SgemmExtra {
    const unsigned* sa = nullptr;
    const unsigned* sb = nullptr;
    unsigned* amax = nullptr;
    unsigned* cmax_a = nullptr;
    unsigned* cmax_b = nullptr;
};

// C (M x N, row-major, ldc = N, fp32) = alpha op(A) op(B) on v_mfma_f32_16x16x4_f32. op(A) = A^T when ta
// (A stored K x M), op(B) = B^T when tb (B stored N x K). EA / EB: float or double (fp64 operands are
// rounded to fp32 as they are staged into LDS). Deterministic: fixed split-K slice order.
template <class EA, class EB>
void sgemm(xrs_handle_t h, float* C, size_t M, size_t N, float alpha, const EA* A, size_t lda, bool ta, size_t K,
           const EB* B, size_t ldb, bool tb, const SgemmExtra& x = SgemmExtra{});

// power-of-two exponent e of a max value's float bits (max|.| * 2^-e in [0.5, 1)); 0 for a zero max
inline int pow2_exponent(unsigned bits) { return bits == 0u ? 0 : int((bits >> 23) & 0xff) - 126; }
// the value of a max word (kMaxLanes lanes) read back to the host
inline unsigned max_word_bits(const unsigned* lanes) {
    unsigned m = 0u;
    for (int i = 0; i < kMaxLanes; ++i) m = lanes[i] > m ? lanes[i] : m;
    return m;
}

}  // namespace xrs
