// fp32 x fp32 instantiation of the fp32-MFMA GEMM (sgemm_impl.hpp) and its C-ABI entry xrs_gemm_f32.
#include "sgemm_impl.hpp"

namespace xrs {
template void sgemm<float, float>(xrs_handle_t, float*, size_t, size_t, float, const float*, size_t, bool, size_t,
                                  const float*, size_t, bool, const SgemmExtra&);
}  // namespace xrs

extern "C" int xrs_gemm_f32(xrs_handle_t h, float* C, size_t M, size_t N, float alpha, const float* A, size_t lda,
                            int transA, size_t K, const float* B, size_t ldb, int transB) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(M == 0 || N == 0 || C, "null C");
        XRS_REQUIRE(K == 0 || M == 0 || N == 0 || (A && B), "null A/B");
        XRS_REQUIRE(transA ? lda >= M || K == 0 : lda >= K || M == 0, "lda too small");
        XRS_REQUIRE(transB ? ldb >= K || N == 0 : ldb >= N || K == 0, "ldb too small");
        XRS_REQUIRE(static_cast<const void*>(C) != static_cast<const void*>(A) &&
                        static_cast<const void*>(C) != static_cast<const void*>(B),
                    "C must not alias A or B");
        xrs::fence_readers(h);
        xrs::sgemm<float, float>(h, C, M, N, alpha, A, lda, transA != 0, K, B, ldb, transB != 0);
    });
}

#ifdef XRS_SG_STAMPS
extern "C" int xrs_debug_sg_stamps(void* buf) {
    unsigned long long* q = static_cast<unsigned long long*>(buf);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sg_stamps), &q, sizeof(q)) == hipSuccess ? 0 : 1;
}
#endif
