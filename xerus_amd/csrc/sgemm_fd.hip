// float x double instantiation of the fp32-MFMA GEMM (sgemm_impl.hpp): fp64 operands are rounded to fp32 as they are
// staged (the fp32 TT zipper, dot32.hip, reads the fp64 cores in place).
#include "sgemm_impl.hpp"

namespace xrs {
template void sgemm<float, double>(xrs_handle_t, float*, size_t, size_t, float, const float*, size_t, bool, size_t,
                                   const double*, size_t, bool, const SgemmExtra&);
}  // namespace xrs
