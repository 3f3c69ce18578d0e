// C++-level entry points of the TT drivers (tt.hip) for the xerus host API. Cores are device buffers of
// the handle's pool; functions that change ranks release the old cores and allocate new ones.
#pragma once
#include "runtime.hpp"

namespace xrs {
namespace tt {
void move_core(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
               size_t pos, bool keep_rank);
void round(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
           const size_t* max_ranks, double eps);
double dot(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y);
void soft_threshold(xrs_handle_t h, size_t d, const size_t* n, size_t* r, double** cores, bool canonicalized, size_t core_pos,
                    const double* taus);
}  // namespace tt
namespace zip {   // zip32.hip: the fused fp32 zipper (xrs_tt_dot_f32's main path)
bool applicable(size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                const double* const* Y);
double dot(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y);
}  // namespace zip
}  // namespace xrs
