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
// The front end alone (E_1 / F_{d-1} and one step per end) for dot32.hip's per-product steps: E_2 and F_{d-2} in fp32
// (row strides lde / ldf), their max words written into mword[0] / mword[1], the cores' maxima into the caller's
// slot arrays (kCmaxSlots words per core: X_k at k, Y_k at d + k), and 4d exponent words at `words` (device; the
// caller reads them back and passes them to front_exponent / front_words_bad). mem holds the buffers: keep it until
// the caller's launches are enqueued.
struct Front {
    unsigned* mword[2] = {nullptr, nullptr};
    unsigned* slots = nullptr;
    const float* E = nullptr;
    const float* F = nullptr;
    size_t lde = 0, ldf = 0;
    int* words = nullptr;
    DevBuf mem;
};
bool front_applicable(size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                      const double* const* Y);
void front(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y, Front& fr);
int front_exponent(const int* hw, size_t d, int end);
bool front_words_bad(const int* hw, size_t d);
}  // namespace zip
}  // namespace xrs
