// ADF measurement-operator kernels (adf.hip). A measurement operator over d modes is, per mode k, either
// the point coordinates pos_k (M int32, single point) or the vectors V_k (M x n_k row-major, rank one);
// a Mode describes one of them. Stacks are M x r row-major fp64 matrices. Everything is enqueued on
// h->stream; every reduction runs in a fixed order (bit-reproducible).
#pragma once
#include <cstddef>

#include "runtime.hpp"

namespace xrs {
namespace adf {

struct Mode {
    const int* pos = nullptr;     // single point: M coordinates of this mode
    const double* vec = nullptr;  // rank one: M x n vectors of this mode
};

// Fout (M x b) = Fprev (M x a) . C_m, C_m = C[:, pos_m, :] or sum_t V[m, t] C[:, t, :]   (adf.cpp:254-288)
void stack_forward(xrs_handle_t h, size_t M, const double* Fprev, const double* C, Mode md, size_t a, size_t n, size_t b, double* Fout);
// Bout (M x a) = C_m . Bnext (M x b)                                                     (adf.cpp:217-251)
void stack_backward(xrs_handle_t h, size_t M, const double* C, Mode md, const double* Bnext, size_t a, size_t n, size_t b, double* Bout);
// out_m = F_m . C_m . B_m, or vals_m - F_m . C_m . B_m when vals is given                (adf.cpp:290-312)
void evaluate(xrs_handle_t h, size_t M, const double* F, const double* C, Mode md, const double* B, size_t a, size_t n, size_t b,
              const double* vals, double* out);
// projected gradient component D (a x n x b): D[i, t, j] = sum_m res_m F[m, i] B[m, j] [pos_m = t] (single
// point: measurements grouped by slice through perm / seg, n + 1 offsets) or res_m V[m, t] F[m, i] B[m, j]
// (rank one)                                                                             (adf.cpp:314-396)
void projected_gradient(xrs_handle_t h, size_t M, const double* F, const double* B, const double* res, Mode md, const int* perm,
                        const int* seg, size_t a, size_t n, size_t b, double* D);
// nrm[t] = sum over the measurements of slice t of v_m^2 (single point), nrm[0] = sum_m v_m^2 and
// nrm[1..n) = 0 (rank one)                                                                (adf.cpp:413-465)
void slice_square_sums(xrs_handle_t h, size_t M, const double* v, Mode md, const int* perm, const int* seg, size_t n, double* nrm);
// C[:, t, :] += ||D[:, t, :]||^2 / nrm[t] D[:, t, :] per slice (single point), C += ||D||^2 / sum(nrm) D
// (rank one)                                                                              (adf.cpp:468-487)
void update_component(xrs_handle_t h, double* C, const double* D, const double* nrm, bool single_point, size_t a, size_t n, size_t b);
// out[0] = sum_m v_m^2 (one workgroup, fixed order)
void sum_squares(xrs_handle_t h, size_t M, const double* v, double* out);

}  // namespace adf
}  // namespace xrs
