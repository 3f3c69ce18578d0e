// Temporary: factorisation and TT entry points not yet implemented in this build step.
#include "runtime.hpp"
using namespace xrs;
#define NI(name) throw Error{XRS_EINVAL, std::string(#name) + ": not implemented yet"}
extern "C" {
int xrs_qc(xrs_handle_t, double*, double*, size_t*, const double*, size_t, size_t) { return guarded([&] { NI(xrs_qc); }); }
int xrs_cq(xrs_handle_t, double*, double*, size_t*, const double*, size_t, size_t) { return guarded([&] { NI(xrs_cq); }); }
int xrs_qr(xrs_handle_t, double*, double*, const double*, size_t, size_t) { return guarded([&] { NI(xrs_qr); }); }
int xrs_rq(xrs_handle_t, double*, double*, const double*, size_t, size_t) { return guarded([&] { NI(xrs_rq); }); }
int xrs_svd(xrs_handle_t, double*, double*, double*, const double*, size_t, size_t) { return guarded([&] { NI(xrs_svd); }); }
int xrs_tt_move_core(xrs_handle_t, size_t, const size_t*, size_t*, double**, int, size_t, size_t, int) { return guarded([&] { NI(xrs_tt_move_core); }); }
int xrs_tt_round(xrs_handle_t, size_t, const size_t*, size_t*, double**, int, size_t, const size_t*, double) { return guarded([&] { NI(xrs_tt_round); }); }
int xrs_tt_dot(xrs_handle_t, double*, size_t, const size_t*, const size_t*, const double* const*, const size_t*, const double* const*) { return guarded([&] { NI(xrs_tt_dot); }); }
}
