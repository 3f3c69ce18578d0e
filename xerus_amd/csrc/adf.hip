// ADF measurement-operator kernels (reference src/xerus/algorithms/adf.cpp:217-487; declarations and
// semantics in adf.hpp). The reference walks the measurements one by one on the host (OpenMP over
// de-duplicated stack entries); here one launch covers all M measurements of a component:
//   - stacks / evaluations: one thread per output entry (m, j), the component slice gathered by the
//     measurement's coordinate (single point) or mixed by its vector (rank one) -- HBM-bound on the
//     M x r stacks, the component itself stays cache-resident;
//   - reductions over measurements (projected gradient, slice norms, residual norm): one workgroup per
//     output entry, a strided partial sum per thread and a fixed-order LDS tree, so results do not depend
//     on scheduling.
#include "adf.hpp"

namespace xrs {
namespace adf {

namespace {

constexpr int kThreads = 256;

unsigned grid_of(size_t n) { return unsigned(std::min<size_t>(std::max<size_t>((n + kThreads - 1) / kThreads, 1), 65535)); }

// entry (i, j) of the measurement's component matrix C_m (a x b)
__device__ __forceinline__ double cm(const double* __restrict__ C, const int* __restrict__ pos, const double* __restrict__ vec, size_t m,
                                     size_t i, size_t j, size_t n, size_t b) {
    if (pos) return C[(i * n + size_t(pos[m])) * b + j];
    double s = 0.0;
    const double* v = vec + m * n;
    for (size_t t = 0; t < n; ++t) s = fma(v[t], C[(i * n + t) * b + j], s);
    return s;
}

__global__ void __launch_bounds__(kThreads) k_stack_forward(size_t M, const double* __restrict__ Fprev, const double* __restrict__ C,
                                                            const int* __restrict__ pos, const double* __restrict__ vec, size_t a,
                                                            size_t n, size_t b, double* __restrict__ Fout) {
    for (size_t e = size_t(blockIdx.x) * kThreads + threadIdx.x; e < M * b; e += size_t(gridDim.x) * kThreads) {
        const size_t m = e / b, j = e - m * b;
        double s = 0.0;
        for (size_t i = 0; i < a; ++i) s = fma(Fprev[m * a + i], cm(C, pos, vec, m, i, j, n, b), s);
        Fout[e] = s;
    }
}

__global__ void __launch_bounds__(kThreads) k_stack_backward(size_t M, const double* __restrict__ C, const int* __restrict__ pos,
                                                             const double* __restrict__ vec, const double* __restrict__ Bnext,
                                                             size_t a, size_t n, size_t b, double* __restrict__ Bout) {
    for (size_t e = size_t(blockIdx.x) * kThreads + threadIdx.x; e < M * a; e += size_t(gridDim.x) * kThreads) {
        const size_t m = e / a, i = e - m * a;
        double s = 0.0;
        for (size_t j = 0; j < b; ++j) s = fma(cm(C, pos, vec, m, i, j, n, b), Bnext[m * b + j], s);
        Bout[e] = s;
    }
}

__global__ void __launch_bounds__(kThreads) k_evaluate(size_t M, const double* __restrict__ F, const double* __restrict__ C,
                                                       const int* __restrict__ pos, const double* __restrict__ vec,
                                                       const double* __restrict__ B, size_t a, size_t n, size_t b,
                                                       const double* __restrict__ vals, double* __restrict__ out) {
    for (size_t m = size_t(blockIdx.x) * kThreads + threadIdx.x; m < M; m += size_t(gridDim.x) * kThreads) {
        double s = 0.0;
        for (size_t i = 0; i < a; ++i) {
            double r = 0.0;
            for (size_t j = 0; j < b; ++j) r = fma(cm(C, pos, vec, m, i, j, n, b), B[m * b + j], r);
            s = fma(F[m * a + i], r, s);
        }
        out[m] = vals ? vals[m] - s : s;
    }
}

// fixed-order sum of the block's partial values (every thread returns the total)
__device__ double block_sum(double v) {
    __shared__ double red[kThreads];
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int o = kThreads / 2; o > 0; o >>= 1) {
        if (int(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double t = red[0];
    __syncthreads();
    return t;
}

// one workgroup per entry (i, t, j) of D (a x n x b)
__global__ void __launch_bounds__(kThreads) k_projected_gradient(size_t M, const double* __restrict__ F, const double* __restrict__ B,
                                                                 const double* __restrict__ res, const double* __restrict__ vec,
                                                                 const int* __restrict__ perm, const int* __restrict__ seg, size_t a,
                                                                 size_t n, size_t b, double* __restrict__ D) {
    const size_t e = blockIdx.x, i = e / (n * b), t = (e / b) % n, j = e % b;
    double s = 0.0;
    if (perm) {   // single point: the measurements of slice t
        for (int q = seg[t] + int(threadIdx.x); q < seg[t + 1]; q += kThreads) {
            const size_t m = size_t(perm[q]);
            s = fma(res[m] * F[m * a + i], B[m * b + j], s);
        }
    } else {      // rank one: every measurement, weighted by its vector entry t
        for (size_t m = threadIdx.x; m < M; m += kThreads) s = fma(res[m] * vec[m * n + t] * F[m * a + i], B[m * b + j], s);
    }
    s = block_sum(s);
    if (threadIdx.x == 0) D[e] = s;
}

// one workgroup per slice t
__global__ void __launch_bounds__(kThreads) k_slice_square_sums(size_t M, const double* __restrict__ v, const int* __restrict__ perm,
                                                                const int* __restrict__ seg, double* __restrict__ nrm) {
    const size_t t = blockIdx.x;
    double s = 0.0;
    if (perm) {
        for (int q = seg[t] + int(threadIdx.x); q < seg[t + 1]; q += kThreads) {
            const double x = v[perm[q]];
            s = fma(x, x, s);
        }
    } else if (t == 0) {
        for (size_t m = threadIdx.x; m < M; m += kThreads) s = fma(v[m], v[m], s);
    }
    s = block_sum(s);
    if (threadIdx.x == 0) nrm[t] = s;
}

// single point: one workgroup per slice t, step ||D_t||^2 / nrm[t]; rank one: one workgroup, step
// ||D||^2 / sum_t nrm[t]
__global__ void __launch_bounds__(kThreads) k_update(double* __restrict__ C, const double* __restrict__ D, const double* __restrict__ nrm,
                                                     int single_point, size_t a, size_t n, size_t b) {
    const size_t t = blockIdx.x;
    double s = 0.0;
    if (single_point) {
        for (size_t e = threadIdx.x; e < a * b; e += kThreads) {
            const double x = D[((e / b) * n + t) * b + e % b];
            s = fma(x, x, s);
        }
        const double step = block_sum(s) / nrm[t];
        for (size_t e = threadIdx.x; e < a * b; e += kThreads) {
            const size_t k = ((e / b) * n + t) * b + e % b;
            C[k] = fma(step, D[k], C[k]);
        }
    } else {
        for (size_t e = threadIdx.x; e < a * n * b; e += kThreads) s = fma(D[e], D[e], s);
        const double pyr = block_sum(s);
        double den = 0.0;
        for (size_t q = 0; q < n; ++q) den += nrm[q];
        const double step = pyr / den;
        for (size_t e = threadIdx.x; e < a * n * b; e += kThreads) C[e] = fma(step, D[e], C[e]);
    }
}

__global__ void __launch_bounds__(kThreads) k_sum_squares(size_t M, const double* __restrict__ v, double* __restrict__ out) {
    double s = 0.0;
    for (size_t m = threadIdx.x; m < M; m += kThreads) s = fma(v[m], v[m], s);
    s = block_sum(s);
    if (threadIdx.x == 0) out[0] = s;
}

}  // namespace

void stack_forward(xrs_handle_t h, size_t M, const double* Fprev, const double* C, Mode md, size_t a, size_t n, size_t b, double* Fout) {
    hipLaunchKernelGGL(k_stack_forward, dim3(grid_of(M * b)), dim3(kThreads), 0, h->stream, M, Fprev, C, md.pos, md.vec, a, n, b, Fout);
    check_launch("k_stack_forward");
}

void stack_backward(xrs_handle_t h, size_t M, const double* C, Mode md, const double* Bnext, size_t a, size_t n, size_t b, double* Bout) {
    hipLaunchKernelGGL(k_stack_backward, dim3(grid_of(M * a)), dim3(kThreads), 0, h->stream, M, C, md.pos, md.vec, Bnext, a, n, b, Bout);
    check_launch("k_stack_backward");
}

void evaluate(xrs_handle_t h, size_t M, const double* F, const double* C, Mode md, const double* B, size_t a, size_t n, size_t b,
              const double* vals, double* out) {
    hipLaunchKernelGGL(k_evaluate, dim3(grid_of(M)), dim3(kThreads), 0, h->stream, M, F, C, md.pos, md.vec, B, a, n, b, vals, out);
    check_launch("k_evaluate");
}

void projected_gradient(xrs_handle_t h, size_t M, const double* F, const double* B, const double* res, Mode md, const int* perm,
                        const int* seg, size_t a, size_t n, size_t b, double* D) {
    XRS_REQUIRE(a * n * b <= size_t(1) << 31, "adf: component too large");
    XRS_REQUIRE(md.pos ? perm != nullptr : md.vec != nullptr, "adf: single point gradient needs the slice grouping");
    hipLaunchKernelGGL(k_projected_gradient, dim3(unsigned(a * n * b)), dim3(kThreads), 0, h->stream, M, F, B, res, md.vec,
                       md.pos ? perm : nullptr, seg, a, n, b, D);
    check_launch("k_projected_gradient");
}

void slice_square_sums(xrs_handle_t h, size_t M, const double* v, Mode md, const int* perm, const int* seg, size_t n, double* nrm) {
    hipLaunchKernelGGL(k_slice_square_sums, dim3(unsigned(n)), dim3(kThreads), 0, h->stream, M, v, md.pos ? perm : nullptr, seg, nrm);
    check_launch("k_slice_square_sums");
}

void update_component(xrs_handle_t h, double* C, const double* D, const double* nrm, bool single_point, size_t a, size_t n, size_t b) {
    hipLaunchKernelGGL(k_update, dim3(single_point ? unsigned(n) : 1u), dim3(kThreads), 0, h->stream, C, D, nrm, int(single_point), a, n, b);
    check_launch("k_update");
}

void sum_squares(xrs_handle_t h, size_t M, const double* v, double* out) {
    hipLaunchKernelGGL(k_sum_squares, dim3(1), dim3(kThreads), 0, h->stream, M, v, out);
    check_launch("k_sum_squares");
}

}  // namespace adf
}  // namespace xrs
