// Level-1 kernels: norms, dot, scaling, axpy, diagonal row scaling.
// Replace blasWrapper::one_norm/two_norm/dot_product (blasLapackWrapper.cpp:76-110), misc::scale /
// add_scaled (misc/basicArraySupport.h:60-110) and the diag(S)*dense product of round_edge
// (sparseTimesFullContraction.cpp:66-96). All HBM-bound; reductions are two-level and deterministic
// (fixed block partial order), fp64 throughout.
#include "elementwise.hpp"

namespace xrs {

constexpr int RB = 256;        // threads per reduction block
constexpr int RMAXB = 1024;    // max partial blocks

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double block_sum(double v) {
    __shared__ double part[RB / 64];
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) part[w] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < RB / 64; ++i) s += part[i];
    }
    __syncthreads();
    return s;  // valid in thread 0
}

// mode 0: sum x^2, 1: sum x*y, 2: sum |x|
template <int MODE>
__global__ void __launch_bounds__(RB) k_reduce_partial(const double* __restrict__ x, const double* __restrict__ y, size_t n,
                                                       double* __restrict__ partial) {
    double acc = 0.0;
    const size_t stride = size_t(gridDim.x) * RB;
    for (size_t i = size_t(blockIdx.x) * RB + threadIdx.x; i < n; i += stride) {
        const double a = x[i];
        if (MODE == 0) acc += a * a;
        else if (MODE == 1) acc += a * y[i];
        else acc += fabs(a);
    }
    const double s = block_sum(acc);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void __launch_bounds__(RB) k_reduce_final(const double* __restrict__ partial, int nb, double* __restrict__ out,
                                                     int take_sqrt) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < nb; i += RB) acc += partial[i];
    const double s = block_sum(acc);
    if (threadIdx.x == 0) out[0] = take_sqrt ? sqrt(s) : s;
}

void reduce_to_device(xrs_handle_t h, int mode, const double* x, const double* y, size_t n, double* out_dev) {
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, 2.0 * double(n), double(mode == 1 ? 2 : 1) * 8.0 * double(n));
    double* partial = static_cast<double*>(h->dev_scratch) + 64;
    const int nb = int(std::max<size_t>(1, std::min<size_t>(RMAXB, (n + RB * 4 - 1) / (RB * 4))));
    if (mode == 0) hipLaunchKernelGGL(k_reduce_partial<0>, dim3(nb), dim3(RB), 0, h->stream, x, y, n, partial);
    else if (mode == 1) hipLaunchKernelGGL(k_reduce_partial<1>, dim3(nb), dim3(RB), 0, h->stream, x, y, n, partial);
    else hipLaunchKernelGGL(k_reduce_partial<2>, dim3(nb), dim3(RB), 0, h->stream, x, y, n, partial);
    check_launch("k_reduce_partial");
    hipLaunchKernelGGL(k_reduce_final, dim3(1), dim3(RB), 0, h->stream, partial, nb, out_dev, mode == 0 ? 1 : 0);
    check_launch("k_reduce_final");
}

double reduce_to_host(xrs_handle_t h, int mode, const double* x, const double* y, size_t n) {
    if (n == 0) return 0.0;
    double* out = static_cast<double*>(h->dev_scratch);
    reduce_to_device(h, mode, x, y, n, out);
    double* host = static_cast<double*>(h->host_scratch);
    XRS_HIP(hipMemcpyAsync(host, out, 8, hipMemcpyDeviceToHost, h->stream));
    XRS_HIP(hipStreamSynchronize(h->stream));
    return host[0];
}

__global__ void __launch_bounds__(256) k_scal(double* __restrict__ x, double alpha, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= alpha;
}

__global__ void __launch_bounds__(256) k_axpy(double* __restrict__ y, double alpha, const double* __restrict__ x, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) y[i] += alpha * x[i];
}

__global__ void __launch_bounds__(256) k_scale_rows(double* __restrict__ X, const double* __restrict__ s, size_t m, size_t n) {
    const size_t total = m * n;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) X[i] *= s[i / n];
}

__global__ void __launch_bounds__(256) k_scale_cols(double* __restrict__ X, const double* __restrict__ s, size_t m, size_t n) {
    const size_t total = m * n;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) X[i] *= s[i % n];
}

static unsigned ew_blocks(size_t n) { return unsigned(std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192))); }

void scal(xrs_handle_t h, double* x, double alpha, size_t n) {
    if (!n || alpha == 1.0) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(n), 16.0 * double(n));
    hipLaunchKernelGGL(k_scal, dim3(ew_blocks(n)), dim3(256), 0, h->stream, x, alpha, n);
    check_launch("k_scal");
}

void axpy(xrs_handle_t h, double* y, double alpha, const double* x, size_t n) {
    if (!n) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, 2.0 * double(n), 24.0 * double(n));
    hipLaunchKernelGGL(k_axpy, dim3(ew_blocks(n)), dim3(256), 0, h->stream, y, alpha, x, n);
    check_launch("k_axpy");
}

void scale_rows(xrs_handle_t h, double* X, const double* s, size_t m, size_t n) {
    if (!m || !n) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(m * n), 16.0 * double(m * n));
    hipLaunchKernelGGL(k_scale_rows, dim3(ew_blocks(m * n)), dim3(256), 0, h->stream, X, s, m, n);
    check_launch("k_scale_rows");
}

void scale_cols(xrs_handle_t h, double* X, const double* s, size_t m, size_t n) {
    if (!m || !n) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(m * n), 16.0 * double(m * n));
    hipLaunchKernelGGL(k_scale_cols, dim3(ew_blocks(m * n)), dim3(256), 0, h->stream, X, s, m, n);
    check_launch("k_scale_cols");
}

}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_nrm2(xrs_handle_t h, double* result, const double* x, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && result && (n == 0 || x), "null argument");
        *result = reduce_to_host(h, 0, x, nullptr, n);
    });
}

int xrs_dot(xrs_handle_t h, double* result, const double* x, const double* y, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && result && (n == 0 || (x && y)), "null argument");
        *result = reduce_to_host(h, 1, x, y, n);
    });
}

int xrs_asum(xrs_handle_t h, double* result, const double* x, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && result && (n == 0 || x), "null argument");
        *result = reduce_to_host(h, 2, x, nullptr, n);
    });
}

int xrs_scal(xrs_handle_t h, double* x, double alpha, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || x), "null argument");
        scal(h, x, alpha, n);
    });
}

int xrs_axpy(xrs_handle_t h, double* y, double alpha, const double* x, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || (x && y)), "null argument");
        axpy(h, y, alpha, x, n);
    });
}

int xrs_scale_rows(xrs_handle_t h, double* X, const double* s, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (m * n == 0 || (X && s)), "null argument");
        scale_rows(h, X, s, m, n);
    });
}

}  // extern "C"
