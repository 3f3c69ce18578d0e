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

void reduce_to_device(xrs_handle_t h, int mode, const double* x, const double* y, size_t n, double* out_dev,
                      double* partial) {
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, 2.0 * double(n), double(mode == 1 ? 2 : 1) * 8.0 * double(n));
    if (partial == nullptr) partial = static_cast<double*>(h->dev_scratch) + 64;
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
    host_wait(h);
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

// out[p] = sum_i X[p][i][i]  (trace of the two trailing modes, Tensor::perform_trace tensor.cpp:781-838)
__global__ void __launch_bounds__(256) k_diag_sum(double* __restrict__ out, const double* __restrict__ X, size_t P, size_t m) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t p = size_t(blockIdx.x) * blockDim.x + threadIdx.x; p < P; p += stride) {
        const double* x = X + p * m * m;
        double s = 0.0;
        for (size_t i = 0; i < m; ++i) s += x[i * m + i];
        out[p] = s;
    }
}

void diag_sum(xrs_handle_t h, double* out, const double* X, size_t P, size_t m) {
    if (!P) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(P * m), 8.0 * double(P * (m + 1)));
    hipLaunchKernelGGL(k_diag_sum, dim3(ew_blocks(P)), dim3(256), 0, h->stream, out, X, P, m);
    check_launch("k_diag_sum");
}

// out[offsets + idx] += alpha * in[idx] for every multi-index idx of `in` (Tensor::offset_add, tensor.cpp:969-1025)
struct OffsetArgs {
    int nd;
    size_t in_dims[16];
    size_t out_str[16];
    size_t base;
};
__global__ void __launch_bounds__(256) k_offset_add(double* __restrict__ out, const double* __restrict__ in, size_t total,
                                                    double alpha, OffsetArgs a) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
        size_t rem = i, off = a.base;
        for (int k = a.nd - 1; k >= 0; --k) {
            off += (rem % a.in_dims[k]) * a.out_str[k];
            rem /= a.in_dims[k];
        }
        out[off] += alpha * in[i];
    }
}

void offset_add(xrs_handle_t h, double* out, const size_t* out_dims, const double* in, const size_t* in_dims, size_t nd,
                const size_t* offsets, double alpha) {
    XRS_REQUIRE(nd <= 16, "offset_add: too many modes");
    OffsetArgs a{};
    a.nd = int(nd);
    size_t total = 1, s = 1;
    a.base = 0;
    for (int k = int(nd) - 1; k >= 0; --k) {
        a.in_dims[k] = in_dims[k];
        a.out_str[k] = s;
        a.base += offsets[k] * s;
        s *= out_dims[k];
        total *= in_dims[k];
    }
    if (!total) return;
    KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(total), 24.0 * double(total));
    hipLaunchKernelGGL(k_offset_add, dim3(ew_blocks(total)), dim3(256), 0, h->stream, out, in, total, alpha, a);
    check_launch("k_offset_add");
}

// Generalised evaluation (internal::evaluate, indexedTensor_tensor_evaluate.cpp:248-390):
// out[o] = sum_{t} in[base + sum_k o_k*in_str[k] + sum_j t_j*tr_str[j]], o over out_dims, t over tr_dims.
// Covers fixed indices (base offset), traces (tr_*) and diagonals in one pass; plain permutations use the
// LDS-tiled permute instead. One thread per output element, consecutive threads walk the last out mode.
struct EvalArgs {
    int nd, nt;
    size_t out_dims[24];
    size_t in_str[24];
    size_t tr_dims[12];
    size_t tr_str[12];
    size_t base;
    size_t tr_total;
};
__global__ void __launch_bounds__(256) k_strided_eval(double* __restrict__ out, const double* __restrict__ in, size_t total,
                                                      EvalArgs a) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
        size_t rem = i, off = a.base;
        for (int k = a.nd - 1; k >= 0; --k) {
            off += (rem % a.out_dims[k]) * a.in_str[k];
            rem /= a.out_dims[k];
        }
        double s = 0.0;
        for (size_t t = 0; t < a.tr_total; ++t) {
            size_t r = t, o2 = off;
            for (int j = a.nt - 1; j >= 0; --j) {
                o2 += (r % a.tr_dims[j]) * a.tr_str[j];
                r /= a.tr_dims[j];
            }
            s += in[o2];
        }
        out[i] = s;
    }
}

void strided_eval(xrs_handle_t h, double* out, const double* in, size_t nd, const size_t* out_dims, const size_t* in_strides,
                  size_t nt, const size_t* tr_dims, const size_t* tr_strides, size_t base) {
    XRS_REQUIRE(nd <= 24 && nt <= 12, "strided_eval: too many modes");
    EvalArgs a{};
    a.nd = int(nd);
    a.nt = int(nt);
    a.base = base;
    size_t total = 1;
    for (size_t k = 0; k < nd; ++k) {
        a.out_dims[k] = out_dims[k];
        a.in_str[k] = in_strides[k];
        total *= out_dims[k];
    }
    a.tr_total = 1;
    for (size_t j = 0; j < nt; ++j) {
        a.tr_dims[j] = tr_dims[j];
        a.tr_str[j] = tr_strides[j];
        a.tr_total *= tr_dims[j];
    }
    if (!total) return;
    KernelTimer timer(h, XRS_KFAM_PERMUTE, double(total * a.tr_total), 8.0 * double(total * (a.tr_total + 1)));
    hipLaunchKernelGGL(k_strided_eval, dim3(ew_blocks(total)), dim3(256), 0, h->stream, out, in, total, a);
    check_launch("k_strided_eval");
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
        fence_readers(h);
        scal(h, x, alpha, n);
    });
}

int xrs_axpy(xrs_handle_t h, double* y, double alpha, const double* x, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || (x && y)), "null argument");
        fence_readers(h);
        axpy(h, y, alpha, x, n);
    });
}

int xrs_scale_rows(xrs_handle_t h, double* X, const double* s, size_t m, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (m * n == 0 || (X && s)), "null argument");
        fence_readers(h);
        scale_rows(h, X, s, m, n);
    });
}

}  // extern "C"
