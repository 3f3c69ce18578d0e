// FETCH_SIZE / WRITE_SIZE calibration for the access widths the kernels use (MI355X_MICROARCH.md, HBM
// section: only 16-B/lane streaming reads are calibrated; "calibrate on a known byte count in your own
// access pattern"). Streams a 1 GiB buffer (past the 256 MiB Infinity Cache) with coalesced 8-B and
// 16-B per-lane loads, and writes 256 MiB with 8-B stores; run under rocprofv3 --pmc FETCH_SIZE (and
// WRITE_SIZE in a second pass) and divide the counter by the bytes printed here.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_read8(const double* __restrict__ p, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) s += p[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void k_read16(const double2* __restrict__ p, size_t n2, double* out) {
    double s = 0.0;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n2; i += size_t(gridDim.x) * blockDim.x) s += p[i].x + p[i].y;
    if (s == 12345.678) out[0] = s;
}
__global__ void k_write8(double* __restrict__ p, size_t n) {
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = double(i);
}

int main() {
    const size_t bytes = size_t(1) << 30, n = bytes / 8;
    double *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes);
    hipDeviceSynchronize();
    k_read8<<<4096, 256>>>(buf, n, out);
    k_read16<<<4096, 256>>>(reinterpret_cast<const double2*>(buf), n / 2, out);
    k_write8<<<4096, 256>>>(buf, n / 4);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("k_read8 bytes %zu\nk_read16 bytes %zu\nk_write8 bytes %zu\n", bytes, bytes, bytes / 4);
    hipFree(buf);
    hipFree(out);
    return 0;
}
