// Accuracy of the hardware v_rcp_f64 / v_rsq_f64 estimates (how many Newton steps the Jacobi rotation
// parameters need): max relative error over 2^24 arguments spanning 2^-30..2^30.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void k(double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = exp2(-30.0 + 60.0 * (double(i) / n)) * (1.0 + 0.37 * sin(double(i)));
    double r = __builtin_amdgcn_rcp(x), s = __builtin_amdgcn_rsq(x);
    out[2 * i] = fabs(r * x - 1.0);
    out[2 * i + 1] = fabs(s * s * x - 1.0);
}

int main() {
    const int n = 1 << 24;
    double* d;
    if (hipMalloc(&d, size_t(n) * 16) != hipSuccess) return 1;
    k<<<n / 256, 256>>>(d, n);
    double* h = new double[size_t(n) * 2];
    if (hipMemcpy(h, d, size_t(n) * 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    double mr = 0, ms = 0;
    for (int i = 0; i < n; ++i) {
        mr = fmax(mr, h[2 * i]);
        ms = fmax(ms, h[2 * i + 1]);
    }
    std::printf("max rel err rcp %.3e (%.1f bits)  rsq^2 %.3e (%.1f bits)\n", mr, -log2(mr), ms, -log2(ms));
    return 0;
}
