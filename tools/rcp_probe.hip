// v_rcp_f64 accuracy probe (diagnostics): max relative error of the hardware reciprocal estimate and
// after one / two Newton steps, over 2^22 inputs spread across many binades
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_rcp(const double* x, double* r0, double* r1, double* r2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r = __builtin_amdgcn_rcp(v);
    r0[i] = r;
    double t = fma(-v, r, 1.0);
    r = fma(r, t, r);
    r1[i] = r;
    t = fma(-v, r, 1.0);
    r2[i] = fma(r, t, r);
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double m = 1.0 + double(s >> 11) * (1.0 / 9007199254740992.0);
        x[i] = std::ldexp(m, int(s % 200) - 100) * ((s >> 9) & 1 ? -1.0 : 1.0);
    }
    double *dx, *d0, *d1, *d2;
    if (hipMalloc(&dx, n * 8) || hipMalloc(&d0, n * 8) || hipMalloc(&d1, n * 8) || hipMalloc(&d2, n * 8)) return 1;
    if (hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice)) return 1;
    hipLaunchKernelGGL(k_rcp, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, n);
    std::vector<double> r0(n), r1(n), r2(n);
    if (hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost) || hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost) ||
        hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost))
        return 1;
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ex = 1.0L / (long double)x[i];
        e0 = std::fmax(e0, double(std::fabs((r0[i] - ex) / ex)));
        e1 = std::fmax(e1, double(std::fabs((r1[i] - ex) / ex)));
        e2 = std::fmax(e2, double(std::fabs((r2[i] - ex) / ex)));
    }
    std::printf("v_rcp_f64 max rel err: estimate %.3e (2^%.1f), 1 Newton %.3e, 2 Newton %.3e (u = 1.11e-16)\n", e0, std::log2(e0), e1, e2);
    return 0;
}
