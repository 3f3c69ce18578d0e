// Diagnostic: sustained v_mfma_f64_16x16x4_f64 rate (independent accumulators, all CUs) and the
// dependent-chain latency on one accumulator.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void __launch_bounds__(256) k_rate(double* out, int iters, long long* cyc) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double* out; long long* cyc;
    hipMalloc(&out, 2048 * 256 * 8); hipMalloc(&cyc, 64);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 4000;
    auto run = [&](auto kern, int nacc, int blocks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            double fl = double(blocks) * 4 * iters * nacc * 2048.0;
            if (rep) printf("%2d acc, %4d blocks: %.2f TFLOP/s, %.1f cycles per MFMA per wave (memtime)\n", nacc, blocks, fl / (ms * 1e-3) / 1e12, double(c) / (iters * nacc));
        }
    };
    for (int blocks : {256, 512, 1024, 2048}) { run(k_rate<4>, 4, blocks); run(k_rate<8>, 8, blocks); run(k_rate<16>, 16, blocks); }
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<1>, dim3(256), dim3(256), 0, 0, out, iters, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("1 acc (dependent chain): %.1f cycles per MFMA\n", double(c) / iters);
    return 0;
}
