// Diagnostic: FP64 VALU issue rate (v_fma_f64 with independent chains) for one workgroup of 512 threads
// (the k_sytrd_l512 shape: 8 waves, two per SIMD) and for the whole chip, plus the s_memtime tick rate
// against the event clock (so the syev stamps' "cycles" can be converted).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int NCH>
__global__ void __launch_bounds__(512) k_fma(double* out, int iters, long long* cyc) {
    double acc[NCH];
    for (int i = 0; i < NCH; ++i) acc[i] = threadIdx.x * 1e-3 + i;
    const double b = 1.0 - blockIdx.x * 1e-9, c = 1e-7;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) acc[i] = fma(acc[i], b, c);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int i = 0; i < NCH; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 4096 * 512 * 8);
    hipMalloc(&cyc, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    auto run = [&](auto kern, int nch, int blocks, int threads) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long c;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double winstr = double(iters) * nch;   // FMA instructions per wave
            const double fl = double(blocks) * threads * winstr * 2;
            if (rep)
                printf("%2d chains, %4d x %3d threads: %.2f TFLOP/s, %.2f ms, %.2f memtime ticks per wave FMA, memtime %.1f MHz\n",
                       nch, blocks, threads, fl / (ms * 1e-3) / 1e12, ms, double(c) / winstr, double(c) / (ms * 1e-3) / 1e6);
        }
    };
    for (int threads : {64, 256, 512}) {
        run(k_fma<1>, 1, 1, threads);
        run(k_fma<4>, 4, 1, threads);
        run(k_fma<8>, 8, 1, threads);
        run(k_fma<16>, 16, 1, threads);
    }
    run(k_fma<8>, 8, 256, 512);
    run(k_fma<8>, 8, 1024, 512);
    run(k_fma<16>, 16, 2048, 256);
    return 0;
}
