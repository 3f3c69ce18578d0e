// Diagnostic: fp64 MFMA issue rate when every substep's fragments come from LDS (the GEMM inner loop
// without global traffic or barriers). One 256-thread workgroup per CU (1 wave per SIMD) or two.
//   TN independent accumulators per wave (16 x 16*TN wave tile), 1 A + TN B fragment reads per substep.
//   PF = 0: reads of substep q then its MFMAs; PF = 1: reads of q+1 issued ahead of the MFMAs of q (pinned).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int TN, int PF, int BAR>
__global__ void __launch_bounds__(256) k_loop(double* out, int iters, long long* cyc) {
    __shared__ double lds[2 * (32 * 80 + 64 * 32)];
    for (int i = threadIdx.x; i < 2 * (32 * 80 + 64 * 32); i += 256) lds[i] = 1e-3 * (i & 127);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const double* as = lds;
    const double* bs = lds + 64 * 32;
    constexpr int STAGE = 32 * 80 + 64 * 32;   // two stages, alternated per iteration (no hoisting)
    d4 acc[TN];
    for (int j = 0; j < TN; ++j) acc[j] = d4{0, 0, 0, 0};
    auto frag = [&](int q, double& a, double (&b)[TN]) {
        const int kk = (q & 7) * 4 + lk;
        const int r = wave * 16 + lr;
        a = as[r * 32 + ((((kk >> 1) ^ (r & 15))) << 1) + (kk & 1)];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = bs[kk * 80 + j * 16 + lr];
    };
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        as = lds + (it & 1) * STAGE;
        bs = as + 64 * 32;
        if (BAR) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        double a[2], b[2][TN];
        frag(0, a[0], b[0]);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (PF) {
                if (q + 1 < 8) frag(q + 1, a[(q + 1) & 1], b[(q + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
            } else if (q > 0) {
                frag(q, a[q & 1], b[q & 1]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q & 1], b[q & 1][j], acc[j], 0, 0, 0);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int j = 0; j < TN; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* out; long long* cyc;
    hipMalloc(&out, 1024 * 256 * 8); hipMalloc(&cyc, 64);
    const int iters = 2000;
    auto run = [&](auto kern, const char* name, int tn, int blocks) {
        long long c = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
            hipDeviceSynchronize();
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        }
        printf("%-22s blocks %4d: %.1f cycles per MFMA per wave\n", name, blocks, double(c) / (iters * 8.0 * tn));
    };
    for (int blocks : {256}) {
        run(k_loop<5, 0, 0>, "TN=5 plain", 5, blocks);
        run(k_loop<5, 1, 0>, "TN=5 read-ahead", 5, blocks);
        run(k_loop<5, 0, 1>, "TN=5 plain+barrier", 5, blocks);
        run(k_loop<5, 1, 1>, "TN=5 read-ahead+barrier", 5, blocks);
        run(k_loop<2, 0, 0>, "TN=2 plain", 2, blocks);
        run(k_loop<2, 1, 1>, "TN=2 read-ahead+barrier", 2, blocks);
    }
    return 0;
}
