// Kernel-boundary cost on one stream: back-to-back dependent launches vs the same launches replayed
// from a hipGraph. hipcc --offload-arch=gfx950 -O3 -o tools/boundary_bench tools/boundary_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));                \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__global__ void k_tiny(double* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

// 512 threads, 16 KB LDS, each block writes 8 KB (like a 32x32 fp64 GEMM tile)
__global__ void __launch_bounds__(512) k_tile(double* p, int n) {
    __shared__ double s[2048];
    for (int i = threadIdx.x; i < 2048; i += 512) s[i] = double(i + blockIdx.x);
    __syncthreads();
    double* o = p + size_t(blockIdx.x) * 1024;
    for (int i = threadIdx.x; i < 1024; i += 512) o[i] = s[i] + s[i + 1024] + double(n);
}

template <class F>
static double time_us(hipStream_t st, int reps, F&& f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3 / reps;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double* p;
    CK(hipMalloc(&p, size_t(4096) * 1024 * 8));
    CK(hipMemset(p, 0, size_t(4096) * 1024 * 8));
    const int chain = 100;
    for (int blocks : {1, 256, 1024, 4096}) {
        auto eager_tiny = [&] { for (int i = 0; i < chain; ++i) hipLaunchKernelGGL(k_tiny, dim3(blocks), dim3(64), 0, st, p); };
        auto eager_tile = [&] { for (int i = 0; i < chain; ++i) hipLaunchKernelGGL(k_tile, dim3(blocks), dim3(512), 0, st, p, i); };
        hipGraph_t g1, g2;
        hipGraphExec_t e1, e2;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        eager_tiny();
        CK(hipStreamEndCapture(st, &g1));
        CK(hipGraphInstantiate(&e1, g1, nullptr, nullptr, 0));
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        eager_tile();
        CK(hipStreamEndCapture(st, &g2));
        CK(hipGraphInstantiate(&e2, g2, nullptr, nullptr, 0));
        const double t1 = time_us(st, 20, eager_tiny) / chain;
        const double t2 = time_us(st, 20, [&] { CK(hipGraphLaunch(e1, st)); }) / chain;
        const double t3 = time_us(st, 20, eager_tile) / chain;
        const double t4 = time_us(st, 20, [&] { CK(hipGraphLaunch(e2, st)); }) / chain;
        std::printf("blocks %5d: tiny eager %.2f us, graph %.2f us | 512-thread tile eager %.2f us, graph %.2f us\n", blocks,
                    t1, t2, t3, t4);
        CK(hipGraphExecDestroy(e1));
        CK(hipGraphExecDestroy(e2));
        CK(hipGraphDestroy(g1));
        CK(hipGraphDestroy(g2));
    }
    // cross-stream hop: kernel on s0, event, s1 waits and runs a kernel, event, s0 waits, ...
    {
        hipStream_t s1;
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        hipEvent_t ev[2];
        CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
        const int hops = 100;
        auto pingpong = [&] {
            for (int i = 0; i < hops; ++i) {
                hipStream_t a = (i & 1) ? s1 : st, b = (i & 1) ? st : s1;
                hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, a, p);
                CK(hipEventRecord(ev[i & 1], a));
                CK(hipStreamWaitEvent(b, ev[i & 1], 0));
            }
        };
        const double t_ev = time_us(st, 10, pingpong) / hops;
        // same chain with hipStreamWriteValue32 / hipStreamWaitValue32 on a device flag
        unsigned* flag;
        CK(hipMalloc(&flag, 64));
        CK(hipMemset(flag, 0, 64));
        unsigned epoch = 0;
        auto pingpong_val = [&] {
            for (int i = 0; i < hops; ++i) {
                hipStream_t a = (i & 1) ? s1 : st, b = (i & 1) ? st : s1;
                hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, a, p);
                ++epoch;
                CK(hipStreamWriteValue32(a, flag, epoch, 0));
                CK(hipStreamWaitValue32(b, flag, epoch, hipStreamWaitValueGte, 0xffffffffu));
            }
        };
        const double t_val = time_us(st, 10, pingpong_val) / hops;
        std::printf("cross-stream hop (tiny kernel + dependency): events %.2f us, write/wait value %.2f us\n", t_ev, t_val);
        CK(hipStreamSynchronize(s1));
        CK(hipFree(flag));
    }
    CK(hipFree(p));
    return 0;
}
