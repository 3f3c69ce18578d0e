// <x,y> of two TTs on fp32 MFMA tiles (xrs_tt_dot_f32): the north star's "dense contraction on MFMA fp32
// tiles" as a side path beside the fp64 zipper (tt.hip: dot_two_ended), which stays the reference-precision
// product (value_t = double, include/xerus/basic.h:44; ttNetwork.cpp:782-789). Same two-ended zipper:
//   left  E_{k+1} = sum_i X_k[:,i,:]^T E_k Y_k[:,i,:]       (E_0 = 1)
//   right F_k     = sum_i X_k[:,i,:] F_{k+1} Y_k[:,i,:]^T   (F_d = 1)
// closed at the middle edge m by sum_ab E_m[a,b] F_m[a,b] (accumulated in fp64).
//
// The cores stay the caller's fp64 blocks: every GEMM reads them from HBM as doubles and rounds them to
// fp32 on the way into LDS (no conversion pass, no second copy). v_mfma_f32_16x16x4_f32 issues every 32
// cycles per SIMD (the fp64 form every 64): 157 TF/s peak against 78.6. Environments and the intermediate
// T live in fp32. Range: after every step the environment is renormalised by a power of two -- the
// reduce kernel that sums the split-K slabs also takes max|E| (atomicMax on the float bits), the next
// step's GEMM scales its environment operand by 2^-e at load (exact) -- and the host adds the exponents
// back in fp64, so long chains neither overflow nor underflow; a single core's entries must fit fp32.
// Accuracy: fp32 rounding of the cores and of each product, ~1e-7 relative to ||x|| ||y|| (tests).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "runtime.hpp"

namespace xrs {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

// 64 x 64 output tile, 32-deep K steps, 512 threads = two groups of 4 waves of 32 x 32 (2 x 2 MFMA 16x16x4
// tiles, four independent accumulation chains against the 40-cycle dependent latency); the two groups take
// the even / odd 4-deep k-substeps of every step and are summed through LDS at the end (the TT-shape grids
// are ~1.25 workgroups per CU: the second group doubles the waves that hide load and LDS latency). LDS
// image [k][m] with a row pitch of 80 floats: the fragment reads (16 rows m x 4 k per wave) land on
// distinct banks.
constexpr int BM = 64, BN = 64, BK = 32, NT = 512, SP = BM + 16;
constexpr int APER = BM * BK / NT, BPER = BN * BK / NT;   // 4 elements per thread and operand

// power-of-two scale 2^-e with max|E| * 2^-e in [0.5, 1) (frexp convention); 1 for a zero environment
__device__ __forceinline__ float pow2_scale(unsigned maxbits) {
    const int ef = int((maxbits >> 23) & 0xff);
    if (maxbits == 0u) return 1.0f;
    return __uint_as_float(unsigned(253 - ef) << 23);   // 2^-(ef - 126)
}

// C (M x N fp32, slab blockIdx.z of a split-K launch: C + z*M*N) = s op(A) op(B) over the K-slice
// [z*kps, z*kps + kps). op(A) = A^T when TA (A stored K x M, lda), else A (M x K); op(B) = B^T when TB
// (B stored N x K), else B (K x N). A, B fp32 or fp64 (rounded to fp32 at load); sa / sb: optional device
// max|.| words whose power-of-two scale is applied to that operand at load.
template <bool TA, bool TB, class EA, class EB>
__global__ void __launch_bounds__(NT) k_gemm32(int M, int N, int K, int kps, const EA* __restrict__ A, size_t lda,
                                               const EB* __restrict__ B, size_t ldb, const unsigned* __restrict__ sa,
                                               const unsigned* __restrict__ sb, float* __restrict__ C,
                                               unsigned* __restrict__ zw) {
    // zw: the max word the slab sum after this launch accumulates into; zeroed here (stream order: the
    // sum's atomics run after this kernel has ended), so no memset launch precedes the zipper
    if (zw != nullptr && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) *zw = 0u;
    __shared__ float As[2][BK * SP];
    __shared__ float Bs[2][BK * SP];
    const int tiles_m = (M + BM - 1) / BM;
    const int m0 = int(blockIdx.x % tiles_m) * BM, n0 = int(blockIdx.x / tiles_m) * BN;
    const int kbeg = int(blockIdx.z) * kps, kend = min(K, kbeg + kps);
    const float fa = sa ? pow2_scale(*sa) : 1.0f, fb = sb ? pow2_scale(*sb) : 1.0f;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kg = wave >> 2, pw = wave & 3;
    const int wm = (pw >> 1) * 32, wn = (pw & 1) * 32;
    const int lr = lane & 15, lk = lane >> 4;

    // thread -> (row, k) of the staged element: the operand's contiguous index fastest (coalesced reads)
    auto a_rk = [&](int e, int& m, int& k) {
        const int idx = tid + e * NT;
        if (TA) { m = idx % BM; k = idx / BM; } else { k = idx % BK; m = idx / BK; }
    };
    auto b_rk = [&](int e, int& n, int& k) {
        const int idx = tid + e * NT;
        if (TB) { k = idx % BK; n = idx / BK; } else { n = idx % BN; k = idx / BN; }
    };
    EA ra[2][APER];
    EB rb[2][BPER];
    auto load = [&](int slot, int k0) {
#pragma unroll
        for (int e = 0; e < APER; ++e) {
            int m, k;
            a_rk(e, m, k);
            const int gm = min(m0 + m, M - 1), gk = min(k0 + k, kend - 1);
            ra[slot][e] = TA ? A[size_t(gk) * lda + gm] : A[size_t(gm) * lda + gk];
        }
#pragma unroll
        for (int e = 0; e < BPER; ++e) {
            int n, k;
            b_rk(e, n, k);
            const int gn = min(n0 + n, N - 1), gk = min(k0 + k, kend - 1);
            rb[slot][e] = TB ? B[size_t(gn) * ldb + gk] : B[size_t(gk) * ldb + gn];
        }
    };
    auto store = [&](int buf, int slot, int k0) {
#pragma unroll
        for (int e = 0; e < APER; ++e) {
            int m, k;
            a_rk(e, m, k);
            const bool ok = m0 + m < M && k0 + k < kend;
            As[buf][k * SP + m] = ok ? float(ra[slot][e]) * fa : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < BPER; ++e) {
            int n, k;
            b_rk(e, n, k);
            const bool ok = n0 + n < N && k0 + k < kend;
            Bs[buf][k * SP + n] = ok ? float(rb[slot][e]) * fb : 0.0f;
        }
    };
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int buf) {
        const float* as = As[buf];
        const float* bs = Bs[buf];
#pragma unroll
        for (int qq = 0; qq < BK / 8; ++qq) {
            const int kr = ((2 * qq + kg) * 4 + lk) * SP;
            const float a0 = as[kr + wm + lr], a1 = as[kr + wm + 16 + lr];
            const float b0 = bs[kr + wn + lr], b1 = bs[kr + wn + 16 + lr];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
    };
    // two register slots: the loads of step t + 2 are issued while step t computes
    const int ns = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    if (ns > 0) {
        load(0, kbeg);
        load(1, kbeg + BK);
        store(0, 0, kbeg);
        __syncthreads();
        // (slot indices compile-time: the loop is unrolled by the two slots, no dynamic register indexing).
        // Branch-free steps: the loads past the slice end read clamped addresses and the stores past it
        // write zeros into the idle buffer, so the waitcnt pass keeps the ring's loads in flight across a
        // step instead of draining vmcnt(0) at a branch.
        auto step = [&](int t, auto s_c) {
            constexpr int s = decltype(s_c)::value;
            compute(s);
            store(s ^ 1, s ^ 1, kbeg + (t + 1) * BK);
            load(s, kbeg + (t + 2) * BK);
            __syncthreads();
        };
        int t = 0;
        for (; t + 2 <= ns; t += 2) {
            step(t, std::integral_constant<int, 0>{});
            step(t + 1, std::integral_constant<int, 1>{});
        }
        if (t < ns) compute(0);
    }
    // second wave group's partial sums -> LDS -> the first group
    __syncthreads();
    float* red = &As[0][0];
    if (kg == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[((pw * 4 + i * 2 + j) * 4 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (kg == 1) return;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] += red[((pw * 4 + i * 2 + j) * 4 + r) * 64 + lane];
    float* out = C + size_t(blockIdx.z) * size_t(M) * size_t(N);
    const int lc = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn + j * 16 + lc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm + i * 16 + lg * 4 + r;   // C/D map of the f32 16x16x4 form
                if (row < M && col < N) out[size_t(row) * N + col] = acc[i][j][r];
            }
        }
}

// E[i] = sum_z slab[z][i] (slice order: deterministic), and max|E| into *amax (non-negative floats order
// as their bit patterns)
__global__ void __launch_bounds__(256) k_slab_sum_max(const float* __restrict__ slab, int S, int MN, float* __restrict__ E,
                                                     unsigned* __restrict__ amax) {
    __shared__ float red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    float m = 0.0f;
    if (i < MN) {
        // slices in order (deterministic); the loads of 8 slices are issued before their sums
        float s = 0.0f;
        int z = 0;
        for (; z + 8 <= S; z += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = slab[size_t(z + u) * MN + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; z < S; ++z) s += slab[size_t(z) * MN + i];
        E[i] = s;
        m = fabsf(s);
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        atomicMax(amax, __float_as_uint(b));
    }
}

// partial[b] = sum over block b's grid-stride share of E[i] F[i], in fp64 (fixed order; the host adds the
// kPairBlocks partials in order)
constexpr int kPairBlocks = 64;
__global__ void __launch_bounds__(256) k_pair_dot(const float* __restrict__ E, const float* __restrict__ F, int n,
                                                 double* __restrict__ partial) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += kPairBlocks * 256) s = fma(double(E[i]), double(F[i]), s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// split-K slice count for an M x N x K product: about 320 workgroups, whole 32-deep steps (160 / 640
// measured the same within the box spread: profiles/r04/dot32_split_ab_r04be.txt)
int splits_for(int M, int N, int K) {
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    int s = std::max(1, std::min(320 / tiles, (K + 4 * BK - 1) / (4 * BK)));   // >= 4 steps per slice
    return s;
}

template <bool TA, bool TB, class EA, class EB>
void launch(hipStream_t st, int M, int N, int K, int splits, const EA* A, size_t lda, const EB* B, size_t ldb,
            const unsigned* sa, const unsigned* sb, float* C, unsigned* zw) {
    XRS_REQUIRE(M > 0 && N > 0 && K > 0, "empty product");
    int kps = (K + splits - 1) / splits;
    kps = (kps + BK - 1) / BK * BK;
    splits = (K + kps - 1) / kps;
    const unsigned tiles = unsigned((M + BM - 1) / BM) * unsigned((N + BN - 1) / BN);
    hipLaunchKernelGGL((k_gemm32<TA, TB, EA, EB>), dim3(tiles, 1, splits), dim3(NT), 0, st, M, N, K, kps, A, lda, B, ldb,
                       sa, sb, C, zw);
    check_launch("k_gemm32");
}

int kps_splits(int K, int splits) {
    int kps = (K + splits - 1) / splits;
    kps = (kps + BK - 1) / BK * BK;
    return (K + kps - 1) / kps;
}

void slab_sum(hipStream_t st, const float* slab, int S, int MN, float* E, unsigned* amax) {
    hipLaunchKernelGGL(k_slab_sum_max, dim3((MN + 255) / 256), dim3(256), 0, st, slab, S, MN, E, amax);
    check_launch("k_slab_sum_max");
}

// device buffers of one zipper: fp32 environments E (left) / F (right), ping-pong per end; T and split-K slabs
// per end; W = the closing sum's partials + the max words (left 0..d, right d+1..2d+1; each word read is
// zeroed by the product launch before its slab sum: no memset)
struct Dot32Bufs {
    float *E0, *E1, *F0, *F1, *TL, *TR, *SL, *SR;
    char* W;
    size_t wbytes;
};

size_t dot32_layout(size_t d, const size_t* n, const size_t* rx, const size_t* ry, size_t off[10]) {
    size_t emax = 1, tmax = 1, smax = 1;
    for (size_t k = 0; k <= d; ++k) emax = std::max(emax, rx[k] * ry[k]);
    for (size_t k = 0; k < d; ++k) {
        tmax = std::max(tmax, std::max(ry[k] * n[k] * rx[k + 1], rx[k] * n[k] * ry[k + 1]));
        const int a2 = int(rx[k + 1]), b2 = int(ry[k + 1]), a = int(rx[k]), b = int(ry[k]);
        smax = std::max(smax, size_t(kps_splits(int(ry[k] * n[k]), splits_for(a2, b2, int(ry[k] * n[k])))) * a2 * b2);
        smax = std::max(smax, size_t(kps_splits(int(n[k] * ry[k + 1]), splits_for(a, b, int(n[k] * ry[k + 1])))) * a * b);
    }
    auto up = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t sz[9] = {emax * 4, emax * 4, emax * 4, emax * 4, tmax * 4, tmax * 4, smax * 4, smax * 4,
                          8 * kPairBlocks + 4 * (2 * d + 2)};
    size_t o = 0;
    for (int i = 0; i < 9; ++i) {
        off[i] = o;
        o += up(sz[i]);
    }
    off[9] = sz[8];
    return o;
}

Dot32Bufs dot32_bufs(char* base, const size_t off[10]) {
    auto f = [&](int i) { return reinterpret_cast<float*>(base + off[i]); };
    return Dot32Bufs{f(0), f(1), f(2), f(3), f(4), f(5), f(6), f(7), base + off[8], off[9]};
}

// enqueues the zipper on h->stream (+ its side stream 0) up to the closing partial sums in b.W
void dot32_enqueue(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                   const double* const* Y, const Dot32Bufs& bf) {
    const size_t m = d / 2;
    float *E = bf.E0, *En = bf.E1, *F = bf.F0, *Fn = bf.F1;
    double* res = reinterpret_cast<double*>(bf.W);
    unsigned* amax = reinterpret_cast<unsigned*>(bf.W + 8 * kPairBlocks);
    unsigned* wr = amax + (d + 1);
    {
        StreamFork fork(h);
        // left end (cores 0..m-1) on the side stream, right end (cores d-1..m) on the main stream; launches
        // interleaved step by step so that both streams have work from the start (the host's enqueue rate,
        // not the GPU, paces a chain of small launches)
        for (size_t s = 0; s < std::max(m, d - m); ++s) {
            if (s < m) {
                fork.side();
                const size_t k = s;
                const int a = int(rx[k]), b = int(ry[k]), nk = int(n[k]), a2 = int(rx[k + 1]), b2 = int(ry[k + 1]);
                const int K2 = b * nk, S = splits_for(a2, b2, K2), Sr = kps_splits(K2, S);
                if (k == 0) {   // E_0 = [1]: T = X_0 exactly
                    launch<true, false, double, double>(h->stream, a2, b2, K2, S, X[0], size_t(a2), Y[0], size_t(b2),
                                                        nullptr, nullptr, bf.SL, amax + 1);
                } else {
                    // T (b x nk a2) = 2^-e E^T X_k
                    launch<true, false, float, double>(h->stream, b, nk * a2, a, 1, E, size_t(b), X[k], size_t(nk) * a2,
                                                       amax + k, nullptr, bf.TL, nullptr);
                    // E' (a2 x b2) = T^T ((b nk) x a2)^T Y_k ((b nk) x b2)
                    launch<true, false, float, double>(h->stream, a2, b2, K2, S, bf.TL, size_t(a2), Y[k],
                                                       size_t(b2), nullptr, nullptr, bf.SL, amax + k + 1);
                }
                slab_sum(h->stream, bf.SL, Sr, a2 * b2, En, amax + k + 1);
                std::swap(E, En);
            }
            if (s < d - m) {
                fork.main();
                const size_t k = d - 1 - s;
                const int a = int(rx[k]), b = int(ry[k]), nk = int(n[k]), a2 = int(rx[k + 1]), b2 = int(ry[k + 1]);
                const int K2 = nk * b2, S = splits_for(a, b, K2), Sr = kps_splits(K2, S);
                if (s == 0) {   // F_d = [1]: T = X_{d-1} exactly
                    launch<false, true, double, double>(h->stream, a, b, K2, S, X[k], size_t(K2), Y[k], size_t(K2), nullptr,
                                                        nullptr, bf.SR, wr + k);
                } else {
                    // T (a nk x b2) = X_k (a nk x a2) 2^-e F
                    launch<false, false, double, float>(h->stream, a * nk, b2, a2, 1, X[k], size_t(a2), F, size_t(b2),
                                                        nullptr, wr + k + 1, bf.TR, nullptr);
                    // F' (a x b) = T (a x nk b2) Y_k^T
                    launch<false, true, float, double>(h->stream, a, b, K2, S, bf.TR, size_t(K2), Y[k],
                                                       size_t(K2), nullptr, nullptr, bf.SR, wr + k);
                }
                slab_sum(h->stream, bf.SR, Sr, a * b, Fn, wr + k);
                std::swap(F, Fn);
            }
        }
        fork.join();
    }
    hipLaunchKernelGGL(k_pair_dot, dim3(kPairBlocks), dim3(256), 0, h->stream, E, F, int(rx[m] * ry[m]), res);
    check_launch("k_pair_dot");
    hipLaunchKernelGGL(k_pair_dot, dim3(kPairBlocks), dim3(256), 0, h->stream, E, F, int(rx[m] * ry[m]), res);
    check_launch("k_pair_dot");
}

}  // namespace

double dot_f32(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
               const double* const* Y) {
    XRS_REQUIRE(d >= 2 && d <= 4096, "the fp32 zipper takes 2..4096 components");
    for (size_t k = 0; k <= d; ++k)
        XRS_REQUIRE(rx[k] * ry[k] < (size_t(1) << 31) && (k == d || n[k] * rx[k] * rx[k + 1] < (size_t(1) << 31)),
                    "fp32 zipper: sizes must fit 32-bit indices");
    const size_t m = d / 2;
    size_t off[10];
    DevBuf mem(h, dot32_layout(d, n, rx, ry, off));
    const Dot32Bufs b = dot32_bufs(mem.as<char>(), off);
    // (a hipGraph replay of these launches measured slower, 0.49 vs 0.26 ms at the bench shape: the replay
    // ran both ends' kernels on one stream)
    dot32_enqueue(h, d, n, rx, X, ry, Y, b);
    // read back the closing sum and the max words; the exponents the GEMMs scaled by are added back here
    char* hs = static_cast<char*>(h->host_scratch);
    XRS_HIP(hipMemcpyAsync(hs, b.W, b.wbytes, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    double v = 0.0;
    for (int blk = 0; blk < kPairBlocks; ++blk) {
        double p;
        std::memcpy(&p, hs + 8 * blk, 8);
        v += p;
    }
    const unsigned* hw = reinterpret_cast<const unsigned*>(hs + 8 * kPairBlocks);
    auto expo = [](unsigned bits) { return bits == 0u ? 0 : int((bits >> 23) & 0xff) - 126; };
    int e = 0;
    for (size_t k = 1; k < m; ++k) e += expo(hw[k]);                  // left GEMMs of cores 1..m-1 read E_k
    for (size_t k = m + 1; k < d; ++k) e += expo(hw[d + 1 + k]);      // right GEMMs of cores d-2..m read F_{k}
    return std::ldexp(v, e);
}

}  // namespace xrs

extern "C" {

int xrs_tt_dot_f32(xrs_handle_t h, double* result, size_t d, const size_t* n, const size_t* rx, const double* const* X,
                   const size_t* ry, const double* const* Y) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h && result && n && rx && ry && X && Y, "null argument");
        XRS_REQUIRE(rx[0] == 1 && ry[0] == 1 && rx[d] == 1 && ry[d] == 1, "boundary ranks must be 1");
        for (size_t k = 0; k < d; ++k) XRS_REQUIRE(X[k] && Y[k] && n[k] > 0 && rx[k + 1] > 0 && ry[k + 1] > 0, "bad TT");
        xrs::fence_readers(h);
        *result = xrs::dot_f32(h, d, n, rx, X, ry, Y);
    });
}

}  // extern "C"
