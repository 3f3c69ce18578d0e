// fp32 GEMM on the CDNA4 fp32 matrix cores: C = alpha op(A) op(B), fp32 result, row-major (ldc = N).
// The reduced-precision form of blasWrapper::matrix_matrix_product (blasLapackWrapper.cpp:149-195, whose
// cblas_dgemm at :177-191 is fp64): the north star's "dense contraction on MFMA fp32 tiles".
//
// Included by one translation unit per operand-type pair (sgemm_ff / sgemm_fd / sgemm_df / sgemm_dd.hip),
// so the four kernel families compile in parallel.
//
// Kernel (k_sgemm): BM x BN output tile, 32-deep K-steps, WGM x WGN x WGK waves; each wave owns a
// (BM/WGM) x (BN/WGN) tile of v_mfma_f32_16x16x4_f32 blocks (32-cycle issue, 40-cycle accumulator latency:
// every wave tile holds >= 2 independent accumulators); WGK wave groups take alternate 16-deep chunks of
// every K-step and are summed through LDS at the end.
//  - Staging: 16-B vector loads per lane (4 floats / 2 doubles; scalar loads when a shape or alignment
//    does not allow them), a 2-slot register ring (the loads of K-step t+2 are in flight while step t
//    computes), fp64 rounded to fp32 and optional power-of-two scales applied as the registers are written
//    to the LDS double buffer. Loads use clamped addresses and no branches, so the waitcnt pass keeps the
//    ring in flight across steps; out-of-range elements are written as zeros.
//  - LDS image of an operand tile: element (k, r) at k P + (r ^ swz(k)), P = rows rounded up to 32 floats,
//    one image layout for both operands and both storage orders (transposed sources are transposed by the
//    staging writes). swz permutes 4-float chunks inside 32-float blocks:
//      bit 4 = bit 2 of k: the fragment reads (ds_read_b32; each 32-lane group reads rows k and k+4 of a
//        16-deep chunk, 16 consecutive r each) hit opposite 16-bank halves;
//      bits 2, 3 = bits 3, 4 of k: the transposed staging writes of a k-contiguous source (8 vectors of
//        4 k x 4 rows per 32-lane group) hit 8 distinct 4-bank slots;
//      row-contiguous staging writes (16 or 8 B per lane along r) keep every vector whole and aligned.
//  - MFMA k order: within a 16-deep chunk, lane group g = lane >> 4 of MFMA j takes k = 4 g + j (A and B
//    alike), so a lane's four k of one chunk are one ds_read offset pattern.
//  - Split-K (grid.z) for grids that cannot fill 256 CUs: the slices store their partial tiles in the
//    accumulator layout with 16-B write-through (sc1) buffer stores, draw an arrival ticket, and the last slice
//    of a tile sums all slabs in a fixed order with 16-B sc1 loads (deterministic), applies alpha and writes C
//    (MI355X_MICROARCH.md, hand-off table row 1: sc1 stores, agent-scope ticket, sc1 loads).
//  - Optional max|C| (atomicMax on the float bits) and power-of-two operand scales from such words, and
//    per-workgroup max|.| slots of fp64 operands: the fp32 TT zipper's range control (dot32.hip, sgemm.hpp).
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include <hip/hip_ext.h>

#include "sgemm.hpp"

#ifdef XRS_SG_STAMPS
// Diagnostic build only (tools/sgemm_stamps.py): thread 0 of every workgroup writes s_memtime at the kernel's
// phase boundaries to g_sg_stamps[8 wg + i]: 0 start, 1 prologue done, 2 main loop done, 3 epilogue / ticket
// done, 4 end (the last slice: after the combine); [7] = XCC id << 32 | HW id.
__device__ unsigned long long* g_sg_stamps = nullptr;
#define XRS_SG_STAMP(i)                                                                                      \
    if (threadIdx.x == 0 && g_sg_stamps != nullptr) {                                                       \
        const size_t wg_ = blockIdx.x + size_t(gridDim.x) * blockIdx.z;                                     \
        g_sg_stamps[8 * wg_ + (i)] = __builtin_amdgcn_s_memtime();                                          \
        if ((i) == 0)                                                                                        \
            g_sg_stamps[8 * wg_ + 7] = (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) | \
                                       __builtin_amdgcn_s_getreg((31 << 11) | 4);                            \
    }
#else
#define XRS_SG_STAMP(i)
#endif

namespace xrs {
namespace sg {
namespace {   // (internal linkage: one copy per instantiating translation unit)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef double d2 __attribute__((ext_vector_type(2)));

// LDS image of an operand tile: R rows x BK k
template <int R, int BK>
struct Img {
    static constexpr int P = (R + 31) / 32 * 32;
    static constexpr int FLOATS = P * BK;
    __device__ static int swz(int k) { return (((k >> 2) & 1) << 4) | (((k >> 3) & 1) << 2) | (((k >> 4) & 1) << 3); }
    __device__ static int at(int k, int r) { return k * P + (r ^ swz(k)); }
};

template <class E, int V> struct VecT;
template <> struct VecT<float, 4> { using T = f4; };
template <> struct VecT<float, 1> { using T = float; };
template <> struct VecT<double, 2> { using T = d2; };
template <> struct VecT<double, 1> { using T = double; };

// 2^-(e) with max|.| 2^-e in [0.5, 1) for a max word (float bits); 1 for a zero word. The exponent is
// clamped to the normal range (a non-finite max gives the smallest scale; its result is non-finite anyway).
__device__ __forceinline__ float pow2_scale(unsigned bits) {
    if (bits == 0u) return 1.0f;
    const int ef = int((bits >> 23) & 0xff);
    const int be = min(max(253 - ef, 1), 254);
    return __uint_as_float(unsigned(be) << 23);
}

// Staging of one operand tile: R rows x BK k per K-step. KMAJ: element (k, r) at src[k ld + r] (rows
// contiguous), else src[r ld + k] (k contiguous). VEC: 16-B vectors along the contiguous index.
// WHOLE: the tile lies inside the matrix and every K-step is whole (the host checks M % BM, N % BN, K % BK and
// 32-bit tile offsets): per-thread offsets are computed once, a load is one global load from the step's
// (wave-uniform) base plus a 32-bit lane offset, a store one ds_write per vector (no masks, no clamps).
// Otherwise (edge tiles, ragged K) coordinates are clamped to valid addresses and out-of-range elements are
// written as zeros.
// vmax: running max|x| of the fp64 values converted (the fp32 zipper's range check, sgemm.hpp).
template <class E, bool KMAJ, bool VEC, int R, int BK, int NT, bool WHOLE>
struct Stager {
    static constexpr int V = VEC ? int(16 / sizeof(E)) : 1;
    using T = typename VecT<E, V>::T;
    static constexpr int NVEC = R * BK / V;
    static constexpr int PER = (NVEC + NT - 1) / NT;
    static_assert(!KMAJ || R % V == 0, "row vectors must tile the rows");
    static_assert(!WHOLE || VEC, "whole tiles use vector staging");
    T v[PER];

    // vector e of this thread -> (k, r) of its first element; threads past the tile repeat the last vector
    // (identical values to identical LDS addresses: no guard, no branch)
    __device__ static void coord(int e, int& k, int& r) {
        const int q = min(int(threadIdx.x) + e * NT, NVEC - 1);
        if constexpr (KMAJ) {
            k = q / (R / V);
            r = (q % (R / V)) * V;
        } else {
            r = q / (BK / V);
            k = (q % (BK / V)) * V;
        }
    }
    // WHOLE: byte offsets of the vectors from the tile's step base, LDS offsets (floats) in a stage image
    unsigned goff[WHOLE ? PER : 1];
    int loff[WHOLE ? PER : 1];
    template <class IMG>
    __device__ void init(size_t ld) {
        if constexpr (WHOLE) {
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                int k, r;
                coord(e, k, r);
                goff[e] = unsigned((KMAJ ? size_t(k) * ld + size_t(r) : size_t(r) * ld + size_t(k)) * sizeof(E));
                loff[e] = IMG::at(k, r);
            }
        }
    }
    // WHOLE: the step's tile base (uniform); else clamped, always valid addresses (vector mode: rtot % V == 0
    // for KMAJ, kend % V == 0 otherwise)
    __device__ void load(const E* __restrict__ src, size_t ld, int r0, int rtot, int k0, int kend) {
        if constexpr (WHOLE) {
            const char* base = reinterpret_cast<const char*>(KMAJ ? src + size_t(k0) * ld + size_t(r0)
                                                                  : src + size_t(r0) * ld + size_t(k0));
#pragma unroll
            for (int e = 0; e < PER; ++e) v[e] = *reinterpret_cast<const T*>(base + goff[e]);
        } else {
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                int k, r;
                coord(e, k, r);
                int gk, gr;
                if constexpr (KMAJ) {
                    gk = min(k0 + k, kend - 1);
                    gr = min(r0 + r, rtot - V);
                } else {
                    gk = min(k0 + k, kend - V);
                    gr = min(r0 + r, rtot - 1);
                }
                const E* p = KMAJ ? src + size_t(gk) * ld + size_t(gr) : src + size_t(gr) * ld + size_t(gk);
                v[e] = *reinterpret_cast<const T*>(p);
            }
        }
    }
    template <class IMG, bool SC>
    __device__ void store(float* __restrict__ img, int r0, int rtot, int k0, int kend, float s, E& vmax) const {
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            int k = 0, r = 0;
            if constexpr (!WHOLE) coord(e, k, r);
            const bool ok = WHOLE || ((k0 + k < kend) && (r0 + r < rtot));
            float f[V];
#pragma unroll
            for (int j = 0; j < V; ++j) {
                E x;
                if constexpr (V == 1) x = v[e];
                else x = v[e][j];
                if constexpr (std::is_same<E, double>::value) vmax = fmax(vmax, fabs(x));
                float y = float(x);
                if constexpr (SC) y *= s;
                f[j] = WHOLE ? y : (ok ? y : 0.0f);
            }
            const int lo = WHOLE ? loff[e] : IMG::at(k, r);
            if constexpr (KMAJ) {
                if constexpr (V == 4) *reinterpret_cast<f4*>(img + lo) = f4{f[0], f[1], f[2], f[3]};
                else if constexpr (V == 2) *reinterpret_cast<f2*>(img + lo) = f2{f[0], f[1]};
                else img[lo] = f[0];
            } else {
                // (k .. k+V-1 share swz(k): V <= 4 and k % V == 0)
#pragma unroll
                for (int j = 0; j < V; ++j) img[lo + j * IMG::P] = f[j];
            }
        }
    }
};

struct Args {
    const void* A;
    size_t lda;
    const void* B;
    size_t ldb;
    float* C;
    int M, N, K, kps;
    float alpha;
    const unsigned* sa;
    const unsigned* sb;
    unsigned* amax;
    unsigned* cmax_a;   // per-workgroup max|A| / max|B| slots of fp64 operands (kCmaxSlots words each)
    unsigned* cmax_b;
    float* slab;
    unsigned slab_bytes;
    int* tickets;
    int tiles_m;
    int xcd;   // 1: tiles sharing a B column panel on one XCD, 2: sharing an A row panel, 0: column-major
};

// an fp64 max|.| as a float for the max slots: above FLT_MAX -> inf, a nonzero max below the fp32 range -> the
// smallest denormal (so that the check sees it as out of range, not as a zero core)
__device__ __forceinline__ float fp64_max_as_float(double m) {
    const float f = float(m);
    return (m > 0.0 && f == 0.0f) ? __uint_as_float(1u) : f;
}

__device__ __forceinline__ void wave_max_atomic(unsigned* w, float m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(w, __float_as_uint(m));
}

// value of a max word: the maximum of its kMaxLanes lanes (wave-uniform loads)
__device__ __forceinline__ unsigned max_word(const unsigned* __restrict__ w) {
    unsigned m = 0u;
#pragma unroll
    for (int i = 0; i < kMaxLanes; ++i) m = max(m, w[i]);
    return m;
}

// workgroup max of m (every thread of the workgroup calls it; `red` holds >= 16 words of LDS that are free)
// into lane (workgroup id % kMaxLanes) of the max word w
__device__ __forceinline__ void block_max_atomic(unsigned* w, float m, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int nw = int(blockDim.x) >> 6;
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = 0.0f;
        for (int i = 0; i < nw; ++i) b = fmaxf(b, red[i]);
        atomicMax(w + (blockIdx.x + gridDim.x * blockIdx.z) % kMaxLanes, __float_as_uint(b));
    }
}

// Main loop: step t computes LDS buffer t % 2, then writes step t+1 (register slot (t+1) % PD) into the other
// buffer and issues the loads of step t+PD into slot t % PD; one barrier per step. PD = 4 keeps twice the
// bytes in flight of PD = 2: short-K slices (the environment products' 10 steps) are load-latency bound. (A 3-stage LDS ring whose last chunk read
// the next step's first fragments ahead of the barrier measured slower on every shape: DESIGN.md §3.6.)
// OCC: minimum waves per SIMD (the second __launch_bounds__ argument): 4 caps the registers at 128 per lane so that two
// 8-wave workgroups share a CU (the concurrent zipper ends: cfg 13; the 64x80 / 80x64 forms 14 / 15 spill at 128)
template <int BM, int BN, int WGM, int WGN, int WGK, int BK, int PD, int ST, bool TA, bool TB, class EA, class EB, int MODE,
          int OCC = 1>
__global__ void __launch_bounds__(WGM * WGN * WGK * 64, OCC) k_sgemm(const Args p) {
    static_assert(ST == 2 || ST == 3, "2 or 3 LDS stages");
    constexpr bool VEC = MODE >= 1, WHOLE = MODE == 2;
    // fp32-only products carry no operand scales (the fp32 zipper's mixed products always do)
    constexpr bool SC = !(std::is_same<EA, float>::value && std::is_same<EB, float>::value);
    constexpr int NT = WGM * WGN * WGK * 64;
    using IA = Img<BM, BK>;
    using IB = Img<BN, BK>;
    constexpr int STAGE = IA::FLOATS + IB::FLOATS;
    __shared__ float lds[ST * STAGE];   // the one LDS array (stages; the epilogue reuses it)
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int TM = WM / 16, TN = WN / 16;
    static_assert(WM % 16 == 0 && WN % 16 == 0 && TM * TN >= 2, "wave tile: >= 2 whole 16x16 blocks");
    constexpr int NQ = BK / 16;
    static_assert(NQ % WGK == 0, "chunks split evenly over the wave groups");
    constexpr int NQW = NQ / WGK;   // chunks per wave per step
    static_assert(WGK == 1 || (WGK - 1) * WGM * WGN * TM * TN * 256 <= ST * STAGE, "LDS reduction buffer");
    using SA = Stager<EA, TA, VEC, BM, BK, NT, WHOLE>;    // op(A) = A^T: A stored K x M (rows contiguous)
    using SB = Stager<EB, !TB, VEC, BN, BK, NT, WHOLE>;   // op(B) = B: B stored K x N (rows contiguous)
    const EA* __restrict__ A = static_cast<const EA*>(p.A);
    const EB* __restrict__ B = static_cast<const EB*>(p.B);

    // tile bx and split-K slice bz: xcd 3 (split-K grids whose slice count is a multiple of 8) deals whole
    // slices to the XCDs (workgroups go to the 8 XCDs round-robin by dispatch order): a slice's operand
    // panels are fetched into one XCD's L2 instead of all eight
    int bx = int(blockIdx.x), bz = int(blockIdx.z);
    if (p.xcd == 3) {
        const int X = int(gridDim.x), L = bx + X * bz, c = L & 7, q = L >> 3;
        bz = c + 8 * (q / X);
        bx = q % X;
    }
    int tm, tn;
    {
        const int b = bx, tiles_n = int(gridDim.x) / p.tiles_m;
        if (p.xcd == 1) {
            const int xcd = b & 7, slot = b >> 3;
            tn = (slot / p.tiles_m) * 8 + xcd;
            tm = slot % p.tiles_m;
        } else if (p.xcd == 2) {
            const int xcd = b & 7, slot = b >> 3;
            tm = (slot / tiles_n) * 8 + xcd;
            tn = slot % tiles_n;
        } else {
            tm = b % p.tiles_m;
            tn = b / p.tiles_m;
        }
    }
    XRS_SG_STAMP(0)
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = bz * p.kps, kend = min(p.K, kbeg + p.kps);
    const int nsteps = (kend - kbeg + BK - 1) / BK;   // >= 1: the host launches non-empty slices only
    const float fa = p.sa ? pow2_scale(max_word(p.sa)) : 1.0f, fb = p.sb ? pow2_scale(max_word(p.sb)) : 1.0f;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kg = wave / (WGM * WGN), pos = wave % (WGM * WGN);
    const int wm = (pos / WGN) * WM, wn = (pos % WGN) * WN;
    const int lr = lane & 15, lg = lane >> 4;

    f4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    static_assert(PD == 2 || PD == 4, "register ring of 2 or 4 K-steps");
    SA ra[PD];
    SB rb[PD];
    EA vmax_a = 0;
    EB vmax_b = 0;
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        ra[u].template init<IA>(p.lda);
        rb[u].template init<IB>(p.ldb);
    }
    auto load = [&](auto slot_c, int t) {
        constexpr int s = decltype(slot_c)::value;
        if constexpr (WHOLE) t = min(t, nsteps - 1);   // (the ring's loads past the slice re-read its last step)
        ra[s].load(A, p.lda, m0, p.M, kbeg + t * BK, kend);
        rb[s].load(B, p.ldb, n0, p.N, kbeg + t * BK, kend);
    };
    auto store = [&](auto slot_c, int buf, int t) {   // register slot s -> LDS buffer buf
        constexpr int s = decltype(slot_c)::value;
        ra[s].template store<IA, SC>(lds + buf * STAGE, m0, p.M, kbeg + t * BK, kend, fa, vmax_a);
        rb[s].template store<IB, SC>(lds + buf * STAGE + IA::FLOATS, n0, p.N, kbeg + t * BK, kend, fb, vmax_b);
    };
    // fragments of one chunk, double-buffered in registers
    float fa_[2][TM][4], fb_[2][TN][4];
    auto frag = [&](auto slot_c, int buf, int qq) {
        constexpr int s = decltype(slot_c)::value;
        const float* as = lds + buf * STAGE;
        const float* bs = as + IA::FLOATS;
        const int q = qq * WGK + kg;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 16 * q + 4 * lg + j;
#pragma unroll
            for (int i = 0; i < TM; ++i) fa_[s][i][j] = as[IA::at(k, wm + 16 * i + lr)];
#pragma unroll
            for (int i = 0; i < TN; ++i) fb_[s][i][j] = bs[IB::at(k, wn + 16 * i + lr)];
        }
    };
    auto mfma = [&](auto slot_c) {
        constexpr int s = decltype(slot_c)::value;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int jj = 0; jj < TN; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa_[s][i][j], fb_[s][jj][j], acc[i][jj], 0, 0, 0);
    };
    // compute LDS buffer `buf`: the reads of chunk q+1 are issued ahead of chunk q's MFMAs
    auto compute = [&](int buf) {
        frag(std::integral_constant<int, 0>{}, buf, 0);
        [&]<int... Q>(std::integer_sequence<int, Q...>) {
            (([&] {
                 constexpr int cur = Q & 1, nxt = (Q + 1) & 1;
                 if constexpr (Q + 1 < NQW) frag(std::integral_constant<int, nxt>{}, buf, Q + 1);
                 __builtin_amdgcn_sched_barrier(0);   // keep those reads ahead of this chunk's MFMAs
                 mfma(std::integral_constant<int, cur>{});
             }()),
             ...);
        }(std::make_integer_sequence<int, NQW>{});
    };
    // ST = 3: chunk 0 of step t is already in fragment set S0 (read during step t-1); the last chunk's MFMAs
    // run beside the reads of step t+1's chunk 0 from buffer `nbuf` (complete since the barrier that ended step
    // t-1), so no barrier sits between a wave's fragment reads and its MFMAs
    auto compute3 = [&](auto s0_c, int buf, int nbuf) {
        constexpr int S0 = decltype(s0_c)::value;
        [&]<int... Q>(std::integer_sequence<int, Q...>) {
            (([&] {
                 constexpr int cur = (S0 + Q) & 1, nxt = (S0 + Q + 1) & 1;
                 if constexpr (Q + 1 < NQW) frag(std::integral_constant<int, nxt>{}, buf, Q + 1);
                 else frag(std::integral_constant<int, nxt>{}, nbuf, 0);
                 __builtin_amdgcn_sched_barrier(0);
                 mfma(std::integral_constant<int, cur>{});
             }()),
             ...);
        }(std::make_integer_sequence<int, NQW>{});
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;

    if constexpr (ST == 3) {
        // register slot (t+2) % PD holds K-step t+2 at the start of step t (its loads issued PD steps before its
        // store); LDS buffer t % 3 holds step t: step t writes step t+2 into buffer (t+2) % 3, last read in step
        // t-1, before the barrier that ends it
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (load(std::integral_constant<int, U>{}, U), ...);
        }(std::make_integer_sequence<int, PD>{});
        store(I0{}, 0, 0);
        store(I1{}, 1, 1);
        load(I0{}, PD);
        load(I1{}, PD + 1);
        __syncthreads();
        XRS_SG_STAMP(1)
        frag(I0{}, 0, 0);
        int t0 = 0, b0 = 0;   // b0 = t0 % 3
        for (; t0 + PD <= nsteps; t0 += PD) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (([&] {
                     const int t = t0 + U;
                     const int bc = (b0 + U) % 3, bn = (b0 + U + 1) % 3, bs = (b0 + U + 2) % 3;
                     compute3(std::integral_constant<int, (U * NQW) & 1>{}, bc, bn);
                     store(std::integral_constant<int, (U + 2) % PD>{}, bs, t + 2);
                     load(std::integral_constant<int, (U + 2) % PD>{}, t + 2 + PD);
                     __syncthreads();
                 }()),
                 ...);
            }(std::make_integer_sequence<int, PD>{});
            b0 = (b0 + PD) % 3;
        }
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (([&] {
                 const int t = t0 + U;
                 if (t < nsteps) {
                     const int bc = (b0 + U) % 3, bn = (b0 + U + 1) % 3, bs = (b0 + U + 2) % 3;
                     compute3(std::integral_constant<int, (U * NQW) & 1>{}, bc, bn);
                     if (t + 2 < nsteps) store(std::integral_constant<int, (U + 2) % PD>{}, bs, t + 2);
                     __syncthreads();
                 }
             }()),
             ...);
        }(std::make_integer_sequence<int, PD>{});
    } else {
        // ring: register slot t % PD holds K-step t (its loads issued PD steps ahead), LDS buffer t % 2
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (load(std::integral_constant<int, U>{}, U), ...);
        }(std::make_integer_sequence<int, PD>{});
        store(I0{}, 0, 0);
        __syncthreads();
        XRS_SG_STAMP(1)
        int t0 = 0;
        // steady state, no guards: the loads of steps past the slice re-read valid addresses and their stores
        // go to the idle buffer
        for (; t0 + PD <= nsteps; t0 += PD) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (([&] {
                     const int t = t0 + U;
                     compute(U & 1);
                     store(std::integral_constant<int, (U + 1) % PD>{}, (U + 1) & 1, t + 1);
                     load(std::integral_constant<int, U>{}, t + PD);
                     __syncthreads();
                 }()),
                 ...);
            }(std::make_integer_sequence<int, PD>{});
        }
        // tail: fewer than PD steps left (no loads: they were issued by the steady state or the prologue)
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (([&] {
                 const int t = t0 + U;
                 if (t < nsteps) {
                     compute(U & 1);
                     if (t + 1 < nsteps) store(std::integral_constant<int, (U + 1) % PD>{}, (U + 1) & 1, t + 1);
                     __syncthreads();
                 }
             }()),
             ...);
        }(std::make_integer_sequence<int, PD>{});
    }

    XRS_SG_STAMP(2)
    // max|.| of the fp64 operands into this workgroup's slot (no single hot word: kCmaxSlots slots per launch)
    {
        const unsigned slot = (blockIdx.x + gridDim.x * blockIdx.z) % unsigned(kCmaxSlots);
        if constexpr (std::is_same<EA, double>::value)
            if (p.cmax_a != nullptr) wave_max_atomic(p.cmax_a + slot, fp64_max_as_float(vmax_a));
        if constexpr (std::is_same<EB, double>::value)
            if (p.cmax_b != nullptr) wave_max_atomic(p.cmax_b + slot, fp64_max_as_float(vmax_b));
    }
    __syncthreads();   // LDS free for the reduction
    if constexpr (WGK > 1) {
        float* red = lds;
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        red[((((kg - 1) * (WGM * WGN) + pos) * TM * TN + i * TN + j) * 4 + r) * 64 + lane] = acc[i][j][r];
        }
        __syncthreads();
        if (kg == 0)
#pragma unroll
            for (int g = 1; g < WGK; ++g)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            acc[i][j][r] += red[((((g - 1) * (WGM * WGN) + pos) * TM * TN + i * TN + j) * 4 + r) * 64 + lane];
    }
    // C/D map of the f32 16x16x4 form: col = lane & 15, row = 4 (lane >> 4) + reg
    const int lc = lane & 15, lq = lane >> 4;
    const int M = p.M, N = p.N;
    if (p.slab == nullptr) {
        float mx = 0.0f;
        if (kg == 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = n0 + wn + 16 * j + lc;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = m0 + wm + 16 * i + 4 * lq + r;
                        if (row < M && col < N) {
                            const float v = p.alpha * acc[i][j][r];
                            p.C[size_t(row) * N + col] = v;
                            mx = fmaxf(mx, fabsf(v));
                        }
                    }
                }
        }
        if (p.amax != nullptr) {
            __syncthreads();   // (the K-group reduction above read the LDS)
            block_max_atomic(p.amax, mx, lds);
        }
        XRS_SG_STAMP(3)
        return;
    }
    // ---- split-K: this slice's partial tile in the accumulator layout -- the float4 of block (i, j) of lane l
    // of the wave at position pos at ((pos TM + i) TN + j) 64 + l, so one wave instruction writes 1 KB
    // contiguously -- at slab + (z tiles + x) BM BN for slice z of tile x; 16-B write-through (sc1) buffer
    // stores, drained before the ticket (MI355X_MICROARCH.md, hand-off table row 1)
    static_assert(WGM * WGN * TM * TN * 256 == BM * BN, "accumulator layout covers the tile");
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.slab, 0, int(p.slab_bytes), 0x00020000);
    auto soff = [&](int z, int i, int j) {
        return int(((size_t(z) * gridDim.x + bx) * (BM * BN) + size_t(((pos * TM + i) * TN + j) * 64 + lane) * 4) * 4);
    };
    if (kg == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) __builtin_amdgcn_raw_buffer_store_b128(acc[i][j], rs, soff(bz, i, j), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float* flag = lds;   // the one LDS array (no second __shared__ object)
    if (tid == 0) {
        const int tk = __hip_atomic_fetch_add(&p.tickets[bx], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = (tk == int(gridDim.z) - 1);
        if (last) __hip_atomic_store(&p.tickets[bx], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = last ? 1.0f : 0.0f;
    }
    __syncthreads();
    XRS_SG_STAMP(3)
    if (flag[0] == 0.0f) return;
    __syncthreads();   // (every thread has read the flag before the LDS is reused below)
    // last slice: wave group g sums the slabs z = g, g + WGK, ... in slice order (16-B sc1 loads, U slabs per
    // round trip), then the groups' sums are added in group order through the LDS: a fixed order, so the
    // result is the same bits whichever slice arrives last
    const int S = int(gridDim.z);
    constexpr int U = (32 / (TM * TN)) < 1 ? 1 : ((32 / (TM * TN)) > 8 ? 8 : (32 / (TM * TN)));
    f4 sum[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) sum[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    for (int z0 = kg; z0 < S; z0 += U * WGK) {
        f4 v[U][TM][TN];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int z = min(z0 + u * WGK, S - 1);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) v[u][i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, soff(z, i, j), 0, 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float keep = (z0 + u * WGK < S) ? 1.0f : 0.0f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) sum[i][j] += keep * v[u][i][j];
        }
    }
    if constexpr (WGK > 1) {
        float* red = lds;
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        red[((((kg - 1) * (WGM * WGN) + pos) * TM * TN + i * TN + j) * 4 + r) * 64 + lane] = sum[i][j][r];
        }
        __syncthreads();
        if (kg == 0)
#pragma unroll
            for (int g = 1; g < WGK; ++g)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            sum[i][j][r] += red[((((g - 1) * (WGM * WGN) + pos) * TM * TN + i * TN + j) * 4 + r) * 64 + lane];
    }
    float mx = 0.0f;
    if (kg == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = n0 + wn + 16 * j + lc;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm + 16 * i + 4 * lq + r;
                    if (row < M && col < N) {
                        const float v = p.alpha * sum[i][j][r];
                        p.C[size_t(row) * N + col] = v;
                        mx = fmaxf(mx, fabsf(v));
                    }
                }
            }
    }
    if (p.amax != nullptr) {
        __syncthreads();   // (the group reduction read the LDS)
        block_max_atomic(p.amax, mx, lds);
    }
    XRS_SG_STAMP(4)
}

// ------------------------------------------------------------------------------------------- host side
struct Cfg {
    int bm, bn, bk;
};
// production tiles: 0: 128x128 (8 waves 2x4, wave 64x32, 2-step ring)   1: 64x64 (8 waves 2x2x2: wave 32x32, K-chunks
// over 2 groups)   2: 64x80 (8 waves 4x1x2, wave 16x80)   3: 80x64 (8 waves 1x4x2, wave 80x16)   4: 32x32 (2 waves, wave
// 16x32, 2-step ring); 1-3 with a 4-step register ring. 5-9: forms measured against them (profiles/r05/), for A/B runs
// only (XRS_SGEMM, fp32 operands): 5 64x64 with 64-deep K-steps, 6 / 7 / 9 the 64x64 / 64x80 / 80x64 tiles with a
// 2-step ring, 8 128x128 with 3 LDS stages, 10 / 11 / 12 the 64x64 / 64x80 / 80x64 tiles with 3 LDS stages (the next
// step's first fragments read ahead of the barrier)
constexpr int kNumCfgs = 16;
constexpr Cfg kCfgs[kNumCfgs] = {{128, 128, 32}, {64, 64, 32}, {64, 80, 32}, {80, 64, 32}, {32, 32, 32},
                                 {64, 64, 64},   {64, 64, 32}, {64, 80, 32}, {128, 128, 32}, {80, 64, 32},
                                 {64, 64, 32},   {64, 80, 32}, {80, 64, 32}, {64, 64, 32},   {64, 80, 32},
                                 {80, 64, 32}};

template <int BM, int BN, int WGM, int WGN, int WGK, int BK, int PD, int ST, class EA, class EB, int OCC = 1>
void launch_cfg(xrs_handle_t h, const Args& p, bool ta, bool tb, int mode, int tiles, int splits, double bytes) {
    const dim3 grid(unsigned(tiles), 1u, unsigned(splits));
    KernelTimer timer(h, XRS_KFAM_GEMM, 2.0 * double(p.M) * double(p.N) * double(p.K), bytes, true);
#define XRS_SG(TA_, TB_, MODE_)                                                                                    \
    hipExtLaunchKernelGGL((k_sgemm<BM, BN, WGM, WGN, WGK, BK, PD, ST, TA_, TB_, EA, EB, MODE_, OCC>), grid, dim3(WGM * WGN * WGK * 64), \
                          0, h->stream, timer.start(), timer.stop(), 0, p)
#define XRS_SG_FLAGS(MODE_)                                  \
    if (!ta && !tb) XRS_SG(false, false, MODE_);              \
    else if (!ta && tb) XRS_SG(false, true, MODE_);           \
    else if (ta && !tb) XRS_SG(true, false, MODE_);           \
    else XRS_SG(true, true, MODE_);
    if (mode == 2) { XRS_SG_FLAGS(2) }
    else if (mode == 1) { XRS_SG_FLAGS(1) }
    else { XRS_SG_FLAGS(0) }
#undef XRS_SG_FLAGS
#undef XRS_SG
    check_launch("k_sgemm");
}

// 16-B vector staging is possible for an operand stored with contiguous extent `ext` (rows of a k-major
// operand, or K of a k-contiguous one), leading dimension ld and base pointer ptr
template <class E>
bool vec_ok(const E* ptr, size_t ld, size_t ext) {
    constexpr size_t V = 16 / sizeof(E);
    return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0 && ld % V == 0 && ext % V == 0;
}

}  // namespace
}  // namespace sg

template <class EA, class EB>
void sgemm(xrs_handle_t h, float* C, size_t Ms, size_t Ns, float alpha, const EA* A, size_t lda, bool ta, size_t Ks,
           const EB* B, size_t ldb, bool tb, const SgemmExtra& x) {
    using namespace sg;
    if (Ms == 0 || Ns == 0) return;
    XRS_REQUIRE(Ms < (1u << 30) && Ns < (1u << 30) && Ks < (1u << 30), "GEMM dimension too large");
    if (Ks == 0) {
        XRS_HIP(hipMemsetAsync(C, 0, Ms * Ns * sizeof(float), h->stream));
        return;
    }
    const int M = int(Ms), N = int(Ns), K = int(Ks);
    // staging mode for both operands: 2 whole tiles (below), 1 vectors with edges, 0 scalar loads
    const bool vec = vec_ok(A, lda, ta ? Ms : Ks) && vec_ok(B, ldb, tb ? Ks : Ns);
    // XRS_SGEMM="cfg,splits": forced tile configuration / split-K slice count (tuning experiments)
    // (read per call: tuning scripts change it between calls)
    std::pair<int, int> g_env(-1, 0);
    if (const char* e = std::getenv("XRS_SGEMM")) std::sscanf(e, "%d,%d", &g_env.first, &g_env.second);
    auto tiles_of = [&](int c) { return ((M + kCfgs[c].bm - 1) / kCfgs[c].bm) * ((N + kCfgs[c].bn - 1) / kCfgs[c].bn); };
    constexpr bool kTune = std::is_same<EA, float>::value && std::is_same<EB, float>::value;
    int cfg = g_env.first;
    if (cfg < 0 || cfg >= kNumCfgs || (!kTune && cfg >= 5 && cfg < 13)) {
        if (tiles_of(0) >= 200) cfg = 0;
        else if (M % 64 == 0 && N % 80 == 0 && tiles_of(2) >= 192 && tiles_of(2) <= 320) cfg = 2;
        else if (M % 80 == 0 && N % 64 == 0 && tiles_of(3) >= 192 && tiles_of(3) <= 320) cfg = 3;
        else if (M >= 48 && N >= 48) cfg = 1;
        else cfg = 4;
        // an fp64 operand (the zipper's cores): the 64x64 tile with a 2-step ring capped at 128 registers, so
        // two workgroups share a CU -- the two zipper ends' launches run concurrently (dot_f32 0.25 -> 0.224 ms,
        // profiles/r05/dot32_occ4_ab_r05aa.txt); the fp32 x fp32 64x64 kernel already fits 120 registers
        if (!kTune && cfg >= 1 && cfg <= 3) cfg = 13;
        // fp32 x fp32 64x64: the 2-step ring (103 registers) measured 1-3 % faster than the 4-step one on
        // 1024^3 (profiles/r05/sgemm_probe_r05ag.txt, r05j)
        if (kTune && cfg == 1) cfg = 6;
    }
    const int bk = kCfgs[cfg].bk, bm = kCfgs[cfg].bm, bn = kCfgs[cfg].bn;
    const int tiles = tiles_of(cfg);
    const bool whole = vec && M % bm == 0 && N % bn == 0 && K % bk == 0 &&
                       double(std::max(bk, bm)) * double(lda) * sizeof(EA) < 2147483648.0 &&
                       double(std::max(bk, bn)) * double(ldb) * sizeof(EB) < 2147483648.0;
    const int mode = whole ? 2 : (vec ? 1 : 0);
    const int ksteps = (K + bk - 1) / bk;
    int splits = g_env.second;
    if (splits <= 0) {
        // split-K toward ~256 workgroups (XRS_SG_TARGET: another count, tuning) with >= 4 K-steps of 32 per slice
        int target = 256;
        if (const char* e = std::getenv("XRS_SG_TARGET")) target = std::max(1, std::atoi(e));
        splits = 1;
        if (tiles < 192) splits = std::max(1, std::min((target + tiles - 1) / tiles, ksteps * bk / 128));
    }
    splits = std::max(1, std::min(splits, ksteps));
    const int kps = (ksteps + splits - 1) / splits * bk;
    splits = (K + kps - 1) / kps;
    int xg = 0;
    {
        const int tm = (M + kCfgs[cfg].bm - 1) / kCfgs[cfg].bm, tn = (N + kCfgs[cfg].bn - 1) / kCfgs[cfg].bn;
        if (double(N) >= double(M)) xg = (tn % 8 == 0) ? 1 : 0;
        else xg = (tm % 8 == 0) ? 2 : 0;
        // whole split-K slices per XCD: XRS_SG_XCD_SPLIT=1 (A/B; off by default: the zipper measured
        // 0.213 vs 0.211 ms with it, profiles/r05/xcd_split_ab_r05aj.txt, where the fp64 Grams' HBM reads fell
        // 56 -> 41 MB per launch at an unchanged step)
        const char* e = std::getenv("XRS_SG_XCD_SPLIT");
        if (e && e[0] == '1' && splits >= 8 && splits % 8 == 0) xg = 3;
    }
    // split-K slabs: one accumulator-layout tile per slice and tile (the in-launch combine reads them)
    DevBuf slab;
    const size_t slab_bytes = splits > 1 ? size_t(splits) * size_t(tiles) * size_t(bm) * size_t(bn) * sizeof(float) : 0;
    XRS_REQUIRE(slab_bytes < (size_t(1) << 31), "split-K slabs exceed 2 GiB");
    XRS_REQUIRE(splits == 1 || tiles <= xrs_handle_s::kTicketCap, "split-K tile grid exceeds the ticket array");
    if (splits > 1) slab = DevBuf(h, slab_bytes);
    Args p{A, lda, B, ldb, C, M, N, K, kps, alpha, x.sa, x.sb, x.amax, x.cmax_a, x.cmax_b, splits > 1 ? slab.as<float>() : nullptr,
           unsigned(slab_bytes), splits > 1 ? h->tickets : nullptr, (M + kCfgs[cfg].bm - 1) / kCfgs[cfg].bm, xg};
    const double bytes = double(sizeof(EA)) * M * K + double(sizeof(EB)) * K * N + 4.0 * M * N * (splits > 1 ? 2 * splits : 1);
#define XRS_CFG(...) launch_cfg<__VA_ARGS__, EA, EB>(h, p, ta, tb, mode, tiles, splits, bytes)
#define XRS_CFG4(...) launch_cfg<__VA_ARGS__, EA, EB, 4>(h, p, ta, tb, mode, tiles, splits, bytes)
    switch (cfg) {
        case 0: XRS_CFG(128, 128, 2, 4, 1, 32, 2, 2); break;
        case 1: XRS_CFG(64, 64, 2, 2, 2, 32, 4, 2); break;
        case 2: XRS_CFG(64, 80, 4, 1, 2, 32, 4, 2); break;
        case 3: XRS_CFG(80, 64, 1, 4, 2, 32, 4, 2); break;
        case 4: XRS_CFG(32, 32, 2, 1, 1, 32, 2, 2); break;
        case 13: XRS_CFG4(64, 64, 2, 2, 2, 32, 2, 2); break;
        case 14: XRS_CFG4(64, 80, 4, 1, 2, 32, 2, 2); break;
        case 15: XRS_CFG4(80, 64, 1, 4, 2, 32, 2, 2); break;
        default:
            if constexpr (kTune) {
                switch (cfg) {
                    case 5: XRS_CFG(64, 64, 2, 2, 2, 64, 2, 2); break;
                    case 6: XRS_CFG(64, 64, 2, 2, 2, 32, 2, 2); break;
                    case 7: XRS_CFG(64, 80, 4, 1, 2, 32, 2, 2); break;
                    case 8: XRS_CFG(128, 128, 2, 4, 1, 32, 4, 3); break;
                    case 9: XRS_CFG(80, 64, 1, 4, 2, 32, 2, 2); break;
                    case 10: XRS_CFG(64, 64, 2, 2, 2, 32, 4, 3); break;
                    case 11: XRS_CFG(64, 80, 4, 1, 2, 32, 4, 3); break;
                    default: XRS_CFG(80, 64, 1, 4, 2, 32, 4, 3); break;
                }
            }
            break;
    }
#undef XRS_CFG
#undef XRS_CFG4
}

}  // namespace xrs
