// The fused fp32 zipper: <x,y> of two TTs on fp32 MFMA tiles with ONE launch per zipper step for both ends
// (xrs_tt_dot_f32's main path; dot32.hip keeps the per-product form for the shapes this one refuses).
// Reference arithmetic: TTNetwork's <x,y> (ttNetwork.cpp:782-789), the zipper of dgemm calls
// (blasLapackWrapper.cpp:177-191) in value_t = double; here fp32 products, fp64 closing sum.
//
// Left environments E_{k+1}[a2,b2] = sum_{a,b,i} E_k[a,b] X_k[a,i,a2] Y_k[b,i,b2], right environments
// F_k[a,b] = sum_{i,a2,b2} X_k[a,i,a2] F_{k+1}[a2,b2] Y_k[b,i,b2], closed at the middle edge by sum E_m o F_m.
//
//  - Start (k_zstart): E_1 = X_0^T Y_0 and F_{d-1} = X_{d-1} Y_{d-1}^T in fp64 (exact; the first step reads them
//    in fp64 and scales them into fp32 range as it loads them).
//  - Step (k_zstep, one launch for both ends, cores 1..m-1 from the left and d-2..m from the right): a
//    workgroup owns one (end, mode index i, 32-wide block of the new environment's first index) unit and
//    computes, for the left end,
//        T   (b x 32) = E_n^T X_k[:, i, blk]            (K = a; E_n = E scaled into [0.5, 1))
//        P   (32 x b2) = (2^-t T)^T Y_k[:, i, :]        (K = b; t = T's own exponent, T stays in LDS)
//    and stores P with t. The right end is the same computation on transposed views of its cores.
//    Operand fragments go from global memory (L2) straight into registers (16-B loads, a 4-deep register
//    ring, no LDS staging and no barrier in either K loop): rows / columns of a 16 x 16 MFMA block are
//    taken as a strided permutation of the wave's 64 rows / columns, so that one lane's 16-B load holds
//    the values of the same k for the 4 row blocks (fp32 E) or 2 / 4 column blocks (fp64 cores); T goes to
//    LDS transposed and un-permuted for the second product. Units are dealt to the XCDs in contiguous
//    ranges, so the units of one mode index (which share Y_k[:, i, :]) share one L2.
//  - Reduce (k_zreduce): E' = sum_i 2^(t_i - t_max) P_i in fixed order (deterministic), max|E'| into an
//    exponent word; the next step scales E' by 2^-u as it loads it. The host adds the exponents back.
//  - Finish (k_zfinish): sum E_m o F_m in fp64 (64 block partials in fixed order), the core maxima.
// Range: every product has one raw core and one operand normalised by a power of two; the cores' max|.| are
// recorded as they are read and a core outside [2^-100, 2^100) sends the product to the fp64 zipper, as in
// dot32.hip. Environments are stored zero-padded to multiples of 32 (no masks in the K loops). Requirements of
// this path (else dot32.hip's per-product form): interior ranks multiples of 4 up to 256, 16-B aligned cores.
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "runtime.hpp"
#include "sgemm.hpp"
#include "tt_internal.hpp"

namespace xrs {
namespace zip {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kBias = 1024;   // exponent words: e + kBias for a max |.| = f 2^e, f in [0.5, 1); 0 = all zero
constexpr int kBad = 0x7fff0000;   // a non-finite max (the host falls back to the fp64 zipper)

__device__ __forceinline__ int exp_word(double m) {
    if (!(m > 0.0)) return 0;
    if (!(m <= 1.7976931348623157e308)) return kBad;
    int e;
    (void)frexp(m, &e);
    return e + kBias;
}
// the exponent a consumer scales a word's operand by (fp32 operands: clamped so that 2^-e is a normal float)
__host__ __device__ __forceinline__ int f32_exp(int w) {
    if (w == 0) return 0;
    const int e = w - kBias;
    return e < -125 ? -125 : (e > 126 ? 126 : e);
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float(unsigned(127 + e) << 23); }   // e in [-126, 127]

__device__ __forceinline__ float fp64_max_as_float(double m) {
    const float f = float(m);
    return (m > 0.0 && f == 0.0f) ? __uint_as_float(1u) : f;
}
__device__ __forceinline__ void wave_max_slot(unsigned* slot, double m) {
    float f = fp64_max_as_float(m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f = fmaxf(f, __shfl_xor(f, o));
    if ((threadIdx.x & 63) == 0) atomicMax(slot, __float_as_uint(f));
}
__device__ __forceinline__ void wave_max_slot_f(unsigned* slot, float f) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f = fmaxf(f, __shfl_xor(f, o));
    if ((threadIdx.x & 63) == 0) atomicMax(slot, __float_as_uint(f));
}
// workgroup max of m (all threads call it; red: >= 8 doubles of free LDS); returned to every thread
__device__ __forceinline__ double block_max(double m, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    double b = 0.0;
    for (int i = 0; i < int(blockDim.x >> 6); ++i) b = fmax(b, red[i]);
    return b;
}

// ------------------------------------------------------------------------------------------------ start
// E_1 (left) = X_0^T Y_0 and F_{d-1} (right) = X_{d-1} Y_{d-1}^T in fp64 (cores 1 x n x r / r x n x 1), written
// into zero-padded K x M buffers (the first step's E); their exponent words; the two cores' max|.|.
struct StartEnd {
    const double *X, *Y;
    double* out;         // ldm = Mp, rows Kp
    int* eword;
    unsigned *cx, *cy;
    int n, ra, rb, Kp, Mp, right, blocks;
};
struct StartArgs {
    StartEnd e[2];
    int blocks0;
};
__global__ void __launch_bounds__(256) k_zstart(const StartArgs args) {
    const int end = int(blockIdx.x) >= args.blocks0 ? 1 : 0;
    const StartEnd& p = args.e[end];
    const int q = (int(blockIdx.x) - (end ? args.blocks0 : 0)) * 256 + int(threadIdx.x);
    __shared__ double red[8];
    const int a = q / p.Mp, b = q % p.Mp;
    const bool in = a < p.Kp;
    const bool ok = in && a < p.ra && b < p.rb;
    double s = 0.0, mx = 0.0, my = 0.0;
    if (ok) {
#pragma unroll 4
        for (int i = 0; i < p.n; ++i) {
            const double x = p.right ? p.X[size_t(a) * p.n + i] : p.X[size_t(i) * p.ra + a];
            const double y = p.right ? p.Y[size_t(b) * p.n + i] : p.Y[size_t(i) * p.rb + b];
            mx = fmax(mx, fabs(x));
            my = fmax(my, fabs(y));
            s = fma(x, y, s);
        }
    }
    if (in) p.out[size_t(a) * p.Mp + b] = s;
    const double m = block_max(fabs(s), red);
    if (threadIdx.x == 0) atomicMax(p.eword, exp_word(m));
    const unsigned slot = unsigned(blockIdx.x) % unsigned(kCmaxSlots);
    wave_max_slot(p.cx + slot, mx);
    wave_max_slot(p.cy + slot, my);
}

// ------------------------------------------------------------------------------------------------ step
// One end's step, written for the left end (the right end: X and Y read transposed, `right`):
//   T (M1 x N1) = E^T (M1 x K1) Xs (K1 x N1),  P (N1 x N2) = T^T (N1 x M1) Ys (M1 x N2)
// with Xs(k, c) = X[i*xi + k*xk + c*xc] and Ys(k, c) = Y[i*yi + k*yk + c*yc]. E: K1 x M1 row-major, both
// padded to multiples of 32 with zeros (K1r / M1r the true ranks: Xs / Ys rows past them are read at clamped
// addresses and meet zero rows / columns of E, so they add exact zeros). Columns of Xs past N1 and of Ys past N2
// are zeroed, so P is exactly zero outside N1 x N2 and the slab (ld N2p = N2 padded) needs no masks.
struct StepEnd {
    const void* E;
    const double* X;
    const double* Y;
    float* slab;          // [n][nblk][32][N2p]
    int* texp;            // [n * nblk] exponent words of the units' T
    int* tmax;            // max over texp
    const int* eword;     // exponent word of E
    unsigned *cx, *cy;    // core max slots
    long long xi, xk, xc, yi, yk, yc;
    int K1, M1, K1r, M1r, N1, N2, N2p, n, nblk;
};
struct StepArgs {
    StepEnd e[2];
    int units0, units;
};

// A K loop of C chunks: raw loads into a register ring of PD slots (fetch(slot, c)), converted operands in two
// register sets (conv(slot, set, c): fp64 -> fp32, scales, masks), MFMAs on a converted set (mma(set, c)).
// Chunk c + 1 is converted while chunk c's MFMAs run (no dependence between the two: the VALU work issues in
// the MFMA pipe's shadow), then the slot chunk c + 1 came from is refilled with chunk c + 1 + PD... at the
// latest one step later. Program order = issue order of the loads, so the waitcnt before a conversion counts
// the PD - 2 chunks of loads still in flight. NC > 0: C == NC, fully unrolled (no back edge for the waitcnt
// pass); NC == 0: a loop over groups of PD chunks (C % PD == 0, PD even).
template <int PD, class Fetch>
__device__ __forceinline__ void k_chain_prologue(Fetch&& fetch) {
    [&]<int... U>(std::integer_sequence<int, U...>) { (fetch(std::integral_constant<int, U>{}, U), ...); }(std::make_integer_sequence<int, PD>{});
}
template <int NC, int PD, class Fetch, class Conv, class Mma>
__device__ __forceinline__ void k_chain(int C, Fetch&& fetch, Conv&& conv, Mma&& mma) {
    using I0 = std::integral_constant<int, 0>;
    conv(I0{}, I0{}, 0);
    auto step = [&](auto slot_c, auto set_c, auto nslot_c, auto nset_c, int c, bool more, bool refill) {
        __builtin_amdgcn_sched_barrier(0);
        mma(set_c, c);
        if (more) conv(nslot_c, nset_c, c + 1);
        __builtin_amdgcn_sched_barrier(0);
        if (refill) fetch(slot_c, c + PD);
    };
    if constexpr (NC > 0) {
        [&]<int... c>(std::integer_sequence<int, c...>) {
            (step(std::integral_constant<int, c % PD>{}, std::integral_constant<int, c & 1>{},
                  std::integral_constant<int, (c + 1) % PD>{}, std::integral_constant<int, (c + 1) & 1>{}, c, c + 1 < NC,
                  c + PD < NC),
             ...);
        }(std::make_integer_sequence<int, NC>{});
    } else {
        static_assert(PD % 2 == 0, "the converted sets alternate with the chunk parity");
        for (int c0 = 0; c0 < C; c0 += PD) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (step(std::integral_constant<int, U>{}, std::integral_constant<int, U & 1>{},
                      std::integral_constant<int, (U + 1) % PD>{}, std::integral_constant<int, (U + 1) & 1>{}, c0 + U,
                      c0 + U + 1 < C, true),
                 ...);
            }(std::make_integer_sequence<int, PD>{});
        }
    }
}

// Diagnostic (XRS_ZIP_STAMPS=1, tools/zip_stamps.py): thread 0 of every k_zstep workgroup writes s_memtime at
// 0 start, 1 phase 1 done, 2 T in LDS, 3 phase 2 done, 4 end, and [7] = XCC id << 32 | HW id, 8 words per workgroup
__device__ unsigned long long* g_zip_stamps = nullptr;
#define XRS_ZIP_STAMP(i)                                                                                      \
    if (threadIdx.x == 0 && g_zip_stamps != nullptr) {                                                       \
        g_zip_stamps[8 * blockIdx.x + (i)] = __builtin_amdgcn_s_memtime();                                   \
        if ((i) == 0)                                                                                        \
            g_zip_stamps[8 * blockIdx.x + 7] = (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) | \
                                               __builtin_amdgcn_s_getreg((31 << 11) | 4);                    \
    }


// FULL: every row / column of the unit is inside the true ranks (K1r = K1, M1r = M1, N1 % 32 == 0, N2 == N2p): no
// masks or clamps. KH: the unit's share of T's rows (= the second product's K): 1 all M1 rows; 2 half h of them
// (twice the units, each half the work -- 640 instead of 320 at rank 256, so the CUs that hold one unit more than
// the others carry half the excess). Phase 1 waves: KH 1: wave w owns rows 64 w + [0, 64) and the unit's 32
// columns (2 col-blocks); KH 2: rows h M1/2 + 64 (w & 1) + [0, 64), columns 16 (w >> 1) + [0, 16) (1 col-block).
template <bool E64, bool RIGHT, int PD, int NC1, int NC2, bool FULL, int KH, int BR, int PD1 = PD>
__device__ __forceinline__ void zstep_unit(const StepEnd& p, const int i, const int blk, const int h, float* ltt, double* red) {
    constexpr int RG = KH == 1 ? 4 : 2;  // waves per column group (phase 1)
    constexpr int CW = BR * RG / 4;      // phase-1 columns per wave
    constexpr int CB = CW / 16;          // phase-1 col-blocks per wave
    static_assert(CB == 1 || CB == 2, "16 or 32 phase-1 columns per wave");
    constexpr int RB2 = BR / 16;         // phase-2 row-blocks
    constexpr int LDT = 256 / KH + 4;    // T^T row stride in LDS (floats): a 4-bank shift per row
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int M1 = p.M1, N1 = p.N1, N2 = p.N2;
    const int mh = M1 / KH;              // rows of T in this unit (K of phase 2)
    const double* __restrict__ X = p.X + size_t(i) * p.xi;
    const double* __restrict__ Y = p.Y + size_t(i) * p.yi + size_t(h) * mh * p.yk;
    // max|.| of the cores as converted to fp32 (one v_max_f32 per element): a core above the fp32 range shows as
    // inf, one whose max lies below 2^-100 as a small or zero max -- the host sends both to the fp64 zipper
    float vmx = 0.0f, vmy = 0.0f;

    // ---- phase 1: T rows of the wave (row-block a <-> rows rowbase + 4 r + a), columns c1 (+ q); K1 in 16-deep
    // chunks, lane group g takes k = 4 g + j (j = MFMA)
    const int rg = w % RG, cg = w / RG;
    const int rowbase = h * mh + 64 * rg;
    const bool rows_ok = FULL || rowbase + 4 * r < M1;
    const int erow = rows_ok ? rowbase + 4 * r : 0;
    const int c1 = blk * BR + cg * CW + (CB == 2 ? 2 * r : r);
    const bool cols1_ok = FULL || c1 < N1;
    const int xcol = cols1_ok ? c1 : 0;
    const int C1 = p.K1 / 16;
    const int kx = p.K1r - 1;   // last real row of Xs
    const int eu = f32_exp(*p.eword);
    const double es64 = E64 ? ldexp(1.0, -(*p.eword == 0 ? 0 : *p.eword - kBias)) : 1.0;
    const float es32 = pow2f(-eu);

    struct R1 {
        f4 e[4];      // E[k][erow .. +3] for j = 0..3 (fp32 E)
        d2 e64[4][2]; // (fp64 E)
        d2 x[4];      // LEFT: x[j] = Xs(k_j, c1 .. c1 + CB - 1); RIGHT: x[2q + hh] = Xs(k0 + 2hh .. +1, c1 + q)
    };
    R1 ring1[PD1];
    float ea[2][4][4], xb[2][4][CB];   // converted operands, two sets
    // FULL: per-lane base addresses once, a wave-uniform offset per chunk (no clamps: every row is real)
    const float* eb = static_cast<const float*>(p.E) + size_t(4 * g) * M1 + erow;
    const double* xb0 = RIGHT ? X + size_t(xcol) * p.xc + 4 * g : X + size_t(4 * g) * p.xk + xcol;
    auto load_x_left = [&](R1& s, int j, const double* xp) {
        if constexpr (CB == 2) s.x[j] = *reinterpret_cast<const d2*>(xp);
        else s.x[j][0] = *xp;
    };
    auto load1 = [&](auto slot_c, int c) {
        R1& s = ring1[decltype(slot_c)::value];
        c = min(c, C1 - 1);
        if constexpr (FULL && !E64) {
            const float* e = eb + size_t(16 * c) * M1;
#pragma unroll
            for (int j = 0; j < 4; ++j) s.e[j] = *reinterpret_cast<const f4*>(e + size_t(j) * M1);
            if constexpr (!RIGHT) {
                const double* x = xb0 + size_t(16 * c) * p.xk;
#pragma unroll
                for (int j = 0; j < 4; ++j) load_x_left(s, j, x + size_t(j) * p.xk);
            } else {
                const double* x = xb0 + 16 * c;
#pragma unroll
                for (int q = 0; q < CB; ++q)
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) s.x[2 * q + hh] = *reinterpret_cast<const d2*>(x + size_t(q) * p.xc + 2 * hh);
            }
            return;
        }
        const int k0 = 16 * c + 4 * g;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (E64) {
                const double* ep = static_cast<const double*>(p.E) + size_t(k0 + j) * M1 + erow;
                s.e64[j][0] = *reinterpret_cast<const d2*>(ep);
                s.e64[j][1] = *reinterpret_cast<const d2*>(ep + 2);
            } else {
                s.e[j] = *reinterpret_cast<const f4*>(static_cast<const float*>(p.E) + size_t(k0 + j) * M1 + erow);
            }
        }
        if constexpr (!RIGHT) {
#pragma unroll
            for (int j = 0; j < 4; ++j) load_x_left(s, j, X + size_t(min(k0 + j, kx)) * p.xk + xcol);
        } else {
            // (K1r even: a pair starting inside the real rows lies inside them)
#pragma unroll
            for (int q = 0; q < CB; ++q)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
                    s.x[2 * q + hh] = *reinterpret_cast<const d2*>(X + size_t(xcol + q) * p.xc + min(k0 + 2 * hh, kx - 1));
        }
    };
    auto conv1 = [&](auto slot_c, auto set_c, int) {
        const R1& s = ring1[decltype(slot_c)::value];
        constexpr int S = decltype(set_c)::value;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float v;
                if constexpr (E64) v = float(s.e64[j][q >> 1][q & 1] * es64);
                else v = s.e[j][q] * es32;
                ea[S][j][q] = rows_ok ? v : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < CB; ++q) {
                double v;
                if constexpr (!RIGHT) v = s.x[j][q];
                else v = s.x[2 * q + (j >> 1)][j & 1];
                const float f = float(v);
                vmx = fmaxf(vmx, fabsf(f));
                xb[S][j][q] = cols1_ok ? f : 0.0f;
            }
        }
        asm volatile("" : "+v"(vmx));   // the running max stays per chunk (no deferred max tree over the loop)
    };
    f4 acc1[4][CB];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < CB; ++b) acc1[a][b] = f4{0.f, 0.f, 0.f, 0.f};
    auto mma1 = [&](auto set_c, int) {
        constexpr int S = decltype(set_c)::value;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < CB; ++b) acc1[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(ea[S][j][a], xb[S][j][b], acc1[a][b], 0, 0, 0);
    };
    XRS_ZIP_STAMP(0)
    if (rowbase < M1) {
        k_chain_prologue<PD1>(load1);
        k_chain<NC1, PD1>(C1, load1, conv1, mma1);
    }
    __builtin_amdgcn_sched_barrier(0);
    XRS_ZIP_STAMP(1)

    // ---- phase 2 operands start loading now (they do not depend on T): Ys(h mh + k, colbase + 4 r + q), wave
    // columns [64 w, 64 w + 64), K = mh
    const int colbase = 64 * w;
    const int c2 = colbase + 4 * r;
    const bool cols2_ok = FULL || c2 < N2;
    const int ycol = cols2_ok ? c2 : 0;
    const int C2 = mh / 16;
    const int ky = p.M1r - 1 - h * mh;   // last real row of this unit's Ys rows
    struct R2 {
        d2 y[8];   // LEFT: y[2j + hh] = Ys(k_j, ycol + 2hh .. +1); RIGHT: y[2q + hh] = Ys(k0 + 2hh .. +1, ycol + q)
    };
    R2 ring2[PD];
    float yb[2][4][4];
    const double* yb0 = RIGHT ? Y + size_t(ycol) * p.yc + 4 * g : Y + size_t(4 * g) * p.yk + ycol;
    auto load2 = [&](auto slot_c, int c) {
        R2& s = ring2[decltype(slot_c)::value];
        c = min(c, C2 - 1);
        if constexpr (FULL) {
            if constexpr (!RIGHT) {
                const double* y = yb0 + size_t(16 * c) * p.yk;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    s.y[2 * j] = *reinterpret_cast<const d2*>(y + size_t(j) * p.yk);
                    s.y[2 * j + 1] = *reinterpret_cast<const d2*>(y + size_t(j) * p.yk + 2);
                }
            } else {
                const double* y = yb0 + 16 * c;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    s.y[2 * q] = *reinterpret_cast<const d2*>(y + size_t(q) * p.yc);
                    s.y[2 * q + 1] = *reinterpret_cast<const d2*>(y + size_t(q) * p.yc + 2);
                }
            }
            return;
        }
        const int k0 = 16 * c + 4 * g;
        if constexpr (!RIGHT) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double* yp = Y + size_t(min(k0 + j, ky)) * p.yk + ycol;
                s.y[2 * j] = *reinterpret_cast<const d2*>(yp);
                s.y[2 * j + 1] = *reinterpret_cast<const d2*>(yp + 2);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double* yp = Y + size_t(ycol + q) * p.yc;
                s.y[2 * q] = *reinterpret_cast<const d2*>(yp + min(k0, ky - 1));
                s.y[2 * q + 1] = *reinterpret_cast<const d2*>(yp + min(k0 + 2, ky - 1));
            }
        }
    };
    auto conv2 = [&](auto slot_c, auto set_c, int) {
        const R2& s = ring2[decltype(slot_c)::value];
        constexpr int S = decltype(set_c)::value;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                double v;
                if constexpr (!RIGHT) v = s.y[2 * j + (q >> 1)][q & 1];
                else v = s.y[2 * q + (j >> 1)][j & 1];
                const float f = float(v);
                vmy = fmaxf(vmy, fabsf(f));
                yb[S][j][q] = cols2_ok ? f : 0.0f;
            }
        asm volatile("" : "+v"(vmy));
    };
    const bool wave2 = colbase < p.N2p;
    if (wave2) k_chain_prologue<PD>(load2);   // in flight across T's reduction and the barrier

    // ---- T's exponent (this unit's own), T^T into LDS scaled by 2^-t: lane (n, mg) holds block (a, q) reg e at
    // T row rowbase + 4 (4 mg + e) + a = local k 64 rg + 16 mg + 4 e + a, column (KH 1) 2 n + q / (KH 2) 16 cg + n
    float tmf = 0.0f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int e = 0; e < 4; ++e) tmf = fmaxf(tmf, fabsf(acc1[a][b][e]));
    const double tm = block_max(double(tmf), red);
    const int tw = exp_word(tm);
    const int te = f32_exp(tw);
    const float ts = pow2f(-te);
    if (rowbase < M1) {
        const int n = lane & 15, mg = lane >> 4;
#pragma unroll
        for (int b = 0; b < CB; ++b)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const f4 v = f4{acc1[0][b][e], acc1[1][b][e], acc1[2][b][e], acc1[3][b][e]} * ts;
                const int col = cg * CW + (CB == 2 ? 2 * n + b : n);
                *reinterpret_cast<f4*>(ltt + col * LDT + 64 * rg + 16 * mg + 4 * e) = v;
            }
    }
    const int unit = (i * p.nblk + blk) * KH + h;
    if (tid == 0) {
        p.texp[unit] = tw == 0 ? 0 : te + kBias;
        atomicMax(p.tmax, tw == 0 ? 0 : te + kBias);
    }
    __syncthreads();
    XRS_ZIP_STAMP(2)

    // ---- phase 2: P (BR x N2p) = (T^T) Ys; row-block a < RB2: rows 16 a + r; col-block q: columns c2 + q
    f4 acc2[RB2][4];
#pragma unroll
    for (int a = 0; a < RB2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc2[a][b] = f4{0.f, 0.f, 0.f, 0.f};
    auto mma2 = [&](auto set_c, int c) {
        constexpr int S = decltype(set_c)::value;
        const int k0 = 16 * c + 4 * g;
        f4 ta[RB2];
#pragma unroll
        for (int a = 0; a < RB2; ++a) ta[a] = *reinterpret_cast<const f4*>(ltt + (16 * a + r) * LDT + k0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int a = 0; a < RB2; ++a)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc2[a][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ta[a][j], yb[S][j][q], acc2[a][q], 0, 0, 0);
    };
    if (wave2) {
        k_chain<NC2, PD>(C2, load2, conv2, mma2);
        XRS_ZIP_STAMP(3)
        // P rows 16 a + 4 mg + e of this unit, columns colbase + 4 n .. +3 (zeros outside N1 x N2)
        const int n = lane & 15, mg = lane >> 4;
        const int col = colbase + 4 * n;
        float* out = p.slab + size_t(unit) * BR * size_t(p.N2p);
        if (col < p.N2p) {
#pragma unroll
            for (int a = 0; a < RB2; ++a)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    *reinterpret_cast<f4*>(out + size_t(16 * a + 4 * mg + e) * p.N2p + col) =
                        f4{acc2[a][0][e], acc2[a][1][e], acc2[a][2][e], acc2[a][3][e]};
        }
    }
    const unsigned slot = unsigned(unit) % unsigned(kCmaxSlots);
    wave_max_slot_f(p.cx + slot, vmx);
    wave_max_slot_f(p.cy + slot, vmy);
    XRS_ZIP_STAMP(4)
}

// units are dealt to the XCDs in contiguous ranges (workgroups go to the 8 XCDs round-robin by dispatch
// order): the units of one (end, i) -- which read the same Y_k[:, i, :] -- run in one L2
template <bool E64, int PD, int NC1, int NC2, bool FULL, int KH, int BR, int PD1 = PD>
__global__ void __launch_bounds__(256, 2) k_zstep(const StepArgs args) {
    __shared__ float ltt[BR * (256 / KH + 4)];
    __shared__ double red[8];
    int u = int(blockIdx.x);
    if (args.units % 8 == 0) u = (u & 7) * (args.units / 8) + (u >> 3);
    const bool left = u < args.units0;
    const StepEnd& p = args.e[left ? 0 : 1];
    if (!left) u -= args.units0;
    const int h = u % KH, q = u / KH;
    if (left) zstep_unit<E64, false, PD, NC1, NC2, FULL, KH, BR, PD1>(p, q / p.nblk, q % p.nblk, h, ltt, red);
    else zstep_unit<E64, true, PD, NC1, NC2, FULL, KH, BR, PD1>(p, q / p.nblk, q % p.nblk, h, ltt, red);
}

// ------------------------------------------------------------------------------------------------ reduce
// E' (N1p x N2p, ld N2p; rows past the last unit block and the padding come out zero) = sum_i 2^(t_i - t_max) P_i
struct RedEnd {
    const float* slab;
    const int* texp;
    const int* tmax;
    float* out;
    int* eword;        // exponent word of max|out|
    unsigned* mword;   // optional: max word (float bits, kMaxLanes lanes) of max|out| (dot32.hip's steps read it)
    int n, nblk, N1p, N2p, kh, br;
    int blocks;
};
struct RedArgs {
    RedEnd e[2];
    int blocks0;
};
constexpr int kRedT = 64;   // threads per reduce block: 4-8 blocks per CU at the TT sizes (latency-bound loads)
__global__ void __launch_bounds__(kRedT) k_zreduce(const RedArgs args) {
    const int end = int(blockIdx.x) >= args.blocks0 ? 1 : 0;
    const RedEnd& p = args.e[end];
    const int b = int(blockIdx.x) - (end ? args.blocks0 : 0);
    __shared__ double red[8];
    const int q = b * kRedT + int(threadIdx.x);   // float4 index
    const int per_row = p.N2p / 4;
    const bool ok = q < p.N1p * per_row;
    const int row = ok ? q / per_row : 0, col = ok ? (q % per_row) * 4 : 0;
    const int blk = row / p.br, rr = row % p.br;
    const int tm = *p.tmax;
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    if (ok) {
        // slab of (i, blk, h): ((i nblk + blk) kh + h); summed over (i, h) in that order. The slabs were written by
        // units on every XCD: loads of up to kRedG slabs in flight per round trip
        const float* src = p.slab + (size_t(blk) * p.kh * p.br + rr) * p.N2p + col;
        const size_t stride_i = size_t(p.nblk) * p.kh * p.br * p.N2p, stride_h = size_t(p.br) * p.N2p;
        const int ns = p.n * p.kh;
        constexpr int kRedG = 20;
        for (int s0 = 0; s0 < ns; s0 += kRedG) {
            f4 v[kRedG];
            float sc[kRedG];
#pragma unroll
            for (int u = 0; u < kRedG; ++u) {
                const int sl = min(s0 + u, ns - 1), i = sl / p.kh, hh = sl % p.kh;
                v[u] = *reinterpret_cast<const f4*>(src + size_t(i) * stride_i + size_t(hh) * stride_h);
                const int tw = p.texp[(i * p.nblk + blk) * p.kh + hh];
                const int de = tw == 0 ? -1000 : tw - tm;
                sc[u] = (de < -126 || s0 + u >= ns) ? 0.0f : pow2f(de);
            }
#pragma unroll
            for (int u = 0; u < kRedG; ++u) s += sc[u] * v[u];
        }
        *reinterpret_cast<f4*>(p.out + size_t(row) * p.N2p + col) = s;
    }
    const double m = block_max(ok ? double(fmaxf(fmaxf(fabsf(s[0]), fabsf(s[1])), fmaxf(fabsf(s[2]), fabsf(s[3])))) : 0.0, red);
    if (threadIdx.x == 0) {
        atomicMax(p.eword, exp_word(m));
        if (p.mword) atomicMax(p.mword + b % kMaxLanes, __float_as_uint(float(m)));
    }
}

// ------------------------------------------------------------------------------------------------ finish
// blocks [0, 64): partial[b] = block b's share of sum E o F in fp64; blocks 64 + c: cmax_out[c] = max of core
// c's slots
constexpr int kPair = 64;
template <class TE, class TF>
__global__ void __launch_bounds__(256) k_zfinish(const TE* __restrict__ E, const TF* __restrict__ F, int n, double* partial,
                                               const unsigned* __restrict__ slots, unsigned* cmax_out) {
    __shared__ double red[4];
    __shared__ unsigned redu[4];
    if (blockIdx.x < kPair) {
        double s = 0.0;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += kPair * 256) s = fma(double(E[i]), double(F[i]), s);
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
        return;
    }
    const int c = int(blockIdx.x) - kPair;
    const unsigned* w = slots + size_t(c) * kCmaxSlots;
    unsigned m = 0u;
    for (int i = threadIdx.x; i < kCmaxSlots; i += 256) m = max(m, w[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, unsigned(__shfl_xor(int(m), o)));
    if ((threadIdx.x & 63) == 0) redu[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) cmax_out[c] = max(max(redu[0], redu[1]), max(redu[2], redu[3]));
}

__global__ void __launch_bounds__(256) k_zinit(unsigned* __restrict__ w, size_t words) {
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < words; i += size_t(gridDim.x) * 256) w[i] = 0u;
}

}  // namespace

// the shapes the fused path takes (else dot32.hip's per-product zipper): interior ranks multiples of 4 up to 256
// (environments padded to multiples of 32; 16-B operand vectors), 16-B aligned cores
bool applicable(size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                const double* const* Y) {
    if (d < 2) return false;
    for (size_t k = 0; k < d; ++k) {
        if ((reinterpret_cast<uintptr_t>(X[k]) | reinterpret_cast<uintptr_t>(Y[k])) & 15) return false;
        if (n[k] == 0 || n[k] > (size_t(1) << 20)) return false;
    }
    for (size_t k = 1; k < d; ++k)
        if (rx[k] % 4 || ry[k] % 4 || rx[k] > 256 || ry[k] > 256) return false;
    return true;
}

namespace {
// fr == null: the whole product (returns it). fr != null: the front end only -- E_1 / F_{d-1} and the first step
// of each end -- with the environments E_2 / F_{d-2} (fp32, padded, max words into fr->mword) and the exponent
// words left for the caller (returns 0); the caller's slot arrays receive the cores' maxima.
double run(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y, Front* fr) {
    const size_t m = d / 2;
    const size_t sl = fr ? 1 : m - 1, sr = fr ? 1 : d - 1 - m;   // steps per end (cores 1..m-1 / d-2..m)
    const size_t steps = std::max(sl, sr);
    auto p32 = [](size_t x) { return (x + 31) / 32 * 32; };
    auto up = [](size_t x) { return (x + 255) / 256 * 256; };
    // ---- device memory
    size_t slab_f = 0, tex = 1, env = 1;
    for (size_t k = 1; k + 1 < d; ++k) {
        const size_t nb = (std::max(rx[k], rx[k + 1]) + 31) / 32;
        slab_f = std::max(slab_f, 2 * n[k] * nb * 32 * p32(std::max(ry[k], ry[k + 1])));   // (2: KH up to 2)
        tex = std::max(tex, 2 * n[k] * nb);
    }
    for (size_t k = 1; k < d; ++k) env = std::max(env, p32(rx[k]) * p32(ry[k]));
    const size_t s0 = p32(rx[1]) * p32(ry[1]), s1 = p32(rx[d - 1]) * p32(ry[d - 1]);
    const size_t nst = std::max<size_t>(steps, 1);
    // words (ints): [0, 2d) exponent words of the environments by (end, edge), [2d, 4d) tmax words by (end, edge),
    // [4d, 6d) the cores' max|.| (finish)
    const size_t nwords = 6 * d;
    const size_t o_start0 = 0, o_start1 = up(8 * s0);
    const size_t o_env = o_start1 + up(8 * s1);
    const size_t o_slab = o_env + 4 * up(4 * env);
    const size_t o_part = o_slab + 2 * up(4 * slab_f);
    const size_t o_words = o_part + up(8 * kPair);
    const size_t o_slots = o_words + up(4 * nwords);
    const size_t o_tex = o_slots + up(4 * 2 * d * kCmaxSlots);
    const size_t total = o_tex + 2 * up(4 * tex * nst);
    DevBuf mem(h, total);
    char* base = mem.as<char>();
    double* start[2] = {reinterpret_cast<double*>(base + o_start0), reinterpret_cast<double*>(base + o_start1)};
    float* envb[2][2];
    for (int e = 0; e < 2; ++e)
        for (int q = 0; q < 2; ++q) envb[e][q] = reinterpret_cast<float*>(base + o_env + (2 * e + q) * up(4 * env));
    float* slab[2] = {reinterpret_cast<float*>(base + o_slab), reinterpret_cast<float*>(base + o_slab + up(4 * slab_f))};
    double* part = reinterpret_cast<double*>(base + o_part);
    int* words = reinterpret_cast<int*>(base + o_words);
    unsigned* slots = fr ? fr->slots : reinterpret_cast<unsigned*>(base + o_slots);
    int* texb[2] = {reinterpret_cast<int*>(base + o_tex), reinterpret_cast<int*>(base + o_tex + up(4 * tex * nst))};
    auto ew = [&](int e, size_t k) { return words + e * d + k; };
    auto tw = [&](int e, size_t k) { return words + 2 * d + e * d + k; };
    unsigned* cmax_out = reinterpret_cast<unsigned*>(words + 4 * d);
    auto sx = [&](size_t k) { return slots + k * kCmaxSlots; };
    auto sy = [&](size_t k) { return slots + (d + k) * kCmaxSlots; };

    {   // words, core-max slots (zeroed: the kernels atomicMax into them; a front end's slots are the caller's)
        const size_t zw = ((fr ? o_slots : o_tex) - o_words) / 4;
        hipLaunchKernelGGL(k_zinit, dim3(256), dim3(256), 0, h->stream, reinterpret_cast<unsigned*>(words), zw);
        check_launch("k_zinit");
    }
    {   // E_1 and F_{d-1} in fp64
        StartArgs sa{};
        sa.e[0] = StartEnd{X[0], Y[0], start[0], ew(0, 1), sx(0), sy(0), int(n[0]), int(rx[1]), int(ry[1]), int(p32(rx[1])),
                           int(p32(ry[1])), 0, int((s0 + 255) / 256)};
        sa.e[1] = StartEnd{X[d - 1], Y[d - 1], start[1], ew(1, d - 1), sx(d - 1), sy(d - 1), int(n[d - 1]), int(rx[d - 1]),
                           int(ry[d - 1]), int(p32(rx[d - 1])), int(p32(ry[d - 1])), 1, int((s1 + 255) / 256)};
        sa.blocks0 = sa.e[0].blocks;
        hipLaunchKernelGGL(k_zstart, dim3(sa.e[0].blocks + sa.e[1].blocks), dim3(256), 0, h->stream, sa);
        check_launch("k_zstart");
    }
    // ---- steps: both ends in one launch while both have one
    static const bool stamps = std::getenv("XRS_ZIP_STAMPS") != nullptr;
    DevBuf stamp_buf;
    if (stamps) {
        size_t mx = 1;
        for (size_t k = 0; k < d; ++k) mx = std::max(mx, 4 * n[k] * ((std::max(rx[k], rx[k + 1]) + 31) / 32));
        stamp_buf = DevBuf(h, mx * 64);
        unsigned long long* sp = stamp_buf.as<unsigned long long>();
        XRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_zip_stamps), &sp, sizeof(sp), 0, hipMemcpyHostToDevice, h->stream));
    }
    const void* cur[2] = {start[0], start[1]};
    for (size_t s = 0; s < steps; ++s) {
        StepArgs sa{};
        RedArgs ra{};
        int units[2] = {0, 0}, rblocks[2] = {0, 0};
        float* nxt[2] = {envb[0][s & 1], envb[1][s & 1]};
        int slot = 0;
        for (int e = 0; e < 2; ++e) {
            if (s >= (e == 0 ? sl : sr)) continue;
            const size_t k = e == 0 ? 1 + s : d - 2 - s;    // core
            const size_t ein = e == 0 ? k : k + 1, eout = e == 0 ? k + 1 : k;
            StepEnd& p = sa.e[slot];
            p.E = cur[e];
            p.X = X[k];
            p.Y = Y[k];
            p.slab = slab[e];
            p.texp = texb[e] + s * tex;
            p.tmax = tw(e, eout);
            p.eword = ew(e, ein);
            p.cx = sx(k);
            p.cy = sy(k);
            const long long nk = (long long)n[k];
            if (e == 0) {
                p.K1r = int(rx[k]), p.M1r = int(ry[k]), p.N1 = int(rx[k + 1]), p.N2 = int(ry[k + 1]);
                p.xi = p.N1, p.xk = nk * p.N1, p.xc = 1;
                p.yi = p.N2, p.yk = nk * p.N2, p.yc = 1;
            } else {
                p.K1r = int(rx[k + 1]), p.M1r = int(ry[k + 1]), p.N1 = int(rx[k]), p.N2 = int(ry[k]);
                p.xi = p.K1r, p.xk = 1, p.xc = nk * p.K1r;
                p.yi = p.M1r, p.yk = 1, p.yc = nk * p.M1r;
            }
            p.K1 = int(p32(p.K1r)), p.M1 = int(p32(p.M1r)), p.N2p = int(p32(p.N2));
            p.n = int(n[k]);
            p.nblk = (p.N1 + 31) / 32;
            units[slot] = p.n * p.nblk;
            RedEnd& q = ra.e[slot];
            q = RedEnd{slab[e], p.texp, p.tmax, nxt[e], ew(e, eout), fr ? fr->mword[e] : nullptr, p.n, p.nblk, 32 * p.nblk,
                       p.N2p, 1, 32, 0};
            q.blocks = (q.N1p * q.N2p / 4 + kRedT - 1) / kRedT;
            rblocks[slot] = q.blocks;
            ++slot;
        }
        // (slot 0 runs the left body, slot 1 the right one: a lone right end goes to slot 1)
        if (slot == 1 && s >= sl) {
            sa.e[1] = sa.e[0];
            ra.e[1] = ra.e[0];
            units[1] = units[0], units[0] = 0;
            rblocks[1] = rblocks[0], rblocks[0] = 0;
        }
        sa.units0 = units[0];
        sa.units = units[0] + units[1];
        {
            // algorithmic flops / bytes of the launch: both products of every unit (true ranks), cores read once
            double flops = 0.0, bytes = 0.0;
            bool all4 = true;
            for (int e = 0; e < 2; ++e) {
                if (!units[e]) continue;
                const StepEnd& p = sa.e[e];
                flops += 2.0 * p.n * (double(p.M1r) * p.K1r * p.N1 + double(p.N1) * p.M1r * p.N2);
                bytes += 8.0 * p.n * (double(p.K1r) * p.N1 + double(p.M1r) * p.N2) + 4.0 * p.n * p.nblk * 32.0 * p.N2p;
                if ((p.K1 / 16) % 4 || (p.M1 / 16) % 4) all4 = false;
            }
            KernelTimer timer(h, XRS_KFAM_GEMM, flops, bytes, true);
            // K of both products (K1, M1) 256 at every end of the launch: the fully unrolled chains, half units
            // (KH 2), and no masks when every unit lies inside the true ranks
            bool full = true, whole = true;
            for (int e = 0; e < 2; ++e) {
                if (!units[e]) continue;
                const StepEnd& p = sa.e[e];
                if (p.K1 != 256 || p.M1 != 256) full = false;
                if (p.K1r != 256 || p.M1r != 256 || p.N1 % 32 || p.N2 != p.N2p) whole = false;
            }
            const bool e64 = s == 0;
            // unit geometry: full steps KH 2 (T rows in halves); 64-row units where every end's N1 allows them
            bool br64 = full;
            for (int e = 0; e < 2; ++e)
                if (units[e] && sa.e[e].N1 % 64) br64 = false;
            const int kh = (!e64 && full) ? 2 : 1, br = br64 ? 64 : 32;
            for (int e = 0; e < 2; ++e) {
                if (!units[e]) continue;
                StepEnd& p = sa.e[e];
                p.nblk = (p.N1 + br - 1) / br;
                units[e] = p.n * p.nblk;
                ra.e[e].nblk = p.nblk;
                ra.e[e].kh = kh;
                ra.e[e].br = br;
            }
            sa.units0 = units[0] * kh;
            sa.units = (units[0] + units[1]) * kh;
            const unsigned grid = unsigned(sa.units);
#define XRS_ZSTEP(E64_, PD_, NC1_, NC2_, FULL_, KH_, BR_, ...) \
    hipExtLaunchKernelGGL((k_zstep<E64_, PD_, NC1_, NC2_, FULL_, KH_, BR_ __VA_OPT__(,) __VA_ARGS__>), dim3(grid), dim3(256), 0, h->stream, timer.start(), timer.stop(), 0, sa)
            if (e64) {
                XRS_ZSTEP(true, 2, 0, 0, false, 1, 32);   // (the fp64 ring of 4 spills; the first step is short)
            } else if (br64) {
                if (whole) XRS_ZSTEP(false, 3, 16, 8, true, 2, 64, 5);
                else XRS_ZSTEP(false, 3, 16, 8, false, 2, 64, 5);
            } else {
                if (full && whole) XRS_ZSTEP(false, 4, 16, 8, true, 2, 32);
                else if (full) XRS_ZSTEP(false, 4, 16, 8, false, 2, 32);
                else if (all4) XRS_ZSTEP(false, 4, 0, 0, false, 1, 32);
                else XRS_ZSTEP(false, 2, 0, 0, false, 1, 32);
            }
#undef XRS_ZSTEP
            check_launch("k_zstep");
            if (stamps) {   // one line per workgroup on stderr: step, wg, xcc<<32|hwid, stamps 0..4
                std::vector<unsigned long long> hv(size_t(grid) * 8);
                XRS_HIP(hipMemcpyAsync(hv.data(), stamp_buf.d(), hv.size() * 8, hipMemcpyDeviceToHost, h->stream));
                host_wait(h);
                for (int wg = 0; wg < int(grid); ++wg) {
                    const unsigned long long* q = hv.data() + 8 * wg;
                    std::fprintf(stderr, "[zip stamps] %zu %d %llu %llu %llu %llu %llu %llu\n", s, wg, q[7], q[0], q[1], q[2], q[3], q[4]);
                }
            }
        }
        ra.blocks0 = rblocks[0];
        hipLaunchKernelGGL(k_zreduce, dim3(rblocks[0] + rblocks[1]), dim3(kRedT), 0, h->stream, ra);
        check_launch("k_zreduce");
        for (int e = 0; e < 2; ++e)
            if (s < (e == 0 ? sl : sr)) cur[e] = nxt[e];
    }
    if (fr) {   // the environments after one step per end, the words the caller reads back with its own
        fr->E = static_cast<const float*>(cur[0]);
        fr->lde = p32(ry[2]);
        fr->F = static_cast<const float*>(cur[1]);
        fr->ldf = p32(ry[d - 2]);
        fr->words = words;
        fr->mem = std::move(mem);
        return 0.0;
    }
    // ---- closing at edge m: E_m (left) and F_m (right), both p32(rx[m]) x p32(ry[m]) (fp64 if an end had no step)
    const int nm = int(p32(rx[m]) * p32(ry[m]));
    const bool l64 = sl == 0, r64 = sr == 0;
    const dim3 fg(kPair + 2 * d);
    if (l64 && r64) hipLaunchKernelGGL((k_zfinish<double, double>), fg, dim3(256), 0, h->stream, static_cast<const double*>(cur[0]), static_cast<const double*>(cur[1]), nm, part, slots, cmax_out);
    else if (l64) hipLaunchKernelGGL((k_zfinish<double, float>), fg, dim3(256), 0, h->stream, static_cast<const double*>(cur[0]), static_cast<const float*>(cur[1]), nm, part, slots, cmax_out);
    else if (r64) hipLaunchKernelGGL((k_zfinish<float, double>), fg, dim3(256), 0, h->stream, static_cast<const float*>(cur[0]), static_cast<const double*>(cur[1]), nm, part, slots, cmax_out);
    else hipLaunchKernelGGL((k_zfinish<float, float>), fg, dim3(256), 0, h->stream, static_cast<const float*>(cur[0]), static_cast<const float*>(cur[1]), nm, part, slots, cmax_out);
    check_launch("k_zfinish");
    // ---- read back: partials, then the words (exponents, core maxima)
    char* hs = static_cast<char*>(h->host_scratch);
    const size_t back = o_words - o_part + 4 * nwords;
    XRS_REQUIRE(back <= (size_t(1) << 16), "fused fp32 zipper: read-back exceeds the host scratch");
    XRS_HIP(hipMemcpyAsync(hs, part, back, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    const int* hw = reinterpret_cast<const int*>(hs + (o_words - o_part));
    const unsigned* hc = reinterpret_cast<const unsigned*>(hw + 4 * d);
    // (a zero max: a zero core, or one whose every entry underflowed in fp32 -- the fp64 zipper decides)
    for (size_t c = 0; c < 2 * d; ++c) {
        const unsigned bits = hc[c];
        const int e = int((bits >> 23) & 0xff) - 127;
        if (bits == 0u || bits >= 0x7f800000u || e < -100 || e >= 100) return tt::dot(h, d, n, rx, X, ry, Y);
    }
    for (size_t i = 0; i < 4 * d; ++i)
        if (hw[i] >= kBad) return tt::dot(h, d, n, rx, X, ry, Y);
    double v = 0.0;
    for (int b = 0; b < kPair; ++b) {
        double p;
        std::memcpy(&p, hs + 8 * b, 8);
        v += p;
    }
    if (!std::isfinite(v)) return tt::dot(h, d, n, rx, X, ry, Y);
    // exponents: the environment out of a step = 2^(g_in + u + t) x its stored values (u: the scale the step
    // applied to its input -- unclamped for the fp64 start environments --, t: the step's tmax); E_1, F_{d-1}: g = 0
    int g = 0;
    for (int e = 0; e < 2; ++e) {
        const size_t ns = e == 0 ? sl : sr;
        for (size_t s = 0; s < ns; ++s) {
            const size_t k = e == 0 ? 1 + s : d - 2 - s;
            const size_t ein = e == 0 ? k : k + 1, eout = e == 0 ? k + 1 : k;
            const int uw = hw[e * d + ein];
            const int u = s == 0 ? (uw == 0 ? 0 : uw - kBias) : f32_exp(uw);
            const int t = hw[2 * d + e * d + eout];
            g += u + (t == 0 ? 0 : t - kBias);
        }
    }
    return std::ldexp(v, g);
}

}  // namespace

double dot(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y) {
    return run(h, d, n, rx, X, ry, Y, nullptr);
}

bool front_applicable(size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                      const double* const* Y) {
    return d >= 6 && applicable(d, n, rx, X, ry, Y);
}

void front(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
           const double* const* Y, Front& fr) {
    run(h, d, n, rx, X, ry, Y, &fr);
}

int front_exponent(const int* hw, size_t d, int end) {
    // the first step's input scale (the fp64 start environment: unclamped) and its tmax (zip32 word layout)
    const size_t ein = end == 0 ? 1 : d - 1, eout = end == 0 ? 2 : d - 2;
    const int uw = hw[end * d + ein], t = hw[2 * d + end * d + eout];
    return (uw == 0 ? 0 : uw - kBias) + (t == 0 ? 0 : t - kBias);
}

bool front_words_bad(const int* hw, size_t d) {
    for (size_t i = 0; i < 4 * d; ++i)
        if (hw[i] >= kBad) return true;
    return false;
}

}  // namespace zip
}  // namespace xrs
