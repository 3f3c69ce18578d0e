// <x,y> of two TTs on fp32 MFMA tiles (xrs_tt_dot_f32): the north star's "dense contraction on MFMA fp32
// tiles" as a side path beside the fp64 zipper (tt.hip: dot_two_ended), which stays the reference-precision
// product (value_t = double, include/xerus/basic.h:44; ttNetwork.cpp:782-789). Same two-ended zipper:
//   left  E_{k+1} = sum_i X_k[:,i,:]^T E_k Y_k[:,i,:]       (E_0 = 1)
//   right F_k     = sum_i X_k[:,i,:] F_{k+1} Y_k[:,i,:]^T   (F_d = 1)
// closed at the middle edge m by sum_ab E_m[a,b] F_m[a,b] (accumulated in fp64).
//
// Every product is one launch of the fp32-MFMA GEMM (sgemm_impl.hpp): the cores stay the caller's fp64
// blocks and are rounded to fp32 as they are staged into LDS (no conversion pass, no fp32 copy in HBM);
// environments and the intermediate T are fp32. Per step and end: T = E^T X_k (K = rank), then the environment
// product E' = T^T Y_k (K = n * rank, split-K with the slabs combined inside the launch).
// Range: each product multiplies ONE raw core by ONE operand normalised by a power of two -- E_0 = F_d = [1],
// and T and every environment record their max|.| in their producing launch (a max word) and are scaled by
// 2^-e into [0.5, 1) as the next launch stages them (exact); the host adds the exponents back in fp64. So a
// product is bounded by (n r) max|core|: every GEMM that reads a core also records the core's max|.| per
// workgroup, and a core whose max lies outside [2^-100, 2^100) (or is not finite) sends the whole product to
// the fp64 zipper (exact, slower); inside, no product leaves the fp32 range or its normal numbers.
// Accuracy: fp32 rounding of the cores and of each product, ~1e-7 relative to |<x,y>| for correlated pairs
// and to ||x|| ||y|| in general (tests).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "runtime.hpp"
#include "sgemm.hpp"
#include "tt_internal.hpp"

namespace xrs {
namespace {

// blocks [0, kPairBlocks): partial[b] = block b's grid-stride share of sum E[i] F[i] in fp64 (fixed order;
// the host adds the partials in order). Blocks kPairBlocks + c (c < ncores): cmax_out[c] = max over the
// kCmaxSlots words of slot array c (the per-workgroup core maxima of the GEMMs). The last block: wmax_out[i] =
// the value of max word i (max over its kMaxLanes lanes), i < nwords.
constexpr int kPairBlocks = 64;
__global__ void __launch_bounds__(256) k_dot32_finish(const float* __restrict__ E, const float* __restrict__ F, int n,
                                                      double* __restrict__ partial, const unsigned* __restrict__ slots,
                                                      int ncores, unsigned* __restrict__ cmax_out,
                                                      const unsigned* __restrict__ words, int nwords,
                                                      unsigned* __restrict__ wmax_out) {
    __shared__ double red[4];
    __shared__ unsigned redu[4];
    if (blockIdx.x < kPairBlocks) {
        double s = 0.0;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += kPairBlocks * 256) s = fma(double(E[i]), double(F[i]), s);
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
        return;
    }
    const int c = int(blockIdx.x) - kPairBlocks;
    if (c == ncores) {
        for (int i = threadIdx.x; i < nwords; i += 256) {
            unsigned m = 0u;
            for (int l = 0; l < kMaxLanes; ++l) m = max(m, words[i * kMaxLanes + l]);
            wmax_out[i] = m;
        }
        return;
    }
    const unsigned* w = slots + size_t(c) * kCmaxSlots;
    unsigned m = 0u;
    for (int i = threadIdx.x; i < kCmaxSlots; i += 256) m = max(m, w[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, unsigned(__shfl_xor(int(m), o)));
    if ((threadIdx.x & 63) == 0) redu[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) cmax_out[c] = max(max(redu[0], redu[1]), max(redu[2], redu[3]));
}

// The zipper's scratch initialisation in one launch (two memsets were three fill launches, ~10 us of the
// 0.22 ms call): the constant [1.0f] and lane 0 of its max word, then zeros up to `bytes` (the max words and
// the core-max slots, which the products atomicMax into).
__global__ void __launch_bounds__(256) k_dot32_init(char* __restrict__ base, size_t zero_off, size_t bytes) {
    const size_t i0 = size_t(blockIdx.x) * 256 + threadIdx.x, stride = size_t(gridDim.x) * 256;
    if (i0 == 0) {
        reinterpret_cast<unsigned*>(base)[0] = 0x3f800000u;
        reinterpret_cast<unsigned*>(base)[1] = 0x3f800000u;
    }
    unsigned* z = reinterpret_cast<unsigned*>(base + zero_off);   // (zero_off, bytes: multiples of 4)
    for (size_t i = i0; i < bytes / 4; i += stride) z[i] = 0u;
}

// Device buffers of one zipper: fp32 environments E (left) / F (right), ping-pong per end; T per end; W:
//   [0, 512)      the closing partials (kPairBlocks doubles)
//   back words    cmax (2d: core maxima, X_k at k, Y_k at d+k), wmax (4d+2: the max words' values)  <- read back
//   one           the constant environment E_0 = F_d = [1.0f], then its max word (lane 0 = 1.0f)
//   max words     4d+2 words of kMaxLanes lanes: left env L(k) at k (1..m), right env R(k) at d+1+k (m..d-1),
//                 left T of core k at 2d+2+k, right T of core k at 3d+2+k
//   slots         2d arrays of kCmaxSlots words (X_k at k, Y_k at d+k)
struct Dot32Bufs {
    float *E0, *E1, *F0, *F1, *TL, *TR;
    char* W;
    size_t back_bytes;   // bytes read back from W
    size_t one_off;      // offset of the constant [1.0f] (followed by its max word)
    size_t zero_off;     // zeroed from here (the constant's lanes 1.. on)
    size_t zero_bytes;
    size_t words_off, slots_off;
};

constexpr size_t up256(size_t x) { return (x + 255) / 256 * 256; }

size_t dot32_layout(size_t d, const size_t* n, const size_t* rx, const size_t* ry, size_t off[7], Dot32Bufs& b) {
    size_t emax = 1, tmax = 1;
    for (size_t k = 0; k <= d; ++k) emax = std::max(emax, rx[k] * ry[k]);
    for (size_t k = 0; k < d; ++k) tmax = std::max(tmax, std::max(ry[k] * n[k] * rx[k + 1], rx[k] * n[k] * ry[k + 1]));
    const size_t nwords = 4 * d + 2;
    b.back_bytes = 8 * kPairBlocks + 4 * (2 * d + nwords);
    b.one_off = up256(b.back_bytes);
    b.words_off = b.one_off + up256(4 + 4 * kMaxLanes);
    b.slots_off = b.words_off + up256(4 * kMaxLanes * nwords);
    b.zero_off = b.one_off + 8;   // (the constant and lane 0 of its max word are set to 1.0f)
    const size_t wsz = b.slots_off + 2 * d * kCmaxSlots * 4;
    b.zero_bytes = wsz - b.zero_off;
    const size_t sz[7] = {emax * 4, emax * 4, emax * 4, emax * 4, tmax * 4, tmax * 4, wsz};
    size_t o = 0;
    for (int i = 0; i < 7; ++i) {
        off[i] = o;
        o += up256(sz[i]);
    }
    return o;
}

// Start of the per-product steps: left cores from kl (environment El at edge kl, row stride lde, its max word is
// L(kl)), right cores from kr down (Fr at edge kr + 1, stride ldf, max word R(kr + 1)); kl = 0 / kr = d - 1 with
// null environments start from E_0 = F_d = [1].
struct Dot32Start {
    size_t kl = 0, kr = size_t(-1);
    const float* El = nullptr;
    const float* Fr = nullptr;
    size_t lde = 0, ldf = 0;
};

// the zeroing of the words and slots (before anything writes them: a front end's kernels atomicMax into them)
void dot32_init(xrs_handle_t h, const Dot32Bufs& bf) {
    const size_t zoff = bf.zero_off - bf.one_off;
    XRS_REQUIRE(zoff % 4 == 0 && bf.zero_bytes % 4 == 0, "fp32 zipper: misaligned scratch");
    const unsigned blocks = unsigned(std::min<size_t>((bf.zero_bytes / 4 + 255) / 256, 256));
    hipLaunchKernelGGL(k_dot32_init, dim3(std::max(1u, blocks)), dim3(256), 0, h->stream, bf.W + bf.one_off, zoff, bf.zero_bytes);
    check_launch("k_dot32_init");
}

// enqueues the zipper on h->stream (+ its side stream 0) up to the closing partial sums in b.W (dot32_init first)
void dot32_enqueue(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
                   const double* const* Y, const Dot32Bufs& bf, const Dot32Start& st = Dot32Start{}) {
    const size_t m = d / 2;
    const size_t kl = st.kl, kr = st.kr == size_t(-1) ? d - 1 : st.kr;
    float *E = bf.E0, *En = bf.E1, *F = bf.F0, *Fn = bf.F1;
    double* res = reinterpret_cast<double*>(bf.W);
    unsigned* cmax = reinterpret_cast<unsigned*>(bf.W + 8 * kPairBlocks);
    unsigned* wmax = cmax + 2 * d;
    float* one = reinterpret_cast<float*>(bf.W + bf.one_off);
    const unsigned* one_max = reinterpret_cast<const unsigned*>(one + 1);
    unsigned* words = reinterpret_cast<unsigned*>(bf.W + bf.words_off);
    unsigned* slots = reinterpret_cast<unsigned*>(bf.W + bf.slots_off);
    auto word = [&](size_t i) { return words + i * kMaxLanes; };
    auto L = [&](size_t k) -> unsigned* { return word(k); };
    auto R = [&](size_t k) -> unsigned* { return word(d + 1 + k); };
    auto TLw = [&](size_t k) { return word(2 * d + 2 + k); };
    auto TRw = [&](size_t k) { return word(3 * d + 2 + k); };
    auto sx = [&](size_t k) { return slots + k * kCmaxSlots; };
    auto sy = [&](size_t k) { return slots + (d + k) * kCmaxSlots; };
    {
        StreamFork fork(h);
        // left end (cores 0..m-1) on the side stream, right end (cores d-1..m) on the main stream; launches
        // interleaved step by step so that both streams have work from the start (the host's enqueue rate,
        // not the GPU, paces a chain of small launches). Every product has one raw core and one operand
        // normalised by its max word; E_0 = F_d = [1].
        const size_t nl = m - kl, nr = kr + 1 - m;   // steps per end
        for (size_t s = 0; s < std::max(nl, nr); ++s) {
            if (s < nl) {
                fork.side();
                const size_t k = kl + s;
                const size_t a = rx[k], b = ry[k], nk = n[k], a2 = rx[k + 1], b2 = ry[k + 1];
                const bool first = s == 0;
                const float* Ek = first ? (st.El ? st.El : one) : E;
                const size_t lda = first && st.El ? st.lde : b;
                // T (b x nk a2) = 2^-e E^T X_k
                SgemmExtra xt;
                xt.sa = (first && !st.El) ? one_max : L(k);
                xt.amax = TLw(k);
                xt.cmax_b = sx(k);
                sgemm<float, double>(h, bf.TL, b, nk * a2, 1.0f, Ek, lda, true, a, X[k], nk * a2, false, xt);
                // E' (a2 x b2) = (2^-e T)^T ((b nk) x a2)^T Y_k ((b nk) x b2)
                SgemmExtra xe;
                xe.sa = TLw(k);
                xe.amax = L(k + 1);
                xe.cmax_b = sy(k);
                sgemm<float, double>(h, En, a2, b2, 1.0f, bf.TL, a2, true, b * nk, Y[k], b2, false, xe);
                std::swap(E, En);
            }
            if (s < nr) {
                fork.main();
                const size_t k = kr - s;
                const size_t a = rx[k], b = ry[k], nk = n[k], a2 = rx[k + 1], b2 = ry[k + 1];
                const bool first = s == 0;
                const float* Fk = first ? (st.Fr ? st.Fr : one) : F;
                const size_t ldb = first && st.Fr ? st.ldf : b2;
                // T (a nk x b2) = X_k (a nk x a2) 2^-e F
                SgemmExtra xt;
                xt.sb = (first && !st.Fr) ? one_max : R(k + 1);
                xt.amax = TRw(k);
                xt.cmax_a = sx(k);
                sgemm<double, float>(h, bf.TR, a * nk, b2, 1.0f, X[k], a2, false, a2, Fk, ldb, false, xt);
                // F' (a x b) = (2^-e T) (a x nk b2) Y_k^T
                SgemmExtra xe;
                xe.sa = TRw(k);
                xe.amax = R(k);
                xe.cmax_b = sy(k);
                sgemm<float, double>(h, Fn, a, b, 1.0f, bf.TR, nk * b2, false, nk * b2, Y[k], nk * b2, true, xe);
                std::swap(F, Fn);
            }
        }
        fork.join();
    }
    hipLaunchKernelGGL(k_dot32_finish, dim3(kPairBlocks + 2 * d + 1), dim3(256), 0, h->stream, E, F, int(rx[m] * ry[m]), res,
                       slots, int(2 * d), cmax, words, int(4 * d + 2), wmax);
    check_launch("k_dot32_finish");
}

}  // namespace

double dot_f32(xrs_handle_t h, size_t d, const size_t* n, const size_t* rx, const double* const* X, const size_t* ry,
               const double* const* Y) {
    XRS_REQUIRE(d >= 2 && d <= 2048, "the fp32 zipper takes 2..2048 components");
    for (size_t k = 0; k <= d; ++k) XRS_REQUIRE(rx[k] * ry[k] < (size_t(1) << 30), "fp32 zipper: rank product too large");
    // zip32.hip's fused forms, opt-in (r06, one box, tools/dot32_probe.py: this per-product form 0.215 ms,
    // XRS_ZIP32=1 -- fused front end, then these steps -- 0.219-0.225 ms, XRS_ZIP32=2 -- fused steps throughout --
    // 0.258 ms; profiles/r06/zip32_ab_r06.txt)
    static const bool no_zip = [] {
        const char* e = std::getenv("XRS_ZIP32");
        return !(e && e[0] == '1');
    }();
    // XRS_ZIP32=2: the fused zipper for every step (zip32.hip; measured slower per full-rank step than the
    // per-product launches below, kept for A/B runs)
    static const bool all_zip = [] {
        const char* e = std::getenv("XRS_ZIP32");
        return e && e[0] == '2';
    }();
    if (all_zip && zip::applicable(d, n, rx, X, ry, Y)) return zip::dot(h, d, n, rx, X, ry, Y);
    const bool use_front = !no_zip && zip::front_applicable(d, n, rx, X, ry, Y);
    const size_t m = d / 2;
    size_t off[7];
    Dot32Bufs b{};
    DevBuf mem(h, dot32_layout(d, n, rx, ry, off, b));
    char* base = mem.as<char>();
    auto f = [&](int i) { return reinterpret_cast<float*>(base + off[i]); };
    b.E0 = f(0), b.E1 = f(1), b.F0 = f(2), b.F1 = f(3), b.TL = f(4), b.TR = f(5);
    b.W = base + off[6];
    dot32_init(h, b);
    // the front end (zip32.hip: E_1 / F_{d-1} and the rank r_1 -> r_2 step of each end in fused launches) where the
    // shapes allow it, then the per-product steps from core 2 / d - 3
    zip::Front fr;
    Dot32Start st;
    if (use_front) {
        unsigned* words = reinterpret_cast<unsigned*>(b.W + b.words_off);
        fr.mword[0] = words + 2 * kMaxLanes;                    // L(2)
        fr.mword[1] = words + (d + 1 + d - 2) * kMaxLanes;      // R(d - 2)
        fr.slots = reinterpret_cast<unsigned*>(b.W + b.slots_off);
        zip::front(h, d, n, rx, X, ry, Y, fr);
        st.kl = 2, st.El = fr.E, st.lde = fr.lde;
        st.kr = d - 3, st.Fr = fr.F, st.ldf = fr.ldf;
    }
    dot32_enqueue(h, d, n, rx, X, ry, Y, b, st);
    // read back the closing sum, the core maxima and the max words' values (+ the front end's exponent words)
    char* hs = static_cast<char*>(h->host_scratch);
    const size_t zoff = (b.back_bytes + 255) / 256 * 256;
    XRS_REQUIRE(zoff + 16 * d <= (size_t(1) << 16), "fp32 zipper: read-back exceeds the host scratch");
    XRS_HIP(hipMemcpyAsync(hs, b.W, b.back_bytes, hipMemcpyDeviceToHost, h->stream));
    if (use_front) XRS_HIP(hipMemcpyAsync(hs + zoff, fr.words, 16 * d, hipMemcpyDeviceToHost, h->stream));
    host_wait(h);
    const int* zw = reinterpret_cast<const int*>(hs + zoff);
    if (use_front && zip::front_words_bad(zw, d)) return tt::dot(h, d, n, rx, X, ry, Y);
    const unsigned* hc = reinterpret_cast<const unsigned*>(hs + 8 * kPairBlocks);
    const unsigned* hw = hc + 2 * d;
    // every core's max|.| in [2^-100, 2^100) or zero, else the fp64 zipper
    for (size_t c = 0; c < 2 * d; ++c) {
        const unsigned bits = hc[c];
        const int e = int((bits >> 23) & 0xff) - 127;   // floor(log2 max)
        // (the front end's step reads cores 1 and d-2 in fp32: a zero max there may be an underflowed core)
        const size_t k = c % d;
        const bool front_core = use_front && (k == 1 || k == d - 2);
        if ((bits != 0u || front_core) && (bits == 0u || bits >= 0x7f800000u || e < -100 || e >= 100))
            return tt::dot(h, d, n, rx, X, ry, Y);
    }
    // a product that left the fp32 range anyway (a max word or the closing sum not finite: products bounded
    // by (n r)^2 max|core|^2 can still overflow at rank products near the 2^30 limit): the fp64 zipper
    for (size_t i = 0; i < 4 * d + 2; ++i)
        if (hw[i] >= 0x7f800000u) return tt::dot(h, d, n, rx, X, ry, Y);
    double v = 0.0;
    for (int blk = 0; blk < kPairBlocks; ++blk) {
        double p;
        std::memcpy(&p, hs + 8 * blk, 8);
        v += p;
    }
    if (!std::isfinite(v)) return tt::dot(h, d, n, rx, X, ry, Y);
    // the powers of two the products scaled their normalised operands by: left E_k (k = 1..m-1; E_0 = [1]:
    // 2^-1) and T of cores 0..m-1, right F_k (k = m+1..d-1; F_d = [1]: 2^-1) and T of cores m..d-1; with the front
    // end: its own exponents for cores 0, 1 / d-1, d-2, then the words from E_2 / T of core 2 (F_{d-2} / core d-3) on
    int e = 0;
    const size_t kl = use_front ? 2 : 1, kr = use_front ? d - 1 : d;   // (words L(kl..m-1), R(m+1..kr-1))
    if (use_front) e += zip::front_exponent(zw, d, 0) + zip::front_exponent(zw, d, 1);
    else e += 2 * pow2_exponent(0x3f800000u);
    for (size_t k = kl; k < m; ++k) e += pow2_exponent(hw[k]);
    for (size_t k = m + 1; k < kr; ++k) e += pow2_exponent(hw[d + 1 + k]);
    for (size_t k = 0; k < d; ++k) {
        if (use_front && (k < 2 || k + 2 >= d)) continue;
        e += pow2_exponent(hw[(k < m ? 2 * d + 2 : 3 * d + 2) + k]);
    }
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
