// Mode permutation (xerus `reshuffle`, indexedTensor_tensor_evaluate.cpp:55-143) for gfx950.
//
// Plan (host): drop size-1 modes, merge old modes that stay adjacent and in order (the reference
// only keeps the trailing identity block, :64-72; merging every such run is the general form).
// Then either
//   (a) the innermost mode stays innermost -> row-block copy (16-B vector loads/stores), or
//   (b) a batched 2-D transpose between the input-contiguous mode `a` and the output-contiguous
//       mode `b`: 32x32 fp64 tiles staged through LDS ([32][33] padding: conflict-free ds_read_b64
//       columns), coalesced 256-B row segments on both the HBM read and the HBM write; or
//       64x64 tiles with 16-B accesses when both modes span whole tiles and everything is 16-B aligned;
//   (c) when those modes are shorter than a tile, the same transpose between GROUPS of innermost
//       input / output modes (flattened indices), so small modes still fill whole tiles.
// Both are HBM-bound: algorithmic bytes = 2 * size * 8.
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdlib>
#include <numeric>

#include "runtime.hpp"

namespace xrs {

constexpr int kMaxModes = 16;

struct PermPlan {
    int n = 0;                 // modes after simplification
    size_t dims[kMaxModes];    // input order
    size_t out_stride[kMaxModes];  // output stride of each OLD (input-order) mode
    size_t total = 1;
};

// Shuffle semantics: shuffle[i] = new position of old mode i.
static PermPlan make_plan(size_t ndim, const size_t* dims, const size_t* shuffle) {
    XRS_REQUIRE(ndim <= 64, "too many modes");
    std::vector<char> seen(ndim, 0);
    for (size_t i = 0; i < ndim; ++i) {
        XRS_REQUIRE(shuffle[i] < ndim && !seen[shuffle[i]], "shuffle is not a permutation");
        seen[shuffle[i]] = 1;
    }
    // drop size-1 modes, keep relative order of new positions
    std::vector<size_t> d, p;
    for (size_t i = 0; i < ndim; ++i) {
        if (dims[i] != 1) {
            d.push_back(dims[i]);
            p.push_back(shuffle[i]);
        }
    }
    // renumber new positions densely
    {
        std::vector<size_t> order(p.size());
        std::iota(order.begin(), order.end(), 0);
        std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return p[a] < p[b]; });
        for (size_t r = 0; r < order.size(); ++r) p[order[r]] = r;
    }
    // merge old modes i-1, i when p[i] == p[i-1] + 1 (they stay adjacent and ordered);
    // each run is represented by the new position of its first mode
    std::vector<size_t> md, mp;
    for (size_t i = 0; i < d.size(); ++i) {
        if (i > 0 && p[i] == p[i - 1] + 1) {
            md.back() *= d[i];
        } else {
            md.push_back(d[i]);
            mp.push_back(p[i]);
        }
    }
    // runs occupy disjoint contiguous ranges of new positions: rank them by their first position
    {
        std::vector<size_t> order(mp.size());
        std::iota(order.begin(), order.end(), 0);
        std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return mp[a] < mp[b]; });
        for (size_t r = 0; r < order.size(); ++r) mp[order[r]] = r;
    }
    PermPlan plan;
    plan.n = static_cast<int>(md.size());
    XRS_REQUIRE(plan.n <= kMaxModes, "permutation has too many non-mergeable modes");
    // output dims in new order
    std::vector<size_t> od(md.size());
    for (size_t i = 0; i < md.size(); ++i) od[mp[i]] = md[i];
    std::vector<size_t> ostr(md.size(), 1);
    for (int k = static_cast<int>(md.size()) - 2; k >= 0; --k) ostr[k] = ostr[k + 1] * od[k + 1];
    for (size_t i = 0; i < md.size(); ++i) {
        plan.dims[i] = md[i];
        plan.out_stride[i] = ostr[mp[i]];
        plan.total *= md[i];
    }
    return plan;
}

// ------------------------------------------------------------------------------------------
// (a) row-block copy: rows of L contiguous elements in input order.
struct RowArgs {
    int nb;                        // number of batch (outer) modes = n-1
    size_t dims[kMaxModes];        // outer dims (input order)
    size_t ostr[kMaxModes];        // output stride of each outer mode
    size_t L;                      // row length
    size_t rows;
};

__global__ void __launch_bounds__(256) k_permute_rows(double* __restrict__ out, const double* __restrict__ in, RowArgs a) {
    // one wave per row chunk; grid-stride over rows
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (size_t(gridDim.x) * blockDim.x) >> 6;
    for (size_t r = wave; r < a.rows; r += nwaves) {
        size_t rem = r, off = 0;
        for (int k = a.nb - 1; k >= 0; --k) {
            const size_t i = rem % a.dims[k];
            rem /= a.dims[k];
            off += i * a.ostr[k];
        }
        const double* src = in + r * a.L;
        double* dst = out + off;
        const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0 && (a.L & 1) == 0;
        if (vec) {
            const double2* s2 = reinterpret_cast<const double2*>(src);
            double2* d2 = reinterpret_cast<double2*>(dst);
            for (size_t j = lane; j < a.L / 2; j += 64) d2[j] = s2[j];
        } else {
            for (size_t j = lane; j < a.L; j += 64) dst[j] = src[j];
        }
    }
}

// ------------------------------------------------------------------------------------------
// (b) batched transpose of modes a (input fastest, index ia) and b (output fastest, index ib).
struct TrArgs {
    size_t da, db;                 // extents
    size_t in_sb;                  // input stride of mode b
    size_t out_sa;                 // output stride of mode a
    int nb;                        // batch modes
    size_t bdims[kMaxModes];
    size_t bin_str[kMaxModes];
    size_t bout_str[kMaxModes];
    unsigned tiles_a, tiles_b;
};

constexpr int TT = 32;

__global__ void __launch_bounds__(256) k_permute_transpose(double* __restrict__ out, const double* __restrict__ in, TrArgs a, size_t batch) {
    __shared__ double tile[TT][TT + 1];
    const unsigned t = blockIdx.x;
    const unsigned ta = t % a.tiles_a;
    const unsigned tb = t / a.tiles_a;
    const size_t a0 = size_t(ta) * TT, b0 = size_t(tb) * TT;
    const int tx = threadIdx.x & 31;   // fast index
    const int ty = threadIdx.x >> 5;   // 0..7
    for (size_t bi = blockIdx.y; bi < batch; bi += gridDim.y) {
        unsigned rem = unsigned(bi);   // batch < 2^32 (host check)
        size_t ioff = 0, ooff = 0;
        for (int k = a.nb - 1; k >= 0; --k) {
            const unsigned dk = unsigned(a.bdims[k]), q = rem / dk, i = rem - q * dk;
            rem = q;
            ioff += size_t(i) * a.bin_str[k];
            ooff += size_t(i) * a.bout_str[k];
        }
        // read: rows along b, contiguous along a
#pragma unroll
        for (int j = 0; j < TT; j += 8) {
            const size_t ib = b0 + ty + j, ia = a0 + tx;
            if (ib < a.db && ia < a.da) tile[ty + j][tx] = in[ioff + ib * a.in_sb + ia];
        }
        __syncthreads();
        // write: rows along a, contiguous along b
#pragma unroll
        for (int j = 0; j < TT; j += 8) {
            const size_t ia = a0 + ty + j, ib = b0 + tx;
            if (ib < a.db && ia < a.da) out[ooff + ia * a.out_sa + ib] = tile[tx][ty + j];
        }
        __syncthreads();
    }
}

// (b') the same batched transpose with 64 x 64 tiles and 16-B accesses, for aligned operands whose two
// modes span whole tiles (da, db % 64 == 0, even strides and offsets): a wave moves 1 KB per instruction
// (two 512-B row segments), each thread keeps 8 loads in flight (32 KB per workgroup per round trip)
// instead of 4 x 8 B -- the mid-size transposes (16-21 MB) are bound by that round trip, not by HBM.
// LDS rows of 65 doubles: the column reads of ds_read_b64 (row stride 130 banks) hit distinct bank pairs.
constexpr int TW = 64;
typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_permute_transpose64(double* __restrict__ out, const double* __restrict__ in, TrArgs a,
                                                             size_t batch) {
    __shared__ double tile[TW][TW + 1];
    const unsigned t = blockIdx.x;
    const size_t a0 = size_t(t % a.tiles_a) * TW, b0 = size_t(t / a.tiles_a) * TW;
    const int tx = threadIdx.x & 31;   // double2 column within a 64-wide row
    const int ty = threadIdx.x >> 5;   // 0..7
    for (size_t bi = blockIdx.y; bi < batch; bi += gridDim.y) {
        unsigned rem = unsigned(bi);
        size_t ioff = 0, ooff = 0;
        for (int k = a.nb - 1; k >= 0; --k) {
            const unsigned dk = unsigned(a.bdims[k]), q = rem / dk, i = rem - q * dk;
            rem = q;
            ioff += size_t(i) * a.bin_str[k];
            ooff += size_t(i) * a.bout_str[k];
        }
        dv2 v[TW / 8];
#pragma unroll
        for (int j = 0; j < TW / 8; ++j)   // input rows along b, 16 B per lane along a
            v[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(in + ioff + (b0 + ty + 8 * j) * a.in_sb + a0) + tx);
#pragma unroll
        for (int j = 0; j < TW / 8; ++j) {
            tile[ty + 8 * j][2 * tx] = v[j].x;
            tile[ty + 8 * j][2 * tx + 1] = v[j].y;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TW / 8; ++j) {   // output rows along a, 16 B per lane along b
            dv2 w;
            w.x = tile[2 * tx][ty + 8 * j];
            w.y = tile[2 * tx + 1][ty + 8 * j];
            __builtin_nontemporal_store(w, reinterpret_cast<dv2*>(out + ooff + (a0 + ty + 8 * j) * a.out_sa + b0) + tx);
        }
        __syncthreads();
    }
}

// (c) the same tiled transpose between GROUPS of modes: a = the innermost input modes (contiguous in the
// input, flattened index fa), b = the innermost output modes (contiguous in the output, index fb). Small
// modes (the 20^6 reversal: 20 x 20 = 400) then fill whole 32 x 32 tiles instead of 20 x 20 of them.
constexpr int kGroupMax = 4;
struct GrArgs {
    int na, nbm;                        // modes in the a / b groups
    size_t adims[kGroupMax], aout[kGroupMax];   // a group, input-fastest first: extent, output stride
    size_t bdims[kGroupMax], bin[kGroupMax];    // b group, output-fastest first: extent, input stride
    size_t pa, pb;                      // flattened extents
    int nbatch;
    size_t bdim[kMaxModes], bin_str[kMaxModes], bout_str[kMaxModes];
    unsigned tiles_a, tiles_b;
};

__global__ void __launch_bounds__(256) k_permute_grouped(double* __restrict__ out, const double* __restrict__ in, GrArgs a, size_t batch) {
    __shared__ double tile[TT][TT + 1];
    const unsigned t = blockIdx.x;
    const size_t a0 = size_t(t % a.tiles_a) * TT, b0 = size_t(t / a.tiles_a) * TT;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    // per-row offsets: input offset of b rows, output offset of a rows (4 rows per thread each)
    size_t boff[TT / 8], aoff[TT / 8];
#pragma unroll
    for (int j = 0; j < TT / 8; ++j) {   // 32-bit index arithmetic (flattened group extents < 2^32)
        unsigned fb = unsigned(b0) + ty + 8 * j, fa = unsigned(a0) + ty + 8 * j;
        size_t ob = 0, oa = 0;
        for (int k = 0; k < a.nbm; ++k) {
            const unsigned dk = unsigned(a.bdims[k]), q = fb / dk;
            ob += size_t(fb - q * dk) * a.bin[k];
            fb = q;
        }
        for (int k = 0; k < a.na; ++k) {
            const unsigned dk = unsigned(a.adims[k]), q = fa / dk;
            oa += size_t(fa - q * dk) * a.aout[k];
            fa = q;
        }
        boff[j] = ob;
        aoff[j] = oa;
    }
    for (size_t bi = blockIdx.y; bi < batch; bi += gridDim.y) {
        unsigned rem = unsigned(bi);   // batch < 2^32 (host check)
        size_t ioff = 0, ooff = 0;
        for (int k = a.nbatch - 1; k >= 0; --k) {
            const unsigned dk = unsigned(a.bdim[k]), q = rem / dk, i = rem - q * dk;
            rem = q;
            ioff += size_t(i) * a.bin_str[k];
            ooff += size_t(i) * a.bout_str[k];
        }
#pragma unroll
        for (int j = 0; j < TT / 8; ++j) {
            const size_t fb = b0 + ty + 8 * j, fa = a0 + tx;
            if (fb < a.pb && fa < a.pa) tile[ty + 8 * j][tx] = in[ioff + boff[j] + fa];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TT / 8; ++j) {
            const size_t fa = a0 + ty + 8 * j, fb = b0 + tx;
            if (fb < a.pb && fa < a.pa) out[ooff + aoff[j] + fb] = tile[tx][ty + 8 * j];
        }
        __syncthreads();
    }
}

void permute(xrs_handle_t h, double* out, const double* in, size_t ndim, const size_t* dims, const size_t* shuffle) {
    PermPlan p = make_plan(ndim, dims, shuffle);
    if (p.total == 0) return;
    const double bytes = 2.0 * double(p.total) * 8.0;
    if (p.n <= 1 || p.out_stride[p.n - 1] == 1) {
        if (p.n <= 1) {
            KernelTimer timer(h, XRS_KFAM_PERMUTE, 0.0, bytes);
            XRS_HIP(hipMemcpyAsync(out, in, p.total * 8, hipMemcpyDeviceToDevice, h->stream));
            return;
        }
        RowArgs ra{};
        ra.nb = p.n - 1;
        for (int k = 0; k < ra.nb; ++k) {
            ra.dims[k] = p.dims[k];
            ra.ostr[k] = p.out_stride[k];
        }
        ra.L = p.dims[p.n - 1];
        ra.rows = p.total / ra.L;
        const size_t waves = std::min<size_t>(ra.rows, 256 * 32);
        const unsigned blocks = unsigned((waves + 3) / 4);
        KernelTimer timer(h, XRS_KFAM_PERMUTE, 0.0, bytes, true);   // the dispatch's own timestamps
        hipExtLaunchKernelGGL(k_permute_rows, dim3(blocks), dim3(256), 0, h->stream, timer.start(), timer.stop(), 0, out, in, ra);
        check_launch("k_permute_rows");
        return;
    }
    // transpose case
    const int ma = p.n - 1;
    int mb = -1;
    for (int k = 0; k < p.n; ++k)
        if (p.out_stride[k] == 1) mb = k;
    XRS_REQUIRE(mb >= 0 && mb != ma, "internal: permutation plan");
    std::vector<size_t> in_str(p.n, 1);
    for (int k = p.n - 2; k >= 0; --k) in_str[k] = in_str[k + 1] * p.dims[k + 1];
    // groups: innermost input modes (a) and innermost output modes (b) until each spans >= one tile
    {
        std::vector<int> out_order(p.n);   // input-mode indices, output-fastest first
        std::iota(out_order.begin(), out_order.end(), 0);
        std::sort(out_order.begin(), out_order.end(), [&](int x, int y) { return p.out_stride[x] < p.out_stride[y]; });
        std::vector<char> inA(p.n, 0);
        std::vector<int> A, B;
        size_t pa = 1, pb = 1;
        for (int k = p.n - 1; k >= 0 && pa < size_t(TT) && int(A.size()) < kGroupMax && k != mb; --k) {
            A.push_back(k);
            inA[k] = 1;
            pa *= p.dims[k];
        }
        for (int r = 0; r < p.n && pb < size_t(TT) && int(B.size()) < kGroupMax && !inA[out_order[r]]; ++r) {
            B.push_back(out_order[r]);
            pb *= p.dims[out_order[r]];
        }
        if (A.size() > 1 || B.size() > 1) {
            GrArgs g{};
            g.na = int(A.size());
            g.nbm = int(B.size());
            for (int i = 0; i < g.na; ++i) {
                g.adims[i] = p.dims[A[i]];
                g.aout[i] = p.out_stride[A[i]];
            }
            for (int i = 0; i < g.nbm; ++i) {
                g.bdims[i] = p.dims[B[i]];
                g.bin[i] = in_str[B[i]];
            }
            g.pa = pa;
            g.pb = pb;
            std::vector<char> grouped(p.n, 0);
            for (int k : A) grouped[k] = 1;
            for (int k : B) grouped[k] = 1;
            size_t batch = 1;
            for (int k = 0; k < p.n; ++k) {
                if (grouped[k]) continue;
                g.bdim[g.nbatch] = p.dims[k];
                g.bin_str[g.nbatch] = in_str[k];
                g.bout_str[g.nbatch] = p.out_stride[k];
                ++g.nbatch;
                batch *= p.dims[k];
            }
            g.tiles_a = unsigned((pa + TT - 1) / TT);
            g.tiles_b = unsigned((pb + TT - 1) / TT);
            const size_t tiles = size_t(g.tiles_a) * g.tiles_b;
            XRS_REQUIRE(tiles < (1ull << 31) && batch < (1ull << 32) && pa < (1ull << 32) && pb < (1ull << 32), "permutation too large");
            // a few batch items per workgroup (the row offsets are computed once per workgroup)
            const unsigned gy = unsigned(std::max<size_t>(1, std::min<size_t>({batch, 65535, (size_t(1) << 13) / tiles})));
            KernelTimer timer(h, XRS_KFAM_PERMUTE, 0.0, bytes, true);
            hipExtLaunchKernelGGL(k_permute_grouped, dim3(unsigned(tiles), gy), dim3(256), 0, h->stream, timer.start(), timer.stop(), 0,
                                  out, in, g, batch);
            check_launch("k_permute_grouped");
            return;
        }
    }
    TrArgs ta{};
    ta.da = p.dims[ma];
    ta.db = p.dims[mb];
    ta.in_sb = in_str[mb];
    ta.out_sa = p.out_stride[ma];
    ta.nb = 0;
    size_t batch = 1;
    for (int k = 0; k < p.n; ++k) {
        if (k == ma || k == mb) continue;
        ta.bdims[ta.nb] = p.dims[k];
        ta.bin_str[ta.nb] = in_str[k];
        ta.bout_str[ta.nb] = p.out_stride[k];
        ++ta.nb;
        batch *= p.dims[k];
    }
    // 64 x 64 tiles with 16-B accesses when every row segment is a whole, 16-B aligned tile row
    bool wide = ta.da % TW == 0 && ta.db % TW == 0 && ta.in_sb % 2 == 0 && ta.out_sa % 2 == 0 &&
                ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    for (int k = 0; k < ta.nb; ++k) wide = wide && ta.bin_str[k] % 2 == 0 && ta.bout_str[k] % 2 == 0;
    const int tw = wide ? TW : TT;
    ta.tiles_a = unsigned((ta.da + tw - 1) / tw);
    ta.tiles_b = unsigned((ta.db + tw - 1) / tw);
    const size_t tiles = size_t(ta.tiles_a) * ta.tiles_b;
    XRS_REQUIRE(tiles < (1ull << 31) && batch < (1ull << 32), "permutation too large");
    const unsigned gy = unsigned(std::min<size_t>(batch, 65535));
    if (wide) {
        // (r06: the tile's two 32-row halves pipelined -- stores of one half under the other's loads -- measured
        // 6.1 -> 4.8 us at 1024^2 on one box and 4.9 -> 5.5 us on another, 45 -> 54 us at 4096^2 on both: not kept,
        // profiles/r06/permute_pipe_ab_r06.txt)
        KernelTimer timer(h, XRS_KFAM_PERMUTE, 0.0, bytes, true);
        hipExtLaunchKernelGGL(k_permute_transpose64, dim3(unsigned(tiles), gy), dim3(256), 0, h->stream, timer.start(), timer.stop(), 0,
                              out, in, ta, batch);
        check_launch("k_permute_transpose64");
        return;
    }
    KernelTimer timer(h, XRS_KFAM_PERMUTE, 0.0, bytes, true);
    hipExtLaunchKernelGGL(k_permute_transpose, dim3(unsigned(tiles), gy), dim3(256), 0, h->stream, timer.start(), timer.stop(), 0, out,
                          in, ta, batch);
    check_launch("k_permute_transpose");
}

}  // namespace xrs

extern "C" int xrs_permute(xrs_handle_t h, double* out, const double* in, size_t ndim, const size_t* dims,
                           const size_t* shuffle) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(ndim == 0 || (dims && shuffle), "null dims/shuffle");
        size_t total = 1;
        for (size_t i = 0; i < ndim; ++i) total *= dims[i];
        XRS_REQUIRE(total == 0 || (out && in), "null data pointer");
        XRS_REQUIRE(out != in || total <= 1, "out must not alias in");
        xrs::fence_readers(h);
        if (ndim == 0) {
            if (total) XRS_HIP(hipMemcpyAsync(out, in, 8, hipMemcpyDeviceToDevice, h->stream));
            return;
        }
        xrs::permute(h, out, in, ndim, dims, shuffle);
    });
}
