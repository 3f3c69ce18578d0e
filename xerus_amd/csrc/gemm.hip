// fp64 GEMM on CDNA4 matrix cores: C = alpha * op(A) * op(B), row-major, beta = 0.
// Replaces blasWrapper::matrix_matrix_product (blasLapackWrapper.cpp:149-195, cblas_dgemm :177-191).
//
// Kernel: 256 threads = 4 waves in a 2x2 arrangement, block tile BM x BN, K-step 16, operands staged
// k-major through LDS ([k][m] and [k][n]) with register double-buffering of the next K-step.
// Each wave owns a (BM/2) x (BN/2) sub-tile made of 16x16 v_mfma_f64_16x16x4_f64 tiles:
//   A operand: lane l holds A[row l&15][k l>>4]; B operand: B[k l>>4][col l&15];
//   C/D (f64 only): col = l&15, row = (l>>4) + 4*reg  (cdna_hip_programming.md §3).
// LDS row stride S = B? + 17 doubles (odd): transposed ds_write_b64 of the k-contiguous operands is
// conflict-free in each 16-lane group, and the k/k+1 fragment rows of ds_read_b64 overlap in one bank.
// Split-K (grid.z) writes fp64 partial slabs that a second kernel reduces in fixed order
// (bitwise reproducible), used when the M x N tile grid alone cannot fill 256 CUs (TT shapes:
// 256 x 256 outputs with K = n*r up to 10240).
#include <algorithm>

#include "runtime.hpp"

namespace xrs {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int GBK = 16;

template <int BM, int BN, bool TA, bool TB>
__global__ void __launch_bounds__(256)
k_gemm_f64(const double* __restrict__ A, size_t lda, const double* __restrict__ B, size_t ldb,
           double* __restrict__ C, int M, int N, int K, int kps, double alpha, double* __restrict__ slab,
           int tiles_m) {
    constexpr int SA = BM + 17;
    constexpr int SB = BN + 17;
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 16, TN = WN / 16;
    // per-thread staging counts (in doubles)
    constexpr int A_PER = BM * GBK / 256;
    constexpr int B_PER = BN * GBK / 256;

    __shared__ double As[2][GBK * SA];
    __shared__ double Bs[2][GBK * SB];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = (wave >> 1) * WM;
    const int wn = (wave & 1) * WN;

    const int tm = blockIdx.x % tiles_m;
    const int tn = blockIdx.x / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = blockIdx.z * kps;
    const int kend = min(K, kbeg + kps);

    d4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

    double ra[A_PER], rb[B_PER];

    // ---- global -> registers for the K-step starting at k0
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int e = 0; e < A_PER; ++e) {
            const int idx = tid + e * 256;
            int m, k;
            if (TA) {  // A stored K x M: contiguous along m
                m = idx % BM; k = idx / BM;
            } else {   // A stored M x K: contiguous along k
                k = idx % GBK; m = idx / GBK;
            }
            const int gm = m0 + m, gk = k0 + k;
            double v = 0.0;
            if (gm < M && gk < kend) v = TA ? A[size_t(gk) * lda + gm] : A[size_t(gm) * lda + gk];
            ra[e] = v;
        }
#pragma unroll
        for (int e = 0; e < B_PER; ++e) {
            const int idx = tid + e * 256;
            int n, k;
            if (TB) {  // B stored N x K: contiguous along k
                k = idx % GBK; n = idx / GBK;
            } else {   // B stored K x N: contiguous along n
                n = idx % BN; k = idx / BN;
            }
            const int gn = n0 + n, gk = k0 + k;
            double v = 0.0;
            if (gn < N && gk < kend) v = TB ? B[size_t(gn) * ldb + gk] : B[size_t(gk) * ldb + gn];
            rb[e] = v;
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int e = 0; e < A_PER; ++e) {
            const int idx = tid + e * 256;
            int m, k;
            if (TA) { m = idx % BM; k = idx / BM; } else { k = idx % GBK; m = idx / GBK; }
            As[buf][k * SA + m] = ra[e];
        }
#pragma unroll
        for (int e = 0; e < B_PER; ++e) {
            const int idx = tid + e * 256;
            int n, k;
            if (TB) { k = idx % GBK; n = idx / GBK; } else { n = idx % BN; k = idx / BN; }
            Bs[buf][k * SB + n] = rb[e];
        }
    };

    const int nsteps = (kend > kbeg) ? (kend - kbeg + GBK - 1) / GBK : 0;
    if (nsteps > 0) {
        load_tile(kbeg);
        store_tile(0);
        __syncthreads();
        const int lr = lane & 15, lk = lane >> 4;
        for (int s = 0; s < nsteps; ++s) {
            const int cur = s & 1;
            if (s + 1 < nsteps) load_tile(kbeg + (s + 1) * GBK);
            const double* as = As[cur];
            const double* bs = Bs[cur];
#pragma unroll
            for (int kk = 0; kk < GBK; kk += 4) {
                double af[TM], bf[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = as[(kk + lk) * SA + wm + i * 16 + lr];
#pragma unroll
                for (int j = 0; j < TN; ++j) bf[j] = bs[(kk + lk) * SB + wn + j * 16 + lr];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
            }
            if (s + 1 < nsteps) {
                store_tile(cur ^ 1);
            }
            __syncthreads();
        }
    }

    // ---- epilogue
    const bool to_slab = slab != nullptr;
    double* out = to_slab ? slab + size_t(blockIdx.z) * size_t(M) * size_t(N) : C;
    const double scale = to_slab ? 1.0 : alpha;
    const int lc = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn + j * 16 + lc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm + i * 16 + lg + 4 * r;
                if (row < M && col < N) out[size_t(row) * N + col] = scale * acc[i][j][r];
            }
        }
}

__global__ void __launch_bounds__(256) k_splitk_reduce(double* __restrict__ C, const double* __restrict__ slab, size_t MN,
                                                       int splits, double alpha) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < MN; i += stride) {
        double s = 0.0;
        for (int z = 0; z < splits; ++z) s += slab[size_t(z) * MN + i];
        C[i] = alpha * s;
    }
}

template <int BM, int BN>
static void launch_tiles(xrs_handle_t h, const double* A, size_t lda, bool ta, const double* B, size_t ldb, bool tb,
                         double* C, int M, int N, int K, int splits, int kps, double alpha, double* slab) {
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    dim3 grid(unsigned(tiles_m * tiles_n), 1, unsigned(splits));
    KernelTimer timer(h, XRS_KFAM_GEMM, 2.0 * double(M) * double(N) * double(K),
                      8.0 * (double(M) * K + double(K) * N + double(M) * N * splits));
#define XRS_GEMM_LAUNCH(TA_, TB_)                                                                             \
    hipLaunchKernelGGL((k_gemm_f64<BM, BN, TA_, TB_>), grid, dim3(256), 0, h->stream, A, lda, B, ldb, C, M, N, K, \
                       kps, alpha, slab, tiles_m)
    if (!ta && !tb) XRS_GEMM_LAUNCH(false, false);
    else if (!ta && tb) XRS_GEMM_LAUNCH(false, true);
    else if (ta && !tb) XRS_GEMM_LAUNCH(true, false);
    else XRS_GEMM_LAUNCH(true, true);
#undef XRS_GEMM_LAUNCH
    check_launch("k_gemm_f64");
}

void gemm(xrs_handle_t h, double* C, size_t Ms, size_t Ns, double alpha, const double* A, size_t lda, bool ta, size_t Ks,
          const double* B, size_t ldb, bool tb) {
    if (Ms == 0 || Ns == 0) return;
    XRS_REQUIRE(Ms < (1u << 30) && Ns < (1u << 30) && Ks < (1u << 30), "GEMM dimension too large");
    const int M = int(Ms), N = int(Ns), K = int(Ks);
    if (K == 0) {
        XRS_HIP(hipMemsetAsync(C, 0, size_t(M) * N * 8, h->stream));
        return;
    }
    // tile choice: 128x128 when that alone yields >= 256 tiles, else 64x64 (+ split-K)
    const long t128 = long((M + 127) / 128) * ((N + 127) / 128);
    const long t64 = long((M + 63) / 64) * ((N + 63) / 64);
    const bool big = t128 >= 240;
    const long tiles = big ? t128 : t64;
    int splits = 1;
    if (tiles < 256) {
        // split K so that tiles*splits ~ 256-512 blocks while each split keeps >= 128 of K
        const long want = (512 + tiles - 1) / tiles;
        const long maxs = std::max<long>(1, K / 128);
        splits = int(std::max<long>(1, std::min(want, maxs)));
    }
    int kps = (K + splits - 1) / splits;
    kps = (kps + GBK - 1) / GBK * GBK;
    splits = (K + kps - 1) / kps;
    DevBuf slab;
    if (splits > 1) slab = DevBuf(h, size_t(splits) * M * N * sizeof(double));
    if (big)
        launch_tiles<128, 128>(h, A, lda, ta, B, ldb, tb, C, M, N, K, splits, kps, alpha, slab.d());
    else
        launch_tiles<64, 64>(h, A, lda, ta, B, ldb, tb, C, M, N, K, splits, kps, alpha, slab.d());
    if (splits > 1) {
        const size_t MN = size_t(M) * N;
        const unsigned blocks = unsigned(std::min<size_t>((MN + 255) / 256, 4096));
        KernelTimer timer(h, XRS_KFAM_ELEMWISE, double(MN) * splits, 8.0 * double(MN) * (splits + 1));
        hipLaunchKernelGGL(k_splitk_reduce, dim3(blocks), dim3(256), 0, h->stream, C, slab.d(), MN, splits, alpha);
        check_launch("k_splitk_reduce");
    }
}

}  // namespace xrs

extern "C" int xrs_gemm(xrs_handle_t h, double* C, size_t M, size_t N, double alpha, const double* A, size_t lda,
                        int transA, size_t K, const double* B, size_t ldb, int transB) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(M == 0 || N == 0 || C, "null C");
        XRS_REQUIRE(K == 0 || M == 0 || N == 0 || (A && B), "null A/B");
        XRS_REQUIRE(transA ? lda >= M || K == 0 : lda >= K || M == 0, "lda too small");
        XRS_REQUIRE(transB ? ldb >= K || N == 0 : ldb >= N || K == 0, "ldb too small");
        XRS_REQUIRE(C != A && C != B, "C must not alias A or B");
        xrs::gemm(h, C, M, N, alpha, A, lda, transA != 0, K, B, ldb, transB != 0);
    });
}
