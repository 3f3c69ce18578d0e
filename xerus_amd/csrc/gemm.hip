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
// Split-K (grid.z) writes fp64 partial slabs that the last-arriving slice of each tile sums in fixed
// order (bitwise reproducible) inside the same launch, used when the M x N tile grid alone cannot fill
// 256 CUs (TT shapes: 256 x 256 outputs with K = n*r up to 10240).
#include <algorithm>
#include <type_traits>
#include <utility>
#include <cstdio>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "elementwise.hpp"
#include "runtime.hpp"

namespace xrs {

typedef double d4 __attribute__((ext_vector_type(4)));

// Operand tables: one GEMM, or a batch of same-shape GEMMs (blockIdx.y = batch entry) in one launch.
struct GemmOne {
    const double* A;
    const double* B;
    double* C;
    __host__ __device__ const double* a(int) const { return A; }
    __host__ __device__ const double* b(int) const { return B; }
    __device__ double* c(int) const { return C; }
};
struct GemmMany {
    const double* A[kGemmBatchMax];
    const double* B[kGemmBatchMax];
    double* C[kGemmBatchMax];
    __host__ __device__ const double* a(int i) const { return A[i]; }
    __host__ __device__ const double* b(int i) const { return B[i]; }
    __device__ double* c(int i) const { return C[i]; }
};

// Occupancy hint: the second __launch_bounds__ argument is the minimum number of waves per SIMD. Two
// 8-wave workgroups per CU need 4 (a 128-VGPR budget); the 128x128 tile keeps 2 (256 VGPRs, 1 per CU).
template <int BM, int BN, int WGM, int WGN, int WGK>
constexpr int gemm_min_waves() { return (BM * BN >= 128 * 128) ? 2 : 4; }

#ifdef XRS_GEMM_TRACE
// Diagnostic build only (tools/gemm_trace.py): per workgroup {start, end, XCC_ID << 32 | HW_ID} in
// s_memrealtime ticks (100 MHz), written by thread 0 of each workgroup.
__device__ unsigned long long* g_gemm_trace = nullptr;
__device__ unsigned long long* g_gemm_steps = nullptr;   // glds kernel: s_memtime after each K-step barrier
#define XRS_TRACE_BEGIN                                                   \
    const unsigned long long xrs_t0 = __builtin_amdgcn_s_memrealtime();  \
    const unsigned long long xrs_c0 = __builtin_amdgcn_s_memtime();
#define XRS_TRACE_STEP(t)                                                                                   \
    if (threadIdx.x == 0 && g_gemm_steps != nullptr && (t) < 15) {                                          \
        const size_t wg = blockIdx.x + size_t(gridDim.x) * (blockIdx.y + size_t(gridDim.y) * blockIdx.z);   \
        g_gemm_steps[16 * wg + (t)] = __builtin_amdgcn_s_memtime() - xrs_c0;                                \
    }
#define XRS_TRACE_END                                                                                     \
    if (threadIdx.x == 0 && g_gemm_trace != nullptr) {                                                    \
        const size_t wg = blockIdx.x + size_t(gridDim.x) * (blockIdx.y + size_t(gridDim.y) * blockIdx.z); \
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();                                   \
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    /* HW_REG_HW_ID */             \
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  /* HW_REG_XCC_ID */            \
        g_gemm_trace[3 * wg] = xrs_t0;                                                                   \
        g_gemm_trace[3 * wg + 1] = t1;                                                                   \
        g_gemm_trace[3 * wg + 2] = (static_cast<unsigned long long>(xcc) << 32) | hw;                    \
        if (g_gemm_steps != nullptr) g_gemm_steps[16 * wg + 15] = __builtin_amdgcn_s_memtime() - xrs_c0;  \
    }
#else
#define XRS_TRACE_BEGIN
#define XRS_TRACE_END
#define XRS_TRACE_STEP(t)
#endif

template <int BM, int BN, int GBK, int WGM, int WGN, int WGK, int PD, bool TA, bool TB, class PTR>
__device__ __forceinline__ void gemm_body(const PTR& ptrs, size_t lda, size_t ldb, int M, int N, int K, int kps,
                                          double alpha, double* __restrict__ slab, int tiles_m, int xcd_group,
                                          int* __restrict__ tickets, int sym);

template <int BM, int BN, int GBK, int WGM, int WGN, int WGK, int PD, bool TA, bool TB, class PTR>
__global__ void __launch_bounds__(WGM * WGN * WGK * 64, (gemm_min_waves<BM, BN, WGM, WGN, WGK>()))
k_gemm_f64(const PTR ptrs, size_t lda, size_t ldb, int M, int N, int K, int kps, double alpha,
           double* __restrict__ slab, int tiles_m, int xcd_group, int* __restrict__ tickets, int sym) {
    XRS_TRACE_BEGIN
    gemm_body<BM, BN, GBK, WGM, WGN, WGK, PD, TA, TB, PTR>(ptrs, lda, ldb, M, N, K, kps, alpha, slab, tiles_m,
                                                          xcd_group, tickets, sym);
    XRS_TRACE_END
}

// Accumulators -> C: sums the NACC accumulator sets, reduces the WGK wave groups through LDS (`lds`, at
// least (WGK-1) * WGM * WGN * TM * TN * 256 doubles, free to overwrite), then stores C (alpha, symmetric
// mirror), a split-K slab, or a slab + the in-launch combine (tickets). Shared by both GEMM kernels.
// xb / yb / zb: the workgroup's tile index, batch entry and split-K slice (blockIdx.x / .y / .z, or the
// XCD-grouped mapping of k_gemm_glds)
template <int TM, int TN, int WGM, int WGN, int WGK, int NACC, class PTR>
__device__ __forceinline__ void gemm_finish(d4 (&acc2)[NACC][TM][TN], double* lds, const PTR& ptrs, int M, int N,
                                            double alpha, double* __restrict__ slab, int* __restrict__ tickets,
                                            int sym, int m0, int n0, int wm, int wn, int kg, int pos, int xb, int yb, int zb) {
    const int bz = yb;
    double* __restrict__ C = ptrs.c(bz);
    const int zslice = bz * int(gridDim.z) + zb;
    const int tslot = bz * int(gridDim.x) + xb;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const bool mirror = sym != 0;
    d4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            acc[i][j] = acc2[0][i][j];
            if constexpr (NACC > 1) acc[i][j] += acc2[1][i][j];
        }
    // ---- intra-workgroup K reduction (wave groups 1.. -> LDS -> group 0)
    if constexpr (WGK > 1) {
        double* red = lds;
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
        if (kg > 0 && tickets == nullptr) return;   // (with tickets every wave stays for the barriers below)
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
    // ---- epilogue
    const bool to_slab = slab != nullptr;
    const size_t MN = size_t(M) * size_t(N);
    double* out = to_slab ? slab + size_t(zslice) * MN : C;
    const double scale = to_slab ? 1.0 : alpha;
    const int lc = lane & 15, lg = lane >> 4;
    if (kg == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = n0 + wn + j * 16 + lc;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm + i * 16 + lg + 4 * r;
                    if (row < M && col < N) {
                        if (tickets != nullptr)   // write-through (sc1): visible to any XCD without a release fence
                            __hip_atomic_store(&out[size_t(row) * N + col], acc[i][j][r], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        else if (!mirror || to_slab)
                            out[size_t(row) * N + col] = scale * acc[i][j][r];
                        else if (row >= col) {
                            out[size_t(row) * N + col] = scale * acc[i][j][r];
                            out[size_t(col) * N + row] = scale * acc[i][j][r];
                        }
                    }
                }
            }
    }
    if (tickets == nullptr) return;
    // ---- in-launch split-K combine (cdna_hip_programming.md §5 projection-GEMM item 2, sc1 form): every
    // slice stores its slab write-through (sc1, above), drains its stores and draws a ticket; the slice
    // that draws splits-1 reads the other slabs with sc1 loads (no fences anywhere) and sums them in
    // slice order 0..splits-1 -- the order of k_splitk_reduce, so both forms are bitwise identical.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double* flag = lds;   // the one LDS array (no second __shared__ object, see the guide's trap 4a)
    if (tid == 0) {
        const int t = __hip_atomic_fetch_add(&tickets[tslot], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = (t == int(gridDim.z) - 1);
        if (last) __hip_atomic_store(&tickets[tslot], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = last ? 1.0 : 0.0;
    }
    __syncthreads();
    if (flag[0] == 0.0 || kg != 0) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn + j * 16 + lc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm + i * 16 + lg + 4 * r;
                if (row < M && col < N && (!mirror || row >= col)) {
                    const size_t o = size_t(row) * N + col;
                    double sum = 0.0;
                    for (int z = 0; z < int(gridDim.z); ++z)
                        sum += (z == zb) ? acc[i][j][r]
                                                      : __hip_atomic_load(&slab[(size_t(bz) * gridDim.z + z) * MN + o], __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_AGENT);
                    C[o] = alpha * sum;
                    if (mirror) C[size_t(col) * N + row] = alpha * sum;
                }
            }
        }
}


template <int BM, int BN, int GBK, int WGM, int WGN, int WGK, int PD, bool TA, bool TB, class PTR>
__device__ __forceinline__ void gemm_body(const PTR& ptrs, size_t lda, size_t ldb, int M, int N, int K, int kps,
                                          double alpha, double* __restrict__ slab, int tiles_m, int xcd_group,
                                          int* __restrict__ tickets, int sym) {
    const int bz = blockIdx.y;   // batch entry
    const double* __restrict__ A = ptrs.a(bz);
    const double* __restrict__ B = ptrs.b(bz);
    constexpr int NT = WGM * WGN * WGK * 64;   // WGK wave groups split every K-step's MFMA k-substeps
    // LDS rows of BM / BN doubles, XOR-swizzled per k row: element (k, m) at k*SA + (m ^ swz(k)) with
    // swz(k) = 16*(k&1) | (k&15). ds_read_b64 banks over 32-lane groups, (a/4) mod 64: the fragment reads
    // (16 m x rows k, k+1) cover all 32 8-byte bank pairs; ds_write_b64 banks over 16-lane groups,
    // (a/4) mod 32: the transposed stores (16 consecutive k, one m) get 16 distinct low nibbles (the
    // former (k>>1) swizzle paired them: SQ_LDS_BANK_CONFLICT ~1 cycle per LDS instruction).
    constexpr int SA = BM;
    constexpr int SB = BN;
    static_assert(BM % 16 == 0 && BN % 16 == 0, "tile rows must be whole MFMA tiles");
    // 32-aligned rows take the 32-wide swizzle; 16-aligned ones (80-wide tiles) stay inside their 16-group
    constexpr bool WIDE_SWZ_A = BM % 32 == 0, WIDE_SWZ_B = BN % 32 == 0;
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int TM = WM / 16, TN = WN / 16;
    static_assert(TM >= 1 && TN >= 1, "wave tile smaller than one MFMA tile");
    // two accumulator sets (even / odd k-substeps) when the wave tile is small: independent MFMA chains
    constexpr int NACC = (TM * TN <= 2) ? 2 : 1;
    // per-thread staging counts (in doubles)
    constexpr int A_PER = (BM * GBK + NT - 1) / NT;
    constexpr int B_PER = (BN * GBK + NT - 1) / NT;

    __shared__ double As[2][GBK * SA];
    __shared__ double Bs[2][GBK * SB];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int kg = wave / (WGM * WGN);
    const int pos = wave % (WGM * WGN);
    const int wm = (pos / WGN) * WM;
    const int wn = (pos % WGN) * WN;
    static_assert(GBK % (4 * WGK) == 0, "K-step must split evenly over the wave groups");
    static_assert(WGK == 1 || (WGK - 1) * BM * BN <= 2 * GBK * (SA + SB), "LDS reduction buffer too small");

    // XCD-aware tile order: workgroups b, b+8, b+16, ... share an XCD (round-robin dispatch), so the
    // tiles that read the same panel of the LARGE operand are given ids congruent mod 8 and that panel
    // is fetched into one XCD's L2 once instead of once per XCD. xcd_group: 1 = tiles sharing a B column
    // panel (same tn) together, 2 = tiles sharing an A row panel (same tm), 0 = plain column-major order.
    int tm, tn;
    {
        const int b = blockIdx.x, tiles_n = gridDim.x / tiles_m;
        if (xcd_group == 1) {
            const int xcd = b & 7, slot = b >> 3;
            tn = (slot / tiles_m) * 8 + xcd;
            tm = slot % tiles_m;
        } else if (xcd_group == 2) {
            const int xcd = b & 7, slot = b >> 3;
            tm = (slot / tiles_n) * 8 + xcd;
            tn = slot % tiles_n;
        } else {
            tm = b % tiles_m;
            tn = b / tiles_m;
        }
    }
    // symmetric result (sym, square tiles, M == N): only tiles on or below the diagonal are computed;
    // each lower element is also written to its mirror position
    if (sym && tm < tn) return;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = blockIdx.z * kps;
    const int kend = min(K, kbeg + kps);

    d4 acc2[NACC][TM][TN];
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc2[a][i][j] = d4{0.0, 0.0, 0.0, 0.0};
    auto swza = [](int k) { return WIDE_SWZ_A ? (((k & 1) << 4) | (k & 15)) : (k & 15); };
    auto swzb = [](int k) { return WIDE_SWZ_B ? (((k & 1) << 4) | (k & 15)) : (k & 15); };

    // register ring: the global loads of K-step t+PD are issued while step t computes, so PD steps of
    // MFMA work cover the global-memory latency (one step is only ~4-8 MFMAs per wave)
    double ra[PD][A_PER], rb[PD][B_PER];

    // ---- global -> registers for the K-step starting at k0. Loads are unconditional (clamped addresses)
    // so that no branch separates them from their use and the waitcnt pass can count them; the
    // out-of-range elements are zeroed when the slot is written to LDS.
    auto a_coord = [&](int e, int& m, int& k) {
        const int idx = tid + e * NT;
        if (TA) { m = idx % BM; k = idx / BM; } else { k = idx % GBK; m = idx / GBK; }
    };
    auto b_coord = [&](int e, int& n, int& k) {
        const int idx = tid + e * NT;
        if (TB) { k = idx % GBK; n = idx / GBK; } else { n = idx % BN; k = idx / BN; }
    };
    auto load_tile = [&](int k0, auto slot_c) {
        constexpr int slot = decltype(slot_c)::value;
#pragma unroll
        for (int e = 0; e < A_PER; ++e) {
            int m, k;
            a_coord(e, m, k);
            const int gm = min(m0 + m, M - 1), gk = min(k0 + k, kend - 1);
            ra[slot][e] = TA ? A[size_t(gk) * lda + gm] : A[size_t(gm) * lda + gk];
        }
#pragma unroll
        for (int e = 0; e < B_PER; ++e) {
            int n, k;
            b_coord(e, n, k);
            const int gn = min(n0 + n, N - 1), gk = min(k0 + k, kend - 1);
            rb[slot][e] = TB ? B[size_t(gn) * ldb + gk] : B[size_t(gk) * ldb + gn];
        }
    };
    auto store_tile = [&](int buf, int k0, auto slot_c) {
        constexpr int slot = decltype(slot_c)::value;
#pragma unroll
        for (int e = 0; e < A_PER; ++e) {
            int m, k;
            a_coord(e, m, k);
            const bool ok = (m0 + m < M) && (k0 + k < kend);
            // (no guard when the tile divides evenly over the threads: a branch here makes the waitcnt
            // pass lose track of the ring's loads and drain vmcnt(0) at the loop head)
            if ((BM * GBK) % NT == 0 || tid + e * NT < BM * GBK) As[buf][k * SA + (m ^ swza(k))] = ok ? ra[slot][e] : 0.0;
        }
#pragma unroll
        for (int e = 0; e < B_PER; ++e) {
            int n, k;
            b_coord(e, n, k);
            const bool ok = (n0 + n < N) && (k0 + k < kend);
            if ((BN * GBK) % NT == 0 || tid + e * NT < BN * GBK) Bs[buf][k * SB + (n ^ swzb(k))] = ok ? rb[slot][e] : 0.0;
        }
    };
    const int lr = lane & 15, lk = lane >> 4;
    auto compute = [&](int buf) {
        const double* as = As[buf];
        const double* bs = Bs[buf];
#pragma unroll
        for (int q = 0; q < GBK / (4 * WGK); ++q) {
            const int kk = (q * WGK + kg) * 4;
            double af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = as[(kk + lk) * SA + ((wm + i * 16 + lr) ^ swza(kk + lk))];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = bs[(kk + lk) * SB + ((wn + j * 16 + lr) ^ swzb(kk + lk))];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc2[q % NACC][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc2[q % NACC][i][j], 0, 0, 0);
        }
    };

    const int nsteps = (kend > kbeg) ? (kend - kbeg + GBK - 1) / GBK : 0;
    if (nsteps > 0) {
        static_assert(PD % 2 == 0, "ring depth must be even (LDS double buffer parity)");
        // unconditional (clamped addresses; slots past the slice end are never stored): branch-free, so
        // the waitcnt pass can count the ring
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (load_tile(kbeg + U * GBK, std::integral_constant<int, U>{}), ...);
        }(std::make_integer_sequence<int, PD>{});
        store_tile(0, kbeg, std::integral_constant<int, 0>{});
        __syncthreads();
        int t0 = 0;
        // steady state: no guards, every iteration issues the loads of step t + PD
        for (; t0 + 2 * PD <= nsteps; t0 += PD) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (([&] {
                     const int t = t0 + U;
                     compute(U & 1);
                     store_tile((U + 1) & 1, kbeg + (t + 1) * GBK, std::integral_constant<int, (U + 1) % PD>{});
                     load_tile(kbeg + (t + PD) * GBK, std::integral_constant<int, U>{});
                     __syncthreads();
                 }()),
                 ...);
            }(std::make_integer_sequence<int, PD>{});
        }
        // tail
        for (; t0 < nsteps; t0 += PD) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (([&] {
                     const int t = t0 + U;
                     if (t < nsteps) {
                         compute(U & 1);
                         if (t + 1 < nsteps)
                             store_tile((U + 1) & 1, kbeg + (t + 1) * GBK, std::integral_constant<int, (U + 1) % PD>{});
                         if (t + PD < nsteps) load_tile(kbeg + (t + PD) * GBK, std::integral_constant<int, U>{});
                     }
                     __syncthreads();
                 }()),
                 ...);
            }(std::make_integer_sequence<int, PD>{});
        }
    }

    gemm_finish<TM, TN, WGM, WGN, WGK, NACC>(acc2, &As[0][0], ptrs, M, N, alpha, slab, tickets, sym, m0, n0, wm, wn, kg, pos,
                                             int(blockIdx.x), int(blockIdx.y), int(blockIdx.z));
}

// ---------------------------------------------------------------------------------------------------
// k_gemm_glds: the pipeline for whole tiles (M % BM == N % BN == 0, K-slices of whole 32-deep steps,
// 16-B aligned operands). Operands go global -> LDS by 16-B global_load_lds (LDS-DMA, no VGPR staging)
// into S = 3 LDS stages; one raw s_barrier per 32-deep K-step, preceded by a counted vmcnt that leaves the
// next stage's DMA in flight across it (cdna_hip_programming.md §5 "Pipelining across barriers"). The
// DMA destination is lane-linear, so the bank swizzle goes on the SOURCE address:
//   RK image (operand stored [r][k], k contiguous): row r = 32 doubles, 16-B chunk c at c ^ (r & 15)
//   KR image (operand stored [k][r], R doubles per k row): chunk c of row k at c ^ (8 (k & 1)) (R % 32 == 0)
// Fragment reads (16 rows x k, k+1 per 32-lane half) then hit 32 distinct 8-B bank pairs in both images.
constexpr int kGldsBK = 32;

template <int R, bool KMAJ, int BK = kGldsBK>
struct GldsImg {
    // k-major rows of R % 32 == 16 doubles alternate bank halves by themselves (640-B rows: k*160 words mod 64 =
    // 0, 32, ...); rows of whole 256-B bank rows take the XOR
    static_assert(!KMAJ || R % 16 == 0, "k-major image rows must be whole MFMA tiles");
    static constexpr int KSWZ = (R % 32 == 0) ? 8 : 0;
    static constexpr int DOUBLES = R * BK;
    static constexpr int INSTR = DOUBLES * 8 / 1024;   // 1-KB wave instructions per stage
    __device__ static int at(int r, int k) {   // LDS offset (doubles) of element (r, k)
        if constexpr (!KMAJ) return r * BK + ((((k >> 1) ^ (r & 15))) << 1) + (k & 1);
        else return k * R + ((((r >> 1) ^ ((k & 1) * KSWZ))) << 1) + (r & 1);
    }
    // Per-lane fragment offsets of the NF 16-row MFMA fragments at rows w0 + 16 i (w0 % 16 == 0) for
    // K-substep q of a wave group kg (of WGK, a power of 2): lane (lr = l & 15, lk = l >> 4) reads element
    // (w0 + 16 i + lr, kk = 4 (q WGK + kg) + lk). The q dependence reduces to a compile-time term (an
    // immediate ds_read offset for KR images; one XOR for RK images, whose 16-B chunk index 2 (q WGK + kg)
    // + (lk >> 1) equals (2 q WGK) ^ (2 kg) ^ (lk >> 1) because the bit ranges are disjoint).
    template <int NF, int WGK>
    struct Frag {
        static_assert((WGK & (WGK - 1)) == 0, "wave groups must be a power of 2");
        int base[KMAJ ? NF : 1];
        int z = 0;
        __device__ Frag(int w0, int kg, int lane) {
            const int lr = lane & 15, lk = lane >> 4;
            if constexpr (!KMAJ) {
                base[0] = (w0 + lr) * BK + (lk & 1);
                z = (2 * kg) ^ (lk >> 1) ^ lr;
            } else {
                const int swz = (lk & 1) * (KSWZ / 8);
#pragma unroll
                for (int i = 0; i < NF; ++i) base[i] = (4 * kg + lk) * R + 16 * ((w0 / 16 + i) ^ swz) + lr;
            }
        }
        __device__ int off(int q, int i) const {
            if constexpr (!KMAJ) return base[0] + i * 16 * BK + (((2 * q * WGK) ^ z) << 1);
            else return base[i] + 4 * q * WGK * R;
        }
    };
    __device__ static void src(int q, int& r, int& k) {   // element (r, k) that starts LDS chunk q
        if constexpr (!KMAJ) {
            constexpr int CPR = BK / 2;   // 16-B chunks per row
            r = q / CPR;
            k = ((q % CPR) ^ (r & 15)) << 1;
        } else {
            constexpr int CR = R / 2;
            k = q / CR;
            r = ((q % CR) ^ ((k & 1) * KSWZ)) << 1;
        }
    }
};

template <int BM, int BN, int WGM, int WGN, int WGK>
constexpr int glds_min_waves() { return (WGM * WGN * WGK * 64 >= 512) ? 2 : 1; }

// LDS of the glds pipeline: S stages of the A and B images -- 3 stages of 32-deep K-steps, or 2 stages
// of 64-deep steps (half the barriers per K; the DMA of step t+1 is issued at the start of step t, the
// same 64-deep lead as 3 x 32)
template <int BK, int ST = 0>
constexpr int glds_stages() { return ST > 0 ? ST : (BK == 64 ? 2 : 3); }
template <int BM, int BN, int BK = kGldsBK, int ST = 0>
constexpr int glds_lds_doubles() { return glds_stages<BK, ST>() * (BM + BN) * BK; }

// One output tile of the glds pipeline for entry blockIdx.y of `ptrs` (tile blockIdx.x, K-slice
// blockIdx.z); `lds` holds glds_lds_doubles<BM, BN>() doubles (k_gemm_glds).
template <int BM, int BN, int WGM, int WGN, int WGK, bool TA, bool TB, class PTR, int BK = kGldsBK, int ST = 0>
__device__ __forceinline__ void glds_body(double* __restrict__ lds, const PTR& ptrs, size_t lda, size_t ldb, int M, int N,
                                          int K, int kps, double alpha, double* __restrict__ slab, int tiles_m,
                                          int xcd_group, int* __restrict__ tickets, int sym, int tri) {
#ifdef XRS_GEMM_TRACE
    const unsigned long long xrs_c0 = __builtin_amdgcn_s_memtime();
#endif
    constexpr int S = glds_stages<BK, ST>();
    constexpr int NW = WGM * WGN * WGK;
    using IA = GldsImg<BM, TA, BK>;   // A stored [m][k] (RK) or, transposed, [k][m] (KR)
    using IB = GldsImg<BN, !TB, BK>;  // B stored [k][n] (KR) or, transposed, [n][k] (RK)
    constexpr int STAGE = IA::DOUBLES + IB::DOUBLES;
    static_assert(S * STAGE == glds_lds_doubles<BM, BN, BK, ST>(), "LDS layout");
    constexpr int INSTR = IA::INSTR + IB::INSTR;
    // wave w issues DMA instructions j = w, w + NW, ...: PER_WAVE of them, or one fewer for w >= INSTR % NW
    constexpr int PER_WAVE = (INSTR + NW - 1) / NW;
    static_assert(PER_WAVE * (S - 2) <= 63, "vmcnt range");
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int TM = WM / 16, TN = WN / 16;
    static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole MFMA tiles");
    static_assert(BK % (4 * WGK) == 0, "K-step must split evenly over the wave groups");
    constexpr int NACC = (TM * TN <= 2) ? 2 : 1;
    static_assert(WGK == 1 || (WGK - 1) * WGM * WGN * TM * TN * 256 <= S * STAGE, "LDS reduction buffer too small");

    // tile index xb, batch entry bz and split-K slice zb. xcd_group 3 (split-K grids whose entry x slice
    // count is a multiple of 8): workgroups are dealt to the 8 XCDs round-robin by dispatch order, so the
    // linear id's residue picks the XCD and every XCD takes whole (entry, slice) pairs -- all tiles of one
    // pair on one XCD: a slice's operand panels are fetched into ONE XCD's L2 instead of all eight (the
    // step's Grams: 56 -> 41 MB of HBM reads per launch, profiles/r05/xcd_split_ab_r05ai.txt)
    int xb = int(blockIdx.x), bz = int(blockIdx.y), zb = int(blockIdx.z);
    if (xcd_group == 3) {
        const int X = int(gridDim.x), Y = int(gridDim.y);
        const int L = xb + X * (bz + Y * zb), c = L & 7, q = L >> 3;
        const int u = c + 8 * (q / X);   // (entry, slice) pair
        xb = q % X;
        bz = u % Y;
        zb = u / Y;
    }
    const double* __restrict__ A = ptrs.a(bz);
    const double* __restrict__ B = ptrs.b(bz);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kg = wave / (WGM * WGN), pos = wave % (WGM * WGN);
    const int wm = (pos / WGN) * WM, wn = (pos % WGN) * WN;
    int tm, tn;
    if (sym) {   // the grid holds the lower tiles only: x -> (tm, tn), tm >= tn, row by row
        const int x = xb;
        tm = int((__builtin_sqrtf(8.0f * float(x) + 1.0f) - 1.0f) * 0.5f);
        while ((tm + 1) * (tm + 2) / 2 <= x) ++tm;
        while (tm * (tm + 1) / 2 > x) --tm;
        tn = x - tm * (tm + 1) / 2;
    } else {
        const int b = xb, tiles_n = gridDim.x / tiles_m;
        if (xcd_group == 1) {
            const int xcd = b & 7, slot = b >> 3;
            tn = (slot / tiles_m) * 8 + xcd;
            tm = slot % tiles_m;
        } else if (xcd_group == 2) {
            const int xcd = b & 7, slot = b >> 3;
            tm = (slot / tiles_n) * 8 + xcd;
            tn = slot % tiles_n;
        } else {
            tm = b % tiles_m;
            tn = b / tiles_m;
        }
    }
    const int m0 = tm * BM, n0 = tn * BN;
    // triangular operands (exact zeros outside the triangle): op(A) lower (bit 0) needs k < m0 + BM only,
    // op(B) lower (bit 1) k >= n0 only -- whole K-steps of the slice's range
    const int klo = (tri & 2) ? (n0 / BK) * BK : 0;
    const int khi = (tri & 1) ? min(K, (m0 + BM + BK - 1) / BK * BK) : K;
    const int kbeg = max(zb * kps, klo);
    const int nsteps = max(0, min(khi, zb * kps + kps) - kbeg) / BK;   // (the host guarantees whole steps)
    const bool full = wave < INSTR % NW || INSTR % NW == 0;     // issues PER_WAVE DMAs per stage (else one fewer)

    // this wave's DMA instructions: j = wave + NW u; j < IA::INSTR -> A image, else B image
    const double* gsrc[PER_WAVE];
    size_t gstep[PER_WAVE];   // source advance per K-step (doubles)
    int ldsoff[PER_WAVE];     // LDS destination (doubles) of the instruction within a stage
#pragma unroll
    for (int u = 0; u < PER_WAVE; ++u) {
        const int j = min(wave + NW * u, INSTR - 1);   // (a wave with one fewer never issues its last slot)
        int r, k;
        if (j < IA::INSTR) {
            IA::src((j * 64) + lane, r, k);
            gsrc[u] = TA ? A + size_t(kbeg + k) * lda + (m0 + r) : A + size_t(m0 + r) * lda + (kbeg + k);
            gstep[u] = TA ? size_t(BK) * lda : size_t(BK);
            ldsoff[u] = j * 128;
        } else {
            IB::src(((j - IA::INSTR) * 64) + lane, r, k);
            gsrc[u] = TB ? B + size_t(n0 + r) * ldb + (kbeg + k) : B + size_t(kbeg + k) * ldb + (n0 + r);
            gstep[u] = TB ? size_t(BK) : size_t(BK) * ldb;
            ldsoff[u] = IA::DOUBLES + (j - IA::INSTR) * 128;
        }
    }
    auto issue = [&](int t) {   // DMA of K-step t into stage t % S
        double* st = lds + (t % S) * STAGE;
#pragma unroll
        for (int u = 0; u < PER_WAVE; ++u)
            if (u < PER_WAVE - 1 || full)
            __builtin_amdgcn_global_load_lds(static_cast<const void*>(gsrc[u] + size_t(t) * gstep[u]),
                                             (__attribute__((address_space(3))) void*)(st + ldsoff[u]),
                                             16, 0, 0);
    };

    d4 acc2[NACC][TM][TN];
#pragma unroll
    for (int a = 0; a < NACC; ++a)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc2[a][i][j] = d4{0.0, 0.0, 0.0, 0.0};
    const typename IA::template Frag<TM, WGK> fa(wm, kg, lane);
    const typename IB::template Frag<TN, WGK> fb(wn, kg, lane);

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nsteps) issue(s);
    for (int t = 0; t < nsteps; ++t) {
        // retire stage t (this wave's DMAs); the stages issued after it (up to S - 2 of them, fewer at the
        // end of the slice) stay in flight across the barrier
        const int ahead = min(S - 2, nsteps - 1 - t);
        if (ahead <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (ahead == 1) {
            if (full) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE - 1) : "memory");
        } else {
            if (full) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE * (S - 2)) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PER_WAVE - 1) * (S - 2)) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of stage t-1 are done
        __builtin_amdgcn_s_barrier();
        XRS_TRACE_STEP(t)
        const double* as = lds + (t % S) * STAGE;
        const double* bs = as + IA::DOUBLES;
        // fragments double-buffered in registers: the reads of substep q+1 are issued ahead of the MFMAs of
        // substep q, so the LDS latency hides behind the MFMA pipe instead of draining it every substep
        constexpr int NQ = BK / (4 * WGK);
        double af[2][TM], bf[2][TN];
        auto frag = [&](int q, double(&a)[TM], double(&b)[TN]) {
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = as[fa.off(q, i)];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = bs[fb.off(q, j)];
        };
        frag(0, af[0], bf[0]);
#ifndef XRS_GLDS_NOLOAD   // (diagnostic builds: compute-only timing, results meaningless)
        if (t + S - 1 < nsteps) issue(t + S - 1);              // overwrites stage t-1 (all waves are past it)
#endif
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) frag(q + 1, af[(q + 1) & 1], bf[(q + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);   // keep those reads ahead of this substep's MFMAs
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc2[q % NACC][i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[q & 1][i], bf[q & 1][j], acc2[q % NACC][i][j], 0, 0, 0);
        }
    }
    __syncthreads();   // every wave is done with the stages before the epilogue reuses the LDS
    gemm_finish<TM, TN, WGM, WGN, WGK, NACC>(acc2, lds, ptrs, M, N, alpha, slab, tickets, sym, m0, n0, wm, wn, kg, pos, xb, bz, zb);
}

template <int BM, int BN, int WGM, int WGN, int WGK, bool TA, bool TB, class PTR, int BK = kGldsBK, int ST = 0>
__global__ void __launch_bounds__(WGM * WGN * WGK * 64, (glds_min_waves<BM, BN, WGM, WGN, WGK>()))
k_gemm_glds(const PTR ptrs, size_t lda, size_t ldb, int M, int N, int K, int kps, double alpha,
            double* __restrict__ slab, int tiles_m, int xcd_group, int* __restrict__ tickets, int sym, int tri) {
    XRS_TRACE_BEGIN
    __shared__ double lds[glds_lds_doubles<BM, BN, BK, ST>()];   // the one LDS array (trap 4a: no second __shared__ object)
    glds_body<BM, BN, WGM, WGN, WGK, TA, TB, PTR, BK, ST>(lds, ptrs, lda, ldb, M, N, K, kps, alpha, slab, tiles_m, xcd_group,
                                                      tickets, sym, tri);
    XRS_TRACE_END
}

#ifndef XRS_REDUCE_CHUNK
#define XRS_REDUCE_CHUNK 16
#endif
constexpr int kReduceChunk = XRS_REDUCE_CHUNK;

// sum over the split-K slabs of element i, in slice order 0..splits-1 (bitwise identical to the in-launch
// combine); the loads of kReduceChunk slices are issued together ahead of their dependent adds. Chunk
// 16 / 20 / 24 / 32 / 48 over the bench step's reduces (40-slice Grams, 16-slice 256^2 products; rocprof
// averages under the step's concurrency): 6.0-6.2 / 6.2-6.3 / 6.0-6.8 / 6.9-7.1 / 8.1 us
// (profiles/r05/reduce_chunk_ab_r05.txt)
__device__ __forceinline__ double slice_sum(const double* __restrict__ slab, size_t MN, int splits, size_t i) {
    double s = 0.0;
    for (int z0 = 0; z0 < splits; z0 += kReduceChunk) {
        double v[kReduceChunk];
#pragma unroll
        for (int u = 0; u < kReduceChunk; ++u)
            v[u] = (z0 + u < splits) ? __builtin_nontemporal_load(&slab[size_t(z0 + u) * MN + i]) : 0.0;
#pragma unroll
        for (int u = 0; u < kReduceChunk; ++u)
            if (z0 + u < splits) s += v[u];
    }
    return s;
}

template <class PTR>
__global__ void __launch_bounds__(256) k_splitk_reduce(const PTR ptrs, const double* __restrict__ slab, size_t MN,
                                                       int splits, double alpha, int symN) {
    double* __restrict__ C = ptrs.c(blockIdx.y);
    slab += size_t(blockIdx.y) * splits * MN;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < MN; i += stride) {
        size_t row = 0, col = 0;
        if (symN) {   // symmetric result: lower elements only (the upper slabs were never written)
            row = i / size_t(symN);
            col = i - row * size_t(symN);
            if (col > row) continue;
        }
        const double s = alpha * slice_sum(slab, MN, splits, i);
        C[i] = s;
        if (symN) C[col * size_t(symN) + row] = s;
    }
}

// Symmetric results by 16 x 16 tiles of the lower triangle (blockIdx.x = ti (ti + 1) / 2 + tj, tj <= ti): every
// thread sums one element, and the tile's mirror goes out through LDS as whole 128-B row segments (the
// elementwise form above writes the mirror one column at a time: a line per lane). Same per-element sums.
constexpr int kSymTile = 16;
template <class PTR>
__global__ void __launch_bounds__(256) k_splitk_reduce_sym(const PTR ptrs, const double* __restrict__ slab, int N,
                                                           int splits, double alpha) {
    __shared__ double t[kSymTile][kSymTile + 1];
    double* __restrict__ C = ptrs.c(blockIdx.y);
    const size_t MN = size_t(N) * N;
    slab += size_t(blockIdx.y) * splits * MN;
    int ti = int((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
    while ((ti + 1) * (ti + 2) / 2 <= int(blockIdx.x)) ++ti;
    while (ti * (ti + 1) / 2 > int(blockIdx.x)) --ti;
    const int tj = int(blockIdx.x) - ti * (ti + 1) / 2;
    const int r = int(threadIdx.x) / kSymTile, c = int(threadIdx.x) % kSymTile;
    const size_t row = size_t(ti) * kSymTile + r, col = size_t(tj) * kSymTile + c;
    const bool diag = ti == tj;
    // (a diagonal tile's upper elements take their mirror's value: the result is exactly symmetric)
    const double s = (!diag || c <= r) ? alpha * slice_sum(slab, MN, splits, row * N + col) : 0.0;
    t[c][r] = s;
    __syncthreads();
    C[row * N + col] = (diag && c > r) ? t[r][c] : s;
    if (!diag) C[(size_t(tj) * kSymTile + r) * N + size_t(ti) * kSymTile + c] = t[r][c];
}

// the split-K slabs -> C (alpha applied). XRS_REDUCE_SYM=0: symmetric results through the elementwise kernel
// (A/B of the tiled form).
template <class PTR>
static void splitk_reduce(xrs_handle_t h, const PTR& P, int count, const double* slab, int M, int N, int splits,
                          double alpha, bool sym) {
    static const bool sym_tiled = [] {
        const char* e = std::getenv("XRS_REDUCE_SYM");
        return !(e && e[0] == '0');
    }();
    const size_t MN = size_t(M) * N;
    // (its own family: the bench reports the GEMM family's fraction with and without these launches; dispatch
    // timestamps like the GEMMs')
    KernelTimer timer(h, XRS_KFAM_SPLITK, count * double(MN) * splits, count * 8.0 * double(MN) * (splits + 1), true);
    if (sym && sym_tiled && N % kSymTile == 0) {
        const unsigned T = unsigned(N / kSymTile);
        hipExtLaunchKernelGGL(k_splitk_reduce_sym<PTR>, dim3(T * (T + 1) / 2, unsigned(count)), dim3(256), 0, h->stream,
                              timer.start(), timer.stop(), 0, P, slab, N, splits, alpha);
        check_launch("k_splitk_reduce_sym");
        return;
    }
    const unsigned blocks = unsigned(std::min<size_t>((MN + 255) / 256, 4096));
    hipExtLaunchKernelGGL(k_splitk_reduce<PTR>, dim3(blocks, unsigned(count)), dim3(256), 0, h->stream, timer.start(),
                          timer.stop(), 0, P, slab, MN, splits, alpha, sym ? N : 0);
    check_launch("k_splitk_reduce");
}

template <int BM, int BN, int GBK, int WGM, int WGN, int WGK, int PD, class PTR>
static void launch_tiles(xrs_handle_t h, const PTR& P, int count, size_t lda, bool ta, size_t ldb, bool tb,
                         int M, int N, int K, int splits, int kps, double alpha, double* slab, int* tickets, int sym) {
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    dim3 grid(unsigned(tiles_m * tiles_n), unsigned(count), unsigned(splits));
    // group by the larger operand's panels (B: K x N, A: M x K) when the tile grid allows a bijection
    int xg = 0;
    if (double(N) >= double(M)) xg = (tiles_n % 8 == 0) ? 1 : 0;
    else xg = (tiles_m % 8 == 0) ? 2 : 0;
    KernelTimer timer(h, XRS_KFAM_GEMM, count * 2.0 * double(M) * double(N) * double(K),
                      count * 8.0 * (double(M) * K + double(K) * N + double(M) * N * splits), true);
#define XRS_GEMM_LAUNCH(TA_, TB_)                                                                             \
    hipExtLaunchKernelGGL((k_gemm_f64<BM, BN, GBK, WGM, WGN, WGK, PD, TA_, TB_, PTR>), grid, dim3(WGM * WGN * WGK * 64), 0, \
                          h->stream, timer.start(), timer.stop(), 0, P, lda, ldb, M, N, K, kps, alpha, slab, tiles_m, xg, tickets, sym)
    if (!ta && !tb) XRS_GEMM_LAUNCH(false, false);
    else if (!ta && tb) XRS_GEMM_LAUNCH(false, true);
    else if (ta && !tb) XRS_GEMM_LAUNCH(true, false);
    else XRS_GEMM_LAUNCH(true, true);
#undef XRS_GEMM_LAUNCH
    check_launch("k_gemm_f64");
}

template <int BM, int BN, int WGM, int WGN, int WGK, int BK = kGldsBK, int ST = 0, class PTR>
static void launch_glds(xrs_handle_t h, const PTR& P, int count, size_t lda, bool ta, size_t ldb, bool tb, int M, int N,
                        int K, int splits, int kps, double alpha, double* slab, int* tickets, int sym, int tri) {
    const int tiles_m = M / BM, tiles_n = N / BN;
    // symmetric: only the lower tiles are launched (the kernel maps x to (tm >= tn)), so the workgroups of
    // every split spread evenly over the XCDs
    dim3 grid(unsigned(sym ? tiles_m * (tiles_m + 1) / 2 : tiles_m * tiles_n), unsigned(count), unsigned(splits));
    int xg = 0;
    if (double(N) >= double(M)) xg = (tiles_n % 8 == 0) ? 1 : 0;
    else xg = (tiles_m % 8 == 0) ? 2 : 0;
    // whole (entry, slice) pairs per XCD: the step's GEMMs read 27.4 -> 20.3 MB of HBM per launch (the Grams
    // 56 -> 41 MB, the batched orthogonality Grams 252 -> 63 MB) at an unchanged step time
    // (profiles/r05/xcd_split_ab_r05aj.txt). XRS_GLDS_XCD_SPLIT=0: the plain order (A/B). (Its first
    // version summed the in-launch combine with the hardware slice index instead of the remapped one; the
    // world-2 cfg5 truncation test caught it, profiles/r05/cfg5_sharded_xcd_split_fail_r05.log.)
    static const bool xcd_split = [] {
        const char* e = std::getenv("XRS_GLDS_XCD_SPLIT");
        return !(e && e[0] == '0');
    }();
    if (xcd_split && splits >= 2 && (count * splits) % 8 == 0) xg = 3;   // whole (entry, split-K slice) pairs per XCD
    // executed K-depth summed over the tile rows / columns (triangular operands skip their zero blocks)
    double kdepth = double(K);
    if (tri & 1) {
        double s = 0;
        for (int m0 = 0; m0 < M; m0 += BM) s += std::min(K, (m0 + BM + BK - 1) / BK * BK);
        kdepth = s / tiles_m;
    } else if (tri & 2) {
        double s = 0;
        for (int n0 = 0; n0 < N; n0 += BN) s += K - (n0 / BK) * BK;
        kdepth = s / tiles_n;
    }
    KernelTimer timer(h, XRS_KFAM_GEMM, count * 2.0 * double(M) * double(N) * kdepth,
                      count * 8.0 * (double(M) * K + double(K) * N + double(M) * N * splits), true);
#define XRS_GLDS_LAUNCH(TA_, TB_)                                                                              \
    hipExtLaunchKernelGGL((k_gemm_glds<BM, BN, WGM, WGN, WGK, TA_, TB_, PTR, BK, ST>), grid, dim3(WGM * WGN * WGK * 64), 0, \
                          h->stream, timer.start(), timer.stop(), 0, P, lda, ldb, M, N, K, kps, alpha, slab, tiles_m, xg, tickets, sym, tri)
    if (!ta && !tb) XRS_GLDS_LAUNCH(false, false);
    else if (!ta && tb) XRS_GLDS_LAUNCH(false, true);
    else if (ta && !tb) XRS_GLDS_LAUNCH(true, false);
    else XRS_GLDS_LAUNCH(true, true);
#undef XRS_GLDS_LAUNCH
    check_launch("k_gemm_glds");
}

// The LDS-DMA pipeline (k_gemm_glds) for whole-tile shapes with 16-B aligned operands; false = not taken
// (the caller runs the general kernel). Tiles: g1 64x80 (4 waves, 16x80 each), g2 80x64 (4 waves, 80x16 each), g3 64x64
// (4 waves, 32x32), g4 64x64 (8 waves, K-substeps split over 2 wave groups), g5 32x32 (4 waves), g6 / g7 the
// 64x80 / 80x64 tiles with 8 waves (K-substeps split over 2 wave groups); g8 / g9 the same tiles with 4
// waves of 32x80 / 80x32 (2 wave groups); g10 64x64 with 4 waves of 64x64 (4 wave groups); g11 64x64 with 4
// waves of 32x64 (2 wave groups).
// XRS_GEMM_GLDS="v,target": v = 0 off, 1-5 forced variant, -1 automatic; target = workgroups aimed at
// by the split-K choice.
template <class PTR>
static bool gemm_glds(xrs_handle_t h, const PTR& P, int count, int M, int N, int K, double alpha, size_t lda, bool ta,
                      size_t ldb, bool tb, bool sym, int tri) {
    // (function-local static initialised once, thread-safe: the DotWorker thread runs GEMMs concurrently)
    static const std::pair<int, int> g_env = [] {
        int v = -1, t = 256;
        if (const char* e = std::getenv("XRS_GEMM_GLDS")) std::sscanf(e, "%d,%d", &v, &t);
        return std::make_pair(v, t);
    }();
    const int g_var = g_env.first, g_target = g_env.second;
    // The 8-wave tiles run with 2 LDS stages of 32-deep K-steps (64-74 KB: two workgroups per CU) instead of
    // 3 (96-110 KB: one), while the split-K choice still counts one workgroup per CU: the concurrent lanes of
    // a round (both Gram chains, <x,y> beside the round) then share every CU, one workgroup's barrier /
    // fragment-read bubbles filled by the other's MFMAs (bench step 1.10 -> 1.00 ms, r05y; alone the TT-shape
    // GEMMs are unchanged within 3 %). XRS_GLDS_ST2=mask (A/B): bit 0 the products (g6 / g7), bit 1 the Grams
    // (g4), bit 2 the one-workgroup split-K rule; default 7, 0 = the 3-stage tiles.
    static const int g_st2 = [] {
        const char* e = std::getenv("XRS_GLDS_ST2");
        return e ? std::atoi(e) : 7;
    }();
    if (g_var == 0) return false;
    if (K % kGldsBK != 0 || (lda & 1) || (ldb & 1)) return false;
    for (int i = 0; i < count; ++i)
        if ((reinterpret_cast<uintptr_t>(P.a(i)) & 15) || (reinterpret_cast<uintptr_t>(P.b(i)) & 15)) return false;
    const int bms[12] = {0, 64, 80, 64, 64, 32, 64, 80, 64, 80, 64, 64},
              bns[12] = {0, 80, 64, 64, 64, 32, 80, 64, 80, 64, 64, 64};
    auto fits = [&](int v) { return M % bms[v] == 0 && N % bns[v] == 0 && (!sym || bms[v] == bns[v]); };
    auto ntiles = [&](int v) {
        const long tm = M / bms[v], tn = N / bns[v];
        return sym ? long(count) * tm * (tm + 1) / 2 : long(count) * tm * tn;
    };
    int var = g_var;
    if (var < 0) {
        // measured on the TT shapes (tools/gemm_tt_bench.py, back-to-back wall per call): 256x5120x256 NN/TN
        // g6 18.7-20.2 us, g1 19.6-19.9, g8 20.0-20.3 (old kernel 24.5-25.1); 5120x256x256 g7 19.0-19.2, g2
        // 19.4; Grams 256^2 x 5120 g4 22.3-23.7, g3 23.4-25.2, g11 24.3-24.6 (old 25.5-28.0); 512x10240x512
        // and 512^2 x 10240: g4 117.8-125 (old 126-128)
        var = 0;
        if (sym) {
            if (fits(4)) var = 4;
            else if (fits(5)) var = 5;
        } else if (fits(6) && ntiles(6) >= 192) var = 6;
        else if (fits(7) && ntiles(7) >= 192) var = 7;
        else if (fits(4)) var = 4;
        else if (fits(5)) var = 5;
        if (var == 0) return false;
    }
    if (var < 1 || var > 11 || !fits(var)) return false;
    // (64-deep K-steps in 2 stages measured no faster: 18.5 vs 18.7 us on 256 x 5120 x 256)
    const int bk = kGldsBK;
    // split-K: whole K-steps per slice, aiming at `target` workgroups
    const long tiles = ntiles(var);
    const int ksteps = K / bk;
    int splits = 1;
    if (tiles < g_target) {
        // Whole waves of workgroups: the launch takes rounds(s) x ceil(ksteps / s) K-steps per CU, where
        // rounds(s) = ceil(tiles s / resident) and resident = target x the workgroups one CU holds (LDS
        // stages of 96-128 KB: one; the 32x32 tile: three). Picking s by the target alone overshoots into a
        // second, mostly idle round (the 6 orthogonality Grams of the bench round: 60 tiles x 5 slices =
        // 300 workgroups on 256 CUs, 64 K-steps per CU, against 40 at 4 slices).
        const int nwaves = (var == 4 || var == 6 || var == 7) ? 8 : 4;
        const bool st2 = (var == 4 && (g_st2 & 2)) || ((var == 6 || var == 7) && (g_st2 & 1));
        const int nst = (bk == 64 || (st2 && !(g_st2 & 4))) ? 2 : 3;
        const int lds_kb = nst * (bms[var] + bns[var]) * bk * 8 / 1024;
        const long resident = long(g_target) * std::max(1, std::min(160 / lds_kb, 16 / nwaves));
        const int smax = std::max(1, ksteps * bk / 128);
        long best = -1;
        for (int s = 1; s <= smax; ++s) {
            const int steps = (ksteps + s - 1) / s, seff = (ksteps + steps - 1) / steps;
            const long cost = (tiles * seff + resident - 1) / resident * steps;
            if (best < 0 || cost < best) best = cost, splits = seff;
        }
    }
    int kps = (ksteps + splits - 1) / splits * bk;
    splits = (K + kps - 1) / kps;
    DevBuf slab;
    if (splits > 1) slab = DevBuf(h, size_t(count) * splits * M * N * sizeof(double));
    const bool small_slab = size_t(splits) * bms[var] * bns[var] * sizeof(double) <= 65536 && bms[var] * bns[var] <= 4096;
    const long grid_tiles = long(count) * (M / bms[var]) * (N / bns[var]);
    int* tickets = (splits > 1 && small_slab && grid_tiles <= xrs_handle_s::kTicketCap) ? h->tickets : nullptr;
#define XRS_GLDS(...) launch_glds<__VA_ARGS__>(h, P, count, lda, ta, ldb, tb, M, N, K, splits, kps, alpha, slab.d(), tickets, sym ? 1 : 0, tri)
    switch (var) {
        case 1: XRS_GLDS(64, 80, 4, 1, 1); break;
        case 2: XRS_GLDS(80, 64, 1, 4, 1); break;
        case 3: XRS_GLDS(64, 64, 2, 2, 1); break;
        case 4: if (g_st2 & 2) XRS_GLDS(64, 64, 2, 2, 2, kGldsBK, 2); else XRS_GLDS(64, 64, 2, 2, 2); break;
        case 6: if (g_st2 & 1) XRS_GLDS(64, 80, 4, 1, 2, kGldsBK, 2); else XRS_GLDS(64, 80, 4, 1, 2); break;
        case 7: if (g_st2 & 1) XRS_GLDS(80, 64, 1, 4, 2, kGldsBK, 2); else XRS_GLDS(80, 64, 1, 4, 2); break;
        case 8: XRS_GLDS(64, 80, 2, 1, 2); break;
        case 9: XRS_GLDS(80, 64, 1, 2, 2); break;
        case 10: XRS_GLDS(64, 64, 1, 1, 4); break;
        case 11: XRS_GLDS(64, 64, 2, 1, 2); break;
        default: XRS_GLDS(32, 32, 2, 2, 1); break;
    }
#undef XRS_GLDS
    if (splits > 1 && tickets == nullptr) splitk_reduce(h, P, count, slab.d(), M, N, splits, alpha, sym);
    return true;
}

template <class PTR>
static void gemm_impl(xrs_handle_t h, const PTR& P, int count, size_t Ms, size_t Ns, double alpha, size_t lda, bool ta,
                      size_t Ks, size_t ldb, bool tb, bool sym = false, int tri = 0) {
    const int M = int(Ms), N = int(Ns), K = int(Ks);
    if (gemm_glds(h, P, count, M, N, K, alpha, lda, ta, ldb, tb, sym, tri)) return;   // (the general kernel ignores tri)
    // Tile choice (XRS_GEMM_CFG="variant,kmin,target" overrides for tuning experiments):
    //   v1 128x128 (8 waves 2x4)              large problems
    //   v2  64x64  (8 waves 2x4)              mid-size
    //   v3  64x32  (8 waves 2x2, K split 2)   split-K Gram shapes (r x r, K = n r)
    //   v4  32x32  (8 waves 2x2, K split 2)   TT "wide"/"tall" shapes (M or N = r, other = n r)
    //   v8/v9: v3/v4 with a 4-deep ring; v10-v13: K-step 32 / 4-wave / 16-wave variants (tuning only)
    // split-K brings the grid to ~target workgroups while every split keeps >= kmin of K.
    struct Cfg { int var = 0, kmin = 256, target = 512; };
    static const Cfg g_cfg = [] {   // thread-safe one-time initialisation (concurrent DotWorker GEMMs)
        Cfg c;
        if (const char* e = std::getenv("XRS_GEMM_CFG")) std::sscanf(e, "%d,%d,%d", &c.var, &c.kmin, &c.target);
        return c;
    }();
    const int cfg_var = g_cfg.var, cfg_kmin = g_cfg.kmin, cfg_target = g_cfg.target;
    // (batched: the tile counts are over the whole batch)
    auto ntiles = [&](int bm, int bn) { return long(count) * ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
    //   v14 64x80 / v15 80x64 (8 waves, K split 2, K-step 32): 256 x 5120 and 5120 x 256 TT shapes in
    //   exactly 256 tiles (one per CU)
    const int bms[16] = {0, 128, 64, 64, 32, 64, 64, 64, 64, 32, 32, 32, 32, 64, 64, 80},
              bns[16] = {0, 128, 64, 32, 32, 32, 64, 64, 32, 32, 32, 32, 32, 32, 80, 64};
    int var = cfg_var;
    long cfg_target_eff = cfg_target;
    // symmetric results aim at 160 workgroups (measured: 160 -> 1.367 ms/step, 384 -> 1.390, 512 -> 1.398,
    // 256 -> 1.481)
    if (sym) cfg_target_eff = 160;
    if (sym) {
        // symmetric result: square tiles only (32, 64, 128), counted over the lower triangle
        auto lower = [&](int b) { const long T = (M + b - 1) / b; return long(count) * T * (T + 1) / 2; };
        auto ntl = [&](int v) { return lower(bms[v]); };
        var = 4;
        if (lower(128) >= 1000) var = 1;
        else if (lower(64) >= 512) var = 2;   // (13 Grams of 512^2: 32x32 unsplit 943 us < 64x64 1165 us)
        else if (lower(32) < 512)
            for (int v : {1, 2, 4}) {
                const long t = ntl(v);
                const long sp = std::min<long>((cfg_target_eff + t - 1) / t, std::max<long>(1, K / cfg_kmin));
                if (t * sp >= cfg_target_eff) { var = v; break; }
            }
    } else if (var == 0) {
        // measured on the TT shapes (tools/gemm_tt_bench.py, profiles/r01/gemm_tt_sweep*.txt; the 32x32
        // and 64x32 tiles use a 2-deep ring since the waitcnt fix: 24.6 vs 27.2 us on 256x5120x256):
        //   256 x 5120 x 256 wide/tall: 32x32 24.8 us < 64x32 26.8 < 64x64 28.6 < 128x128 44.5 (alone;
        //                               with 3 concurrent streams 64x32 wins, see below)
        //   512 x 10240 x 512:          64x64 131 us < 64x32 148 < 128x128 154
        //   Gram 256^2, K 5120:         64x32 x16 splits 29-31 us < 32x32 x8 34;
        //   Gram 512^2, K 10240:        128x128 x32 splits 130 us < 32x32 x2 167
        // so: no split while the grid has >= 512 tiles of some size (the largest such tile wins up to
        // 64x64; 128x128 only from ~1000 tiles), else the largest tile whose split-K grid reaches
        // `target` workgroups (fewer, larger tiles re-read less of the long-K operands).
        if (ntiles(128, 128) >= 1000) var = 1;
        else if (ntiles(64, 64) >= 512) var = 2;
        else if (ntiles(32, 32) >= 1024) var = 4;
        else if (ntiles(64, 32) >= 256) var = 3;
        else if (ntiles(32, 32) >= 512) var = 4;
        else {
            var = 4;
            for (int v : {1, 2, 3}) {
                const long t = ntiles(bms[v], bns[v]);
                const long sp = std::min<long>((cfg_target_eff + t - 1) / t, std::max<long>(1, K / cfg_kmin));
                if (t * sp >= cfg_target_eff) { var = v; break; }
            }
        }
    }
    const long tiles = sym ? long(count) * ((M + bms[var] - 1) / bms[var]) * ((M + bms[var] - 1) / bms[var] + 1) / 2
                           : ntiles(bms[var], bns[var]);
    int splits = 1;
    if (tiles < cfg_target_eff) {
        const long want = (cfg_target_eff + tiles - 1) / tiles;
        const long maxs = std::max<long>(1, K / cfg_kmin);
        splits = int(std::max<long>(1, std::min(want, maxs)));
    }
    const int bk = ((var >= 5 && var <= 7) || var == 10 || var == 12 || var == 13 || var == 14 || var == 15) ? 32 : 16;
    int kps = (K + splits - 1) / splits;
    kps = (kps + bk - 1) / bk * bk;
    splits = (K + kps - 1) / kps;
    if (std::is_same<PTR, GemmMany>::value && var >= 5 && var <= 13) var = (var == 5 || var == 8 || var == 13) ? 3 : ((var == 9 || var >= 10) ? 4 : 2);   // tuning-only tiles: single GEMMs
    DevBuf slab;
    if (splits > 1) slab = DevBuf(h, size_t(count) * splits * M * N * sizeof(double));
    // one-launch split-K when the tile grid fits the stream's ticket array. The last arriver reads splits x
    // BM x BN doubles serially: worth it for small tiles only (the guide's "a few tens of KB" per tile;
    // 128x128 tiles at 2 splits measured 70 us slower than the reduce kernel, larger slab caps 0.3 ms/step)
    const bool small_slab = size_t(splits) * bms[var] * bns[var] * sizeof(double) <= 65536 && bms[var] * bns[var] <= 4096;
    int* tickets = (splits > 1 && small_slab && ntiles(bms[var], bns[var]) <= xrs_handle_s::kTicketCap)
                       ? h->tickets : nullptr;
#define XRS_TILES(...) launch_tiles<__VA_ARGS__>(h, P, count, lda, ta, ldb, tb, M, N, K, splits, kps, alpha, slab.d(), tickets, sym ? 1 : 0)
    switch (var) {
        case 1: XRS_TILES(128, 128, 16, 2, 4, 1, 2); break;
        case 2: XRS_TILES(64, 64, 16, 2, 4, 1, 4); break;
        case 3: XRS_TILES(64, 32, 16, 2, 2, 2, 2); break;
        case 5: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(64, 32, 32, 2, 2, 2, 4); break;
        case 6: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(64, 64, 32, 2, 2, 1, 4); break;
        case 7: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(64, 64, 32, 2, 2, 2, 4); break;
        case 8: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(64, 32, 16, 2, 2, 2, 4); break;
        case 9: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(32, 32, 16, 2, 2, 2, 4); break;
        case 10: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(32, 32, 32, 2, 2, 2, 2); break;
        case 11: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(32, 32, 16, 2, 2, 1, 2); break;
        case 12: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(32, 32, 32, 2, 2, 4, 2); break;
        case 13: if constexpr (std::is_same<PTR, GemmOne>::value) XRS_TILES(64, 32, 32, 2, 2, 2, 2); break;
        case 14: XRS_TILES(64, 80, 32, 4, 1, 2, 2); break;
        case 15: XRS_TILES(80, 64, 32, 1, 4, 2, 2); break;
        default: XRS_TILES(32, 32, 16, 2, 2, 2, 2); break;
    }
#undef XRS_TILES
    if (splits > 1 && tickets == nullptr) splitk_reduce(h, P, count, slab.d(), M, N, splits, alpha, sym);
}

void gemm(xrs_handle_t h, double* C, size_t Ms, size_t Ns, double alpha, const double* A, size_t lda, bool ta, size_t Ks,
          const double* B, size_t ldb, bool tb, int tri) {
    if (Ms == 0 || Ns == 0) return;
    XRS_REQUIRE(Ms < (1u << 30) && Ns < (1u << 30) && Ks < (1u << 30), "GEMM dimension too large");
    if (Ks == 0) {
        XRS_HIP(hipMemsetAsync(C, 0, Ms * Ns * 8, h->stream));
        return;
    }
    gemm_impl(h, GemmOne{A, B, C}, 1, Ms, Ns, alpha, lda, ta, Ks, ldb, tb, false, tri);
}

void gemm_sym(xrs_handle_t h, double* C, size_t Ns, double alpha, const double* A, size_t lda, bool ta, size_t Ks,
              const double* B, size_t ldb, bool tb) {
    if (Ns == 0) return;
    XRS_REQUIRE(Ns < (1u << 30) && Ks < (1u << 30), "GEMM dimension too large");
    if (Ks == 0) {
        XRS_HIP(hipMemsetAsync(C, 0, Ns * Ns * 8, h->stream));
        return;
    }
    gemm_impl(h, GemmOne{A, B, C}, 1, Ns, Ns, alpha, lda, ta, Ks, ldb, tb, true);
}

void gemm_batched(xrs_handle_t h, int count, double* const* C, size_t Ms, size_t Ns, double alpha, const double* const* A,
                  size_t lda, bool ta, size_t Ks, const double* const* B, size_t ldb, bool tb, bool sym, int tri) {
    XRS_REQUIRE(!sym || Ms == Ns, "symmetric batch needs square results");
    if (Ms == 0 || Ns == 0 || count <= 0) return;
    XRS_REQUIRE(Ms < (1u << 30) && Ns < (1u << 30) && Ks < (1u << 30), "GEMM dimension too large");
    if (Ks == 0) {
        for (int i = 0; i < count; ++i) XRS_HIP(hipMemsetAsync(C[i], 0, Ms * Ns * 8, h->stream));
        return;
    }
    for (int b0 = 0; b0 < count; b0 += kGemmBatchMax) {
        const int c = std::min(kGemmBatchMax, count - b0);
        GemmMany P{};
        for (int i = 0; i < c; ++i) {
            P.A[i] = A[b0 + i];
            P.B[i] = B[b0 + i];
            P.C[i] = C[b0 + i];
        }
        gemm_impl(h, P, c, Ms, Ns, alpha, lda, ta, Ks, ldb, tb, sym, tri);
    }
}

}  // namespace xrs

#ifdef XRS_GEMM_TRACE
extern "C" int xrs_debug_gemm_trace(void* buf, void* steps) {
    unsigned long long* p = static_cast<unsigned long long*>(buf);
    unsigned long long* q = static_cast<unsigned long long*>(steps);
    return hipMemcpyToSymbol(HIP_SYMBOL(xrs::g_gemm_trace), &p, sizeof(p)) == hipSuccess &&
                   hipMemcpyToSymbol(HIP_SYMBOL(xrs::g_gemm_steps), &q, sizeof(q)) == hipSuccess
               ? 0 : 1;
}
#endif

extern "C" int xrs_gemm(xrs_handle_t h, double* C, size_t M, size_t N, double alpha, const double* A, size_t lda,
                        int transA, size_t K, const double* B, size_t ldb, int transB) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(M == 0 || N == 0 || C, "null C");
        XRS_REQUIRE(K == 0 || M == 0 || N == 0 || (A && B), "null A/B");
        XRS_REQUIRE(transA ? lda >= M || K == 0 : lda >= K || M == 0, "lda too small");
        XRS_REQUIRE(transB ? ldb >= K || N == 0 : ldb >= N || K == 0, "ldb too small");
        XRS_REQUIRE(C != A && C != B, "C must not alias A or B");
        xrs::fence_readers(h);
        xrs::gemm(h, C, M, N, alpha, A, lda, transA != 0, K, B, ldb, transB != 0);
    });
}

extern "C" int xrs_gemm_batched(xrs_handle_t h, size_t count, double* const* C, size_t M, size_t N, double alpha,
                                const double* const* A, size_t lda, int transA, size_t K, const double* const* B,
                                size_t ldb, int transB) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(count == 0 || (A && B && C), "null pointer table");
        XRS_REQUIRE(count < (1u << 20), "batch too large");
        XRS_REQUIRE(transA ? lda >= M || K == 0 : lda >= K || M == 0, "lda too small");
        XRS_REQUIRE(transB ? ldb >= K || N == 0 : ldb >= N || K == 0, "ldb too small");
        for (size_t i = 0; i < count; ++i) {
            XRS_REQUIRE(M == 0 || N == 0 || C[i], "null C");
            XRS_REQUIRE(K == 0 || M == 0 || N == 0 || (A[i] && B[i]), "null A/B");
            XRS_REQUIRE(C[i] != A[i] && C[i] != B[i], "C must not alias A or B");
        }
        xrs::fence_readers(h);
        xrs::gemm_batched(h, int(count), C, M, N, alpha, A, lda, transA != 0, K, B, ldb, transB != 0, false);
    });
}

extern "C" int xrs_gemm_sym(xrs_handle_t h, double* C, size_t N, double alpha, const double* A, size_t lda, int transA,
                            size_t K, const double* B, size_t ldb, int transB) {
    return xrs::guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_REQUIRE(N == 0 || C, "null C");
        XRS_REQUIRE(K == 0 || N == 0 || (A && B), "null A/B");
        XRS_REQUIRE(transA ? lda >= N || K == 0 : lda >= K || N == 0, "lda too small");
        XRS_REQUIRE(transB ? ldb >= K || N == 0 : ldb >= N || K == 0, "ldb too small");
        XRS_REQUIRE(C != A && C != B, "C must not alias A or B");
        xrs::fence_readers(h);
        xrs::gemm_sym(h, C, N, alpha, A, lda, transA != 0, K, B, ldb, transB != 0);
    });
}
