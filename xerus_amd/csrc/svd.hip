// Right singular vectors of a small dense matrix by one-sided Jacobi on its rows (the SVD inside TT
// truncation: round_edge's calculate_svd, tensorNetwork.cpp:764 -> tensor.cpp:1424-1489 ->
// blasWrapper::svd / dgesdd, blasLapackWrapper.cpp:201-232).
//
// For W (p x q, p <= q) the rows are rotated pairwise until mutually orthogonal: J W = Wr, so
// sigma_i = ||Wr_i||, Vt_i = Wr_i / sigma_i and W = U S Vt with U S = W Vt^T -- the caller never needs J,
// so nothing but W is stored and for p*q <= 18 K doubles W lives in LDS for the whole solve.
//
// Layout of one round (round-robin "circle" pairing of the P = p rounded up to even players): pair t is
// (player at position t, player at position P-1-t); position 0 is fixed, the others rotate by one per
// round, so P-1 rounds meet every pair once (a sweep). A pair is handled by a group of 8 lanes (LDS
// kernel, 512 threads) or 16 lanes (global kernel): its three dot products are reduced with DPP
// butterflies (identical bits in every lane of the group, so all compute the same rotation), the
// rotation parameters come from hardware rcp/rsq estimates + Newton steps, and the rotation is applied
// in Rutishauser's form x' = x - s (y + tau x), y' = y + s (x - tau y) (O(u s) perturbation for
// nearly-identity rotations). 64 groups: up to 64 pairs per round in flight, one barrier per round.
// Convergence: no pair with |w_i . w_j| > tol ||w_i|| ||w_j||, tol = sqrt(q) u (dgesvj's criterion).
#include <cmath>
#include <cstdlib>

#include "smallla.hpp"

namespace xrs {

namespace {

constexpr int SV_LDS = 18432;   // doubles (144 KiB)
constexpr int SV_MAXP = 512;

// DPP move of a double (two 32-bit moves); CTRL is a DPP16 control word whose every lane has a valid
// source (row rotations / mirrors / quad permutations), so no "old" value is needed (mov_dpp: no
// zero-initialised destination, which update_dpp(0, ...) costs two extra moves per double)
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}


// Sum over a group of G (8, 16 or 32) consecutive lanes. Every lane of the group ends with the same bits:
// each step adds two values that are equal up to the order of operands of commutative adds.
//   G = 16: row_ror 8, 4, 2, 1 (rotations of an increasingly periodic sequence)
//   G = 8:  row_half_mirror (i <-> 7-i), quad_perm [2,3,0,1] (i <-> i^2), quad_perm [1,0,3,2] (i <-> i^1)
template <int G>
__device__ __forceinline__ double gsum(double v) {
    if constexpr (G == 16 || G == 32) {
        v += dpp<0x128>(v);
        v += dpp<0x124>(v);
        v += dpp<0x122>(v);
        v += dpp<0x121>(v);
        if constexpr (G == 32) {   // the two DPP rows of the group: the two results of v_permlane16_swap(v, v)
            // are {own, partner} on every lane, so their sum is the pair sum without a per-lane select
            const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
            v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
        }
    } else {
        static_assert(G == 8, "groups of 8 or 16 lanes");
        v += dpp<0x141>(v);
        v += dpp<0x4E>(v);
        v += dpp<0xB1>(v);
    }
    return v;
}

// 1/x and sqrt(x) to ~1 ulp from the hardware estimates + Newton steps (rotation parameters only need
// to be mutually consistent; no IEEE division / square-root sequences in the per-round critical path)
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double fsqrt(double x) {   // x > 0
    double y = __builtin_amdgcn_rsq(x);
    double h = 0.5 * y;
    double g = x * y;
    double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    r = fma(-g, h, 0.5);
    return fma(g, r, g);
}

// Jacobi rotation zeroing the (i,j) entry of [[a c][c b]]: t = tan(theta) = sign(b - a) 2c /
// (|b - a| + sqrt((b - a)^2 + 4 c^2)) (the smaller root), c = 1/sqrt(1+t^2), s = t c, tau = s / (1 + c)
__device__ __forceinline__ void rotation(double a, double b, double c, double& s, double& tau, double& tn) {
    const double dd = b - a;
    const double hh = fsqrt(fma(dd, dd, 4.0 * c * c));
    tn = copysign(2.0, dd) * c * frcp(fabs(dd) + hh);
    const double qq = fsqrt(fma(tn, tn, 1.0));   // 1 / cos
    s = tn * frcp(qq);
    tau = tn * frcp(1.0 + qq);   // = s / (1 + cos); Rutishauser: x' = x - s (y + tau x), y' = y + s (x - tau y)
}
__device__ __forceinline__ void rotation(double a, double b, double c, double& s, double& tau) {
    double tn;
    rotation(a, b, c, s, tau, tn);
}

// Early stop of the block kernel (flags & 2, the truncation sweeps): a sweep whose rotations all had
// |cos| = |w_i . w_j| / (||w_i|| ||w_j||) <= 1e-7 ends the iteration. Cyclic Jacobi converges quadratically,
// so the sweep that would follow rotates by ~1e-14 / (relative gap) at most: it only confirms convergence
// (measured on the graded cfg3 edges: the 5th sweep's largest |cos| was 2e-10 .. 2e-8, the 6th rotated
// nothing). The rows stay exactly a product of rotations (orthonormal V); the singular values move by
// O(cos^2) relatively.
constexpr double kEarlyCos2 = 1e-14;

// rows padded with zeros to E * G (no bounds checks: the padding stays zero under rotations)
template <int G, int E>
__device__ __forceinline__ void load_row_full(double (&x)[E], const double* __restrict__ w, int l) {
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = w[l + e * G];
}
template <int G, int E>
__device__ __forceinline__ void store_row_full(const double (&x)[E], double* __restrict__ w, int l) {
#pragma unroll
    for (int e = 0; e < E; ++e) w[l + e * G] = x[e];
}

// One Jacobi step on the row pair (wi, wj) of length q by a group of G lanes (lane l): orthogonalise the
// rows if |wi . wj| > tol ||wi|| ||wj||; true if rotated. E > 0: q <= E * G, the lane's elements are held
// in registers (all loads issued before any use); E = 0: any q, streamed.
// The register core: the lane's E elements of each row (zero beyond q, which rotations keep zero)
// (the inner products run over the first ew elements: the rest may carry accumulated rotations)
template <int G, int E>
__device__ __forceinline__ bool rotate_regs(double (&x)[E], double (&y)[E], double tol2, int ew = E, bool* big = nullptr) {
    double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (e < ew) {
            a = fma(x[e], x[e], a);
            b = fma(y[e], y[e], b);
            c = fma(x[e], y[e], c);
        }
    }
    a = gsum<G>(a);
    b = gsum<G>(b);
    c = gsum<G>(c);
    if (!(c * c > tol2 * a * b)) return false;
    if (big && c * c > kEarlyCos2 * a * b) *big = true;
    double s, tau;
    rotation(a, b, c, s, tau);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const double xe = x[e], ye = y[e];
        x[e] = xe - s * fma(tau, xe, ye);
        y[e] = ye + s * fma(-tau, ye, xe);
    }
    return true;
}

template <int G, int E>
__device__ __forceinline__ void load_row(double (&x)[E], const double* __restrict__ w, int q, int l) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = l + e * G;
        x[e] = k < q ? w[k] : 0.0;
    }
}

template <int G, int E>
__device__ __forceinline__ void store_row(const double (&x)[E], double* __restrict__ w, int q, int l) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = l + e * G;
        if (k < q) w[k] = x[e];
    }
}

// One Jacobi step on the row pair (wi, wj) of length q by a group of G lanes (lane l): orthogonalise the
// rows if |wi . wj| > tol ||wi|| ||wj||; true if rotated. E > 0: q <= E * G, the lane's elements are held
// in registers (all loads issued before any use); E = 0: any q, streamed.
template <int G, int E>
__device__ __forceinline__ bool rotate_pair(double* __restrict__ wi, double* __restrict__ wj, int q, int l, double tol2) {
    if constexpr (E > 0) {
        double x[E], y[E];
        load_row<G, E>(x, wi, q, l);
        load_row<G, E>(y, wj, q, l);
        if (!rotate_regs<G, E>(x, y, tol2)) return false;
        store_row<G, E>(x, wi, q, l);
        store_row<G, E>(y, wj, q, l);
        return true;
    } else {
        double a = 0.0, b = 0.0, c = 0.0;
        for (int k = l; k < q; k += G) {
            const double x = wi[k], y = wj[k];
            a = fma(x, x, a);
            b = fma(y, y, b);
            c = fma(x, y, c);
        }
        a = gsum<G>(a);
        b = gsum<G>(b);
        c = gsum<G>(c);
        if (!(c * c > tol2 * a * b)) return false;
        double s, tau;
        rotation(a, b, c, s, tau);
        for (int k = l; k < q; k += G) {
            const double x = wi[k], y = wj[k];
            wi[k] = x - s * fma(tau, x, y);
            wj[k] = y + s * fma(-tau, y, x);
        }
        return true;
    }
}

// player at position x of round `round` (circle method, P players, position 0 fixed)
__device__ __forceinline__ int player(int x, int round, int P) { return x == 0 ? 0 : 1 + (x - 1 + round) % (P - 1); }

// W (ldw) is the working copy (LDS or global scratch); Win (row stride ldin, or transposed) the input.
// E > 0: q <= E * G, the lane's elements of a row pair are held in registers (unrolled); E = 0: any q
template <int G, int NT, int E>
__device__ void jacobi_rows_body(double* __restrict__ W, int ldw, const double* __restrict__ Win, int ldin, bool trans, int p, int q,
                                 int max_sweeps, double* __restrict__ S, double* __restrict__ Vt, int ldvt,
                                 int* __restrict__ status) {
    constexpr int GROUPS = NT / G;
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    __shared__ int rotated;
    __shared__ double sn[SV_MAXP];
    __shared__ int rk[SV_MAXP];
    if (trans) {   // W[i][k] = Win[k][i]: read along Win's rows
        for (int e = tid; e < p * q; e += NT) {
            const int k = e / p, i = e - k * p;
            W[size_t(i) * ldw + k] = Win[size_t(k) * ldin + i];
        }
    } else {
        for (int e = tid; e < p * q; e += NT) {
            const int i = e / q, k = e - i * q;
            W[size_t(i) * ldw + k] = Win[size_t(i) * ldin + k];
        }
    }
    __syncthreads();
    const int P = (p + 1) & ~1;
    const double tol = sqrt(double(q)) * 1.1102230246251565e-16;
    const double tol2 = tol * tol;
    int sweep = 0;
    bool converged = false;
    for (; sweep < max_sweeps && !converged; ++sweep) {
        if (tid == 0) rotated = 0;
        __syncthreads();
        for (int round = 0; round < P - 1; ++round) {
            for (int t = g; t < P / 2; t += GROUPS) {
                int i = 0, j;   // players at positions t and P-1-t (player() without the integer divisions)
                if (t > 0) {
                    i = t + round;
                    i = i >= P ? i - (P - 1) : i;
                }
                j = P - 1 - t + round;
                j = j >= P ? j - (P - 1) : j;
                if (i >= p || j >= p) continue;
                if (rotate_pair<G, E>(W + size_t(i) * ldw, W + size_t(j) * ldw, q, l, tol2) && l == 0) rotated = 1;
            }
            __syncthreads();
        }
        converged = rotated == 0;
        __syncthreads();
    }
    // singular values = row norms, ranked descending (ties by index: a stable order)
    for (int i = g; i < p; i += GROUPS) {
        const double* wi = W + size_t(i) * ldw;
        double a = 0.0;
        for (int k = l; k < q; k += G) a = fma(wi[k], wi[k], a);
        a = gsum<G>(a);
        if (l == 0) sn[i] = sqrt(a);
    }
    __syncthreads();
    for (int i = tid; i < p; i += NT) {
        const double si = sn[i];
        int r = 0;
        for (int j2 = 0; j2 < p; ++j2) r += (sn[j2] > si) || (sn[j2] == si && j2 < i);
        rk[i] = r;
        S[r] = si;
    }
    __syncthreads();
    for (int e = tid; e < p * q; e += NT) {
        const int i = e / q, k = e - i * q;
        const double s = sn[i];
        Vt[size_t(rk[i]) * ldvt + k] = s > 0.0 ? W[size_t(i) * ldw + k] / s : 0.0;
    }
    if (tid == 0) status[0] = converged ? sweep : -1;
}

// LDS-resident: 512 threads, 8 lanes per pair (64 pairs in flight, two waves per SIMD)
constexpr int SVL_THREADS = 512;
__global__ void __launch_bounds__(SVL_THREADS) k_jacobi_vt_lds(const double* __restrict__ Win, int ldin, int trans, int p, int q,
                                                               int max_sweeps, double* __restrict__ S, double* __restrict__ Vt,
                                                               int ldvt, int* __restrict__ status) {
    __shared__ double Ws[SV_LDS];
    const int ldw = q + ((q & 1) ? 0 : 1);   // odd stride: the rows a wave touches spread over the banks
    jacobi_rows_body<8, SVL_THREADS, 16>(Ws, ldw, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
}

// W in global memory (L2-resident) for larger matrices: 1024 threads, 16 lanes per pair
constexpr int SVG_THREADS = 1024;
__global__ void __launch_bounds__(SVG_THREADS) k_jacobi_vt_global(double* __restrict__ Wg, const double* __restrict__ Win, int ldin,
                                                                  int trans, int p, int q, int max_sweeps, double* __restrict__ S,
                                                                  double* __restrict__ Vt, int ldvt, int* __restrict__ status) {
    if (q <= 256) jacobi_rows_body<16, SVG_THREADS, 16>(Wg, q, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
    else jacobi_rows_body<16, SVG_THREADS, 0>(Wg, q, Win, ldin, trans != 0, p, q, max_sweeps, S, Vt, ldvt, status);
}


// ---- multi-workgroup block Jacobi (p >= 32): the rows are cut into nb blocks of BR rows (the last ones
// padded with zero rows); workgroup w holds the block pair at positions (w, nb-1-w) of the circle
// tournament over blocks -- 2 BR rows x q in LDS, each block contiguous -- and per outer round
// orthogonalises the BR x BR cross pairs (BR rounds of BR disjoint pairs, a 16-lane group per pair, the
// group's top row register-resident); the pairs inside each block are done once per sweep, in its
// first outer round. Then every block goes through global memory to the workgroup that pairs it next.
// nb - 1 outer rounds are one sweep (every row pair exactly once); converged when a whole sweep rotated
// nothing.
// Hand-off between outer rounds (MI355X_MICROARCH.md, inter-workgroup visibility, row 1 of the sc1
// table): every byte of a block is stored and loaded with 16-B write-through (sc1) buffer accesses,
// every wave drains its stores (vmcnt(0)) before the workgroup barrier behind which lane 0 adds to the
// grid counter (agent atomic), the poll is an sc1 load and the other waves load after the workgroup
// barrier that the polling wave joins -- no release/acquire fences (no L2 write-back or L1 invalidate
// per round). The poll is bounded (status -2 instead of a hang if a workgroup were never scheduled).
constexpr int SVB_G = 16, SVB_LDS = 16384, SVB_QMAX = 512;
constexpr int SVB_SYNC_WORDS = 128;  // [0] barrier counter, [1 + sweep] rotated flags, [64 + sweep] |cos| > 1e-7 flags
typedef int svb_v4i __attribute__((ext_vector_type(4)));
constexpr int kBufCfg = 0x00020000;  // raw buffer descriptor word 3 (32-bit data format)
constexpr int kSc1 = 16;             // cache policy: sc1 (write-through stores, L1-bypassing loads)

__device__ __forceinline__ void grid_arrive_wait(unsigned* counter, unsigned target, int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 26)) {
                *err = 1;
                break;
            }
        }
    }
    __syncthreads();
}

// LDS block (contiguous, 16-B aligned) <-> global slot, 16-B sc1 accesses, 4 per lane in flight
template <int NT>
__device__ __forceinline__ void block_out(const double* lds, __amdgpu_buffer_rsrc_t rs, int byte0, int units, int tid) {
    for (int u0 = 0; u0 < units; u0 += 4 * NT) {
        svb_v4i v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int u = u0 + i * NT + tid;
            if (u < units) v[i] = *reinterpret_cast<const svb_v4i*>(lds + 2 * u);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int u = u0 + i * NT + tid;
            if (u < units) __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, byte0 + 16 * u, 0, kSc1);
        }
    }
}
template <int NT>
__device__ __forceinline__ void block_in(double* lds, __amdgpu_buffer_rsrc_t rs, int byte0, int units, int tid) {
    for (int u0 = 0; u0 < units; u0 += 8 * NT) {
        svb_v4i v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int u = u0 + i * NT + tid;
            if (u < units) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, byte0 + 16 * u, 0, kSc1);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int u = u0 + i * NT + tid;
            if (u < units) *reinterpret_cast<svb_v4i*>(lds + 2 * u) = v[i];
        }
    }
}

template <int BR, int G, int E, bool ACC>
__global__ void __launch_bounds__(BR * G) k_jacobi_vt_blocks(const double* __restrict__ Win, int ldin, int trans, int p, int q,
                                                                 int nb, int max_sweeps, double* __restrict__ slots,
                                                                 unsigned* __restrict__ sync, double* __restrict__ norms,
                                                                 double* __restrict__ S, double* __restrict__ Vt, int ldvt,
                                                                 double* __restrict__ U, int ldu, int* __restrict__ status, int flags) {
    constexpr int NT = BR * G, R2 = 2 * BR;
    const bool stamps = (flags & 1) != 0, early = (flags & 2) != 0;
    // diagnostics (stamps != 0, XRS_SVD_TIMING): cycles of thread 0 per cross-round phase -- dot + sum,
    // rotation parameters, update + store, barrier wait -- and the rotation count, into status[4..8]
    unsigned long long st_ph[5] = {0ull, 0ull, 0ull, 0ull, 0ull};
    static_assert((BR & (BR - 1)) == 0 && BR >= 4, "BR: a power of two");
    __shared__ __attribute__((aligned(16))) double Ws[SVB_LDS];
    __shared__ int rotated, err, bigrot;
    __shared__ double bn[BR];   // squared norms of the bottom rows during the cross rounds
    __shared__ int part[NT / 64 > 0 ? NT / 64 : 1];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int w = blockIdx.x, nwg = gridDim.x;
    constexpr int ldw = E * G;      // rows zero-padded to the register tiling; blocks contiguous
    constexpr int bunits = BR * ldw / 2;   // 16-B units per block
    static_assert(2 * BR * ldw <= SVB_LDS, "block pair exceeds the LDS buffer");
    double* const Wb = Ws + BR * ldw;   // bottom block
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slots, 0, nb * BR * ldw * 8, kBufCfg);
    // with U: every row carries its row of the accumulated rotation J (W' = J W) after the zero-padded
    // data, [w (ew * G) | j (p)]; dots and norms run over the first ew register elements only
    const int ew = ACC ? (q + G - 1) / G : E;
    const int qpad = ew * G;
    const double tol = sqrt(double(q)) * 1.1102230246251565e-16;
    const double tol2 = tol * tol;
    if (tid == 0) err = 0;
    // block id at tournament position x in outer round t
    auto block_at = [&](int x, int t) { return x == 0 ? 0 : 1 + (x - 1 + t) % (nb - 1); };
    auto row_of = [&](int r, int top, int bot) { return (r < BR ? top : bot) * BR + (r % BR); };
    unsigned barriers = 0;
    long long t_bar = 0, t_xch = 0;
    const long long t_start = wall_clock64();
    int top = block_at(w, 0), bot = block_at(nb - 1 - w, 0);
    for (int e = tid; e < R2 * ldw; e += NT) {
        const int r = e / ldw, k = e % ldw;
        const int row = row_of(r, top, bot);
        double v = 0.0;
        if (row < p) {
            if (k < q) v = trans ? Win[size_t(k) * ldin + row] : Win[size_t(row) * ldin + k];
            else if (ACC && k - qpad == row) v = 1.0;
        }
        Ws[e] = v;
    }
    __syncthreads();
    int sweep = 0;
    bool converged = false;
    while (sweep < max_sweeps && !converged) {
        if (tid == 0) {
            rotated = 0;
            bigrot = 0;
        }
        __syncthreads();
        bool big = false;   // (this thread's group rotated by |cos| > 1e-7 in this sweep)
        for (int t = 0; t < nb - 1; ++t) {
            if (t == 0) {
                // first outer round of the sweep: the pairs inside each block (circle method over BR
                // rows; the first half of the groups on the top block, the second on the bottom one)
                constexpr int HALF = BR / 2;
                const int gg = g % HALF, base = g < HALF ? 0 : BR;
                for (int round = 0; round < BR - 1; ++round) {
                    const int i = player(gg, round, BR), j = player(BR - 1 - gg, round, BR);
                    double x[E], y[E];
                    load_row_full<G, E>(x, Ws + (base + i) * ldw, l);
                    load_row_full<G, E>(y, Ws + (base + j) * ldw, l);
                    if (rotate_regs<G, E>(x, y, tol2, ew, &big)) {
                        store_row_full<G, E>(x, Ws + (base + i) * ldw, l);
                        store_row_full<G, E>(y, Ws + (base + j) * ldw, l);
                        if (l == 0) rotated = 1;
                    }
                    __syncthreads();
                }
            }
            // the cross pairs: group g keeps top row g in registers and meets bottom row (g + s) mod BR
            // in round s. Squared norms are computed once per outer round and then updated with the
            // rotation (a' = a - t c, b' = b + t c); a drop below half is recomputed (cancellation guard)
            {
                double x[E], y[E];
                load_row_full<G, E>(x, Ws + g * ldw, l);
                load_row_full<G, E>(y, Wb + g * ldw, l);
                double a = 0.0, bb = 0.0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if (e < ew) {
                        a = fma(x[e], x[e], a);
                        bb = fma(y[e], y[e], bb);
                    }
                }
                a = gsum<G>(a);
                bb = gsum<G>(bb);
                if (l == 0) bn[g] = bb;
                __syncthreads();
                bool rot = false;
                for (int sr = 0; sr < BR; ++sr) {
                    const unsigned long long c0 = stamps ? __builtin_amdgcn_s_memtime() : 0ull;
                    const int jb = (g + sr) & (BR - 1);
                    double* wb = Wb + jb * ldw;
                    load_row_full<G, E>(y, wb, l);
                    const double b = bn[jb];
                    double c4[4] = {0.0, 0.0, 0.0, 0.0};   // four chains: the dot is latency-bound
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        if (e < ew) c4[e & 3] = fma(x[e], y[e], c4[e & 3]);
                    const double c = gsum<G>((c4[0] + c4[1]) + (c4[2] + c4[3]));
                    const bool do_rot = c * c > tol2 * a * b;
                    big = big || (do_rot && c * c > kEarlyCos2 * a * b);
                    unsigned long long c1 = 0ull, c2 = 0ull;
                    if (stamps) {
                        c1 = __builtin_amdgcn_s_memtime() + (do_rot ? 0ull : 0ull);
                        st_ph[0] += c1 - c0;
                    }
                    if (do_rot) {
                        double sn, tau, tn = 0.0;
                        rotation(a, b, c, sn, tau, tn);
                        if (stamps) {
                            c2 = __builtin_amdgcn_s_memtime() + (sn != sn ? 1ull : 0ull);
                            st_ph[1] += c2 - c1;
                            ++st_ph[4];
                        }
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const double xe = x[e], ye = y[e];
                            x[e] = xe - sn * fma(tau, xe, ye);
                            y[e] = ye + sn * fma(-tau, ye, xe);
                        }
                        double an = fma(-tn, c, a), bnew = fma(tn, c, b);
                        if (an < 0.5 * a) {
                            an = 0.0;
#pragma unroll
                            for (int e = 0; e < E; ++e)
                                if (e < ew) an = fma(x[e], x[e], an);
                            an = gsum<G>(an);
                        }
                        if (bnew < 0.5 * b) {
                            bnew = 0.0;
#pragma unroll
                            for (int e = 0; e < E; ++e)
                                if (e < ew) bnew = fma(y[e], y[e], bnew);
                            bnew = gsum<G>(bnew);
                        }
                        a = an;
                        store_row_full<G, E>(y, wb, l);
                        if (l == 0) bn[jb] = bnew;
                        rot = true;
                        if (stamps) {
                            const unsigned long long c3 = __builtin_amdgcn_s_memtime();
                            st_ph[2] += c3 - c2;
                            c1 = c3;
                        }
                    }
                    __syncthreads();
                    if (stamps) st_ph[3] += __builtin_amdgcn_s_memtime() - c1;
                }
                store_row_full<G, E>(x, Ws + g * ldw, l);
                if (rot && l == 0) rotated = 1;
                __syncthreads();
            }
            // exchange: every block to the slot of its id, then the pair of the next outer round (block 0
            // never leaves workgroup 0's top)
            const long long t0 = wall_clock64();
            if (top != 0) block_out<NT>(Ws, rs, top * bunits * 16, bunits, tid);
            block_out<NT>(Wb, rs, bot * bunits * 16, bunits, tid);
            if (t == nb - 2 && early) {
                if (big && l == 0) bigrot = 1;
                __syncthreads();
            }
            if (t == nb - 2 && tid == 0 && rotated)
                __hip_atomic_fetch_or(&sync[1 + sweep], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t == nb - 2 && tid == 0 && early && bigrot)
                __hip_atomic_fetch_or(&sync[64 + sweep], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long t1 = wall_clock64();
            grid_arrive_wait(&sync[0], ++barriers * unsigned(nwg), &err);
            const long long t2 = wall_clock64();
            const int tn = (t + 1) % (nb - 1);
            top = block_at(w, tn);
            bot = block_at(nb - 1 - w, tn);
            if (top != 0) block_in<NT>(Ws, rs, top * bunits * 16, bunits, tid);
            block_in<NT>(Wb, rs, bot * bunits * 16, bunits, tid);
            __syncthreads();
            t_bar += t2 - t1;
            t_xch += (t1 - t0) + (wall_clock64() - t2);
        }
        // every workgroup reads the same flag (all were set before the last barrier of the sweep)
        if (tid == 0) {
            rotated = int(__hip_atomic_load(&sync[1 + sweep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (early && rotated) rotated = int(__hip_atomic_load(&sync[64 + sweep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        __syncthreads();
        converged = rotated == 0;
        ++sweep;
        if (err) break;
        __syncthreads();
    }
    // singular values = row norms (published with sc1 stores); global ranks after one more barrier
    for (int r = g; r < R2; r += BR) {
        const double* wr = Ws + r * ldw;
        double a = 0.0;
        for (int k = l; k < qpad; k += G) a = fma(wr[k], wr[k], a);
        a = gsum<G>(a);
        const int row = row_of(r, top, bot);
        if (l == 0 && row < p) __hip_atomic_store(&norms[row], sqrt(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_arrive_wait(&sync[0], ++barriers * unsigned(nwg), &err);
    for (int r = 0; r < R2; ++r) {
        const int row = row_of(r, top, bot);
        if (row >= p) continue;
        const double si = __hip_atomic_load(&norms[row], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int rk = 0;
        for (int j2 = tid; j2 < p; j2 += NT) {
            const double sj = __hip_atomic_load(&norms[j2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            rk += (sj > si) || (sj == si && j2 < row);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) rk += __shfl_xor(rk, o, 64);
        if ((tid & 63) == 0) part[tid >> 6] = rk;
        __syncthreads();
        int rank = 0;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) rank += part[i];
        __syncthreads();
        if (tid == 0) S[rank] = si;
        const double inv = si > 0.0 ? 1.0 / si : 0.0;
        for (int k = tid; k < q; k += NT) Vt[size_t(rank) * ldvt + k] = Ws[r * ldw + k] * inv;
        if (ACC)   // W = J^T W': U = J^T, column `rank` = row r of J
            for (int i2 = tid; i2 < p; i2 += NT) U[size_t(i2) * ldu + rank] = Ws[r * ldw + qpad + i2];
    }
    if (w == 0 && tid == 0) {
        status[0] = err ? -2 : (converged ? sweep : -1);
        status[1] = int(wall_clock64() - t_start);   // 100 MHz ticks (diagnostics)
        status[2] = int(t_bar);
        status[3] = int(t_xch);
        if (stamps)
            for (int i = 0; i < 5; ++i) status[4 + i] = int(st_ph[i]);
    }
}

}  // namespace

bool jacobi_vt_fits_lds(int p, int q) { return q <= 128 && size_t(p) * size_t(q + 1) <= size_t(SV_LDS); }

namespace {

// block kernel launch: nb = ceil(p / BR) rounded up to even, nb / 2 one-CU workgroups (<= 32 here:
// co-resident on any MI355X, which the grid barrier needs)
template <int BR, int G, int E, bool ACC>
void launch_blocks(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* S, double* Vt, int ldvt, double* U,
                   int ldu, int* status_dev, int max_sweeps, bool stamps = false, bool early = false) {
    int nb = (p + BR - 1) / BR;
    nb += nb & 1;
    const int sweeps = std::min(max_sweeps, 63);
    DevBuf slots(h, size_t(nb) * BR * E * G * 8), sync(h, SVB_SYNC_WORDS * 4), norms(h, size_t(p) * 8);
    XRS_HIP(hipMemsetAsync(sync.d(), 0, SVB_SYNC_WORDS * 4, h->stream));
    hipLaunchKernelGGL((k_jacobi_vt_blocks<BR, G, E, ACC>), dim3(nb / 2), dim3(BR * G), 0, h->stream, W, ldw, int(trans), p, q, nb, sweeps,
                       slots.d(), sync.as<unsigned>(), norms.d(), S, Vt, ldvt, U, ldu, status_dev, (stamps ? 1 : 0) | (early ? 2 : 0));
    check_launch("k_jacobi_vt_blocks");
}

}  // namespace

void jacobi_vt(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* S, double* Vt, int ldvt,
               int* status_dev, int max_sweeps, int kernel, bool stamps, bool early) {
    XRS_REQUIRE(p >= 1 && p <= q && (p <= SV_MAXP || (q <= 2 * SVB_QMAX && kernel != 1)),
                "jacobi_vt: need 1 <= p <= q, p <= 512 (one workgroup) or q <= 1024 (blocks)");
    XRS_REQUIRE(kernel >= 0 && kernel <= 2, "jacobi_vt: kernel is 0 (auto), 1 (one workgroup) or 2 (blocks)");
    KernelTimer timer(h, XRS_KFAM_SVD, 3.5 * double(p) * p * q * 6.0, 16.0 * double(p) * q);
    // smallest p handed to the multi-workgroup block kernel (measured faster than the one-workgroup kernel
    // from p = 64 on: 0.59 vs 0.73 ms at 64, 1.19 vs 2.62 ms at 128)
    constexpr int block_min = 32;
    const bool blocks_ok = q <= 2 * SVB_QMAX;
    XRS_REQUIRE(kernel != 2 || blocks_ok, "jacobi_vt: the block kernel needs q <= 1024");
    if (q > SVB_QMAX) {   // rows of up to 1024 columns: blocks of 8 rows (2 x 8 x 1024 doubles of LDS)
        launch_blocks<8, 32, 32, false>(h, W, ldw, trans, p, q, S, Vt, ldvt, nullptr, 0, status_dev, max_sweeps, stamps, early);
    } else if (blocks_ok && (kernel == 2 || (kernel == 0 && p >= block_min))) {
        // register tiling E * 32 columns: the narrowest that holds q (padding costs FMAs and LDS traffic)
        if (q <= 64) launch_blocks<16, 32, 2, false>(h, W, ldw, trans, p, q, S, Vt, ldvt, nullptr, 0, status_dev, max_sweeps, stamps, early);
        else if (q <= 128) launch_blocks<16, 32, 4, false>(h, W, ldw, trans, p, q, S, Vt, ldvt, nullptr, 0, status_dev, max_sweeps, stamps, early);
        else if (q <= 256) launch_blocks<16, 32, 8, false>(h, W, ldw, trans, p, q, S, Vt, ldvt, nullptr, 0, status_dev, max_sweeps, stamps, early);
        else launch_blocks<16, 32, 16, false>(h, W, ldw, trans, p, q, S, Vt, ldvt, nullptr, 0, status_dev, max_sweeps, stamps, early);
    } else if (jacobi_vt_fits_lds(p, q)) {
        hipLaunchKernelGGL(k_jacobi_vt_lds, dim3(1), dim3(SVL_THREADS), 0, h->stream, W, ldw, int(trans), p, q, max_sweeps, S, Vt,
                           ldvt, status_dev);
        check_launch("k_jacobi_vt_lds");
    } else {
        DevBuf Wg(h, size_t(p) * q * 8);
        hipLaunchKernelGGL(k_jacobi_vt_global, dim3(1), dim3(SVG_THREADS), 0, h->stream, Wg.d(), W, ldw, int(trans), p, q, max_sweeps,
                           S, Vt, ldvt, status_dev);
        check_launch("k_jacobi_vt_global");
    }
}

bool jacobi_usv_fits(int p, int q) { return p >= 1 && p <= q && 32 * ((q + 31) / 32) + p <= 1024; }

void jacobi_usv(xrs_handle_t h, const double* W, int ldw, bool trans, int p, int q, double* U, int ldu, double* S, double* Vt, int ldvt,
                int* status_dev, int max_sweeps, bool early) {
    XRS_REQUIRE(jacobi_usv_fits(p, q), "jacobi_usv: need p <= q and 32 ceil(q / 32) + p <= 1024");
    KernelTimer timer(h, XRS_KFAM_SVD, 3.5 * double(p) * p * (q + p) * 6.0, 16.0 * double(p) * (q + p));
    const int width = 32 * ((q + 31) / 32) + p;
    if (width <= 128) launch_blocks<16, 32, 4, true>(h, W, ldw, trans, p, q, S, Vt, ldvt, U, ldu, status_dev, max_sweeps, false, early);
    else if (width <= 256) launch_blocks<16, 32, 8, true>(h, W, ldw, trans, p, q, S, Vt, ldvt, U, ldu, status_dev, max_sweeps, false, early);
    else if (width <= 512) launch_blocks<16, 32, 16, true>(h, W, ldw, trans, p, q, S, Vt, ldvt, U, ldu, status_dev, max_sweeps, false, early);
    else launch_blocks<8, 32, 32, true>(h, W, ldw, trans, p, q, S, Vt, ldvt, U, ldu, status_dev, max_sweeps, false, early);
}

int jacobi_settle(xrs_handle_t h, int* status_dev, int p, int q, const std::function<void(int kernel)>& rerun) {
    int sweeps = 0;
    read_status(h, status_dev, 1, &sweeps);
    for (int attempt = 0; sweeps == -2 && attempt < 2; ++attempt) {
        // one workgroup where it fits (no grid barrier at all), else the block kernel once more
        const int kernel = (p <= SV_MAXP && attempt == 0) ? 1 : 2;
        std::fprintf(stderr, "[xerus_amd warning] multi-workgroup Jacobi barrier timed out (%d x %d); rerun (kernel %d)\n", p, q, kernel);
        XRS_HIP(hipMemsetAsync(status_dev, 0, 4, h->stream));
        rerun(kernel);
        read_status(h, status_dev, 1, &sweeps);
    }
    if (sweeps == -2) throw Error{XRS_ENUMERIC, "one-sided Jacobi: the multi-workgroup kernel's grid barrier timed out twice"};
    if (sweeps < 0)
        std::fprintf(stderr, "[xerus_amd warning] SVD failed: one-sided Jacobi of a %d x %d matrix did not converge (status %d)\n", p, q,
                     sweeps);
    return sweeps;
}

// Right singular vectors of a g x g triangular factor F (rows of Vt, S descending) for the truncation
// sweeps. A lower factor (wide edge, B = L Q) is handled through the rows of F^T with the rotations
// accumulated: J F^T = S U^T gives F = U S J, so V = J^T is a product of rotations (orthonormal to u,
// no division by S), and Jacobi on the columns of a triangular factor converges in about as many sweeps
// for graded as for flat spectra (10-11 at g = 128; the rows of a lower factor of a graded matrix take
// ~30). An upper factor (tall edge, B = Q R) already has the good orientation: rows of F.
void jacobi_right_vectors(xrs_handle_t h, const double* F, int g, bool lower, double* S, double* Vt, int* status_dev, int max_sweeps,
                          bool early) {
    if (!lower || !jacobi_usv_fits(g, g)) {
        jacobi_vt(h, F, g, false, g, g, S, Vt, g, status_dev, max_sweeps, 0, false, early);
        return;
    }
    DevBuf J(h, size_t(g) * g * 8), Ul(h, size_t(g) * g * 8);
    jacobi_usv(h, F, g, true, g, g, J.d(), g, S, Ul.d(), g, status_dev, max_sweeps, early);   // J.d()[i][j] = v_j[i]
    transpose(h, Vt, J.d(), size_t(g), size_t(g));
}

}  // namespace xrs
