// Diagnostic microbenchmark of the single-workgroup Cholesky (k_potrf_rr) and the MFMA TRSM:
// per-phase s_memtime stamps of one factorisation plus mean kernel times over repetitions.
// Build: make -C tools potrf_bench  (compiles smallla.hip into this TU with XRS_POTRF_STAMPS).
#define XRS_POTRF_STAMPS 1
#include "../xerus_amd/csrc/smallla.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace xrs;

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 256;
    const int m = argc > 2 ? atoi(argv[2]) : 5120;
    xrs_handle_t h;
    if (xrs_create(&h, 0) != 0) { printf("no device\n"); return 1; }
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd;
    std::vector<double> A(size_t(m) * n), G(size_t(n) * n, 0.0);
    for (auto& v : A) v = nd(rng);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k <= i; ++k) {
            double s = 0;
            for (int r = 0; r < m; ++r) s += A[size_t(r) * n + i] * A[size_t(r) * n + k];
            G[size_t(i) * n + k] = G[size_t(k) * n + i] = s;
        }
    double *dG, *dW, *dDi, *dA, *dX;
    int* dst;
    long long* dstamps;
    hipMalloc(&dG, G.size() * 8); hipMalloc(&dW, G.size() * 8); hipMalloc(&dDi, size_t(n + 32) * 32 * 8);
    hipMalloc(&dA, A.size() * 8); hipMalloc(&dX, A.size() * 8); hipMalloc(&dst, 64); hipMalloc(&dstamps, 4096 * 8);
    hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpyToSymbol(HIP_SYMBOL(g_potrf_stamps), &dstamps, sizeof(dstamps));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int reps = 20;
    float ms = 0;
    // Cholesky
    for (int it = 0; it < reps + 2; ++it) {
        hipMemcpyAsync(dW, dG, G.size() * 8, hipMemcpyDeviceToDevice, h->stream);
        if (it == 2) hipEventRecord(e0, h->stream);
        potrf(h, dW, n, 0.0, dDi, dst, nullptr);
    }
    hipEventRecord(e1, h->stream);
    hipStreamSynchronize(h->stream);
    hipEventElapsedTime(&ms, e0, e1);
    printf("potrf n=%d: %.1f us per call (incl. %zu-byte copy)\n", n, ms * 1e3 / reps, G.size() * 8);
    std::vector<long long> st(4096);
    hipMemcpy(st.data(), dstamps, st.size() * 8, hipMemcpyDeviceToHost);
    const int T = (n + 15) / 16;
    double tA = 0, tB = 0, tC = 0, tD = 0;
    for (int j = 0; j < T; ++j) {
        const long long a = st[2 + 4 * j], b = st[3 + 4 * j], c = st[4 + 4 * j];
        const long long nxt = (j + 1 < T) ? st[2 + 4 * (j + 1)] : st[1];
        const long long prev = (j == 0) ? st[0] : st[4 + 4 * (j - 1)];
        tA += a - prev; tB += b - a; tC += c - b; tD += nxt - c;
        if (j < 3 || j == T - 1)
            printf("  j=%2d  A(+D prev) %6lld  B %6lld  C %6lld\n", j, a - prev, b - a, c - b);
    }
    printf("  last block: factor %lld  inverse+rest %lld\n", st[1000] - st[2 + 4 * (T - 1)], st[3 + 4 * (T - 1)] - st[1000]);
    printf("  totals (memtime ticks): A+Dprev %.0f  B %.0f  C %.0f  total %lld\n", tA, tB, tC, st[1] - st[0]);
    // TRSM (tall: X = A L^{-T})
    for (int it = 0; it < reps + 2; ++it) {
        if (it == 2) hipEventRecord(e0, h->stream);
        trsm(h, false, dW, dDi, n, dA, n, dX, n, m);
    }
    hipEventRecord(e1, h->stream);
    hipStreamSynchronize(h->stream);
    hipEventElapsedTime(&ms, e0, e1);
    printf("trsm rows n=%d m=%d: %.1f us per call  (%.2f TFLOP/s)\n", n, m, ms * 1e3 / reps,
           double(n) * n * m / (ms * 1e-3 / reps) / 1e12);
    // TRSM (wide: X = L^{-1} Y, the chain-round transform shape)
    for (int it = 0; it < reps + 2; ++it) {
        if (it == 2) hipEventRecord(e0, h->stream);
        trsm(h, true, dW, dDi, n, dA, m, dX, m, m);
    }
    hipEventRecord(e1, h->stream);
    hipStreamSynchronize(h->stream);
    hipEventElapsedTime(&ms, e0, e1);
    printf("trsm cols n=%d m=%d: %.1f us per call  (%.2f TFLOP/s)\n", n, m, ms * 1e3 / reps,
           double(n) * n * m / (ms * 1e-3 / reps) / 1e12);
    // check Cholesky residual on the host
    std::vector<double> L(G.size());
    hipMemcpy(L.data(), dW, L.size() * 8, hipMemcpyDeviceToHost);
    double err = 0, nrm = 0;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k <= i; ++k) {
            double s = 0;
            for (int r = 0; r <= k; ++r) s += L[size_t(i) * n + r] * L[size_t(k) * n + r];
            err = std::max(err, std::fabs(s - G[size_t(i) * n + k]));
            nrm = std::max(nrm, std::fabs(G[size_t(i) * n + k]));
        }
    printf("max |L L^T - G| / max|G| = %.3e\n", err / nrm);
    xrs_destroy(h);
    return 0;
}
