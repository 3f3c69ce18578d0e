"""Kernel microbenchmarks through the C-ABI (kernel time from HIP events around each launch)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402


def bench_gemm(h, M, N, K, ta, tb, reps=20):
    rng = np.random.default_rng(0)
    A = h.array(rng.standard_normal((K, M) if ta else (M, K)))
    B = h.array(rng.standard_normal((N, K) if tb else (K, N)))
    C = h.empty((M, N))
    for _ in range(3):
        h.gemm(C, M, N, 1.0, A, A.shape[1], ta, K, B, B.shape[1], tb)
    h.synchronize()
    h.prof_begin(capi.KFAM_GEMM)
    t0 = time.perf_counter()
    for _ in range(reps):
        h.gemm(C, M, N, 1.0, A, A.shape[1], ta, K, B, B.shape[1], tb)
    h.synchronize()
    wall = (time.perf_counter() - t0) / reps
    p = h.prof_end()
    ms = p["ms"] / reps
    tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
    print(f"gemm {M}x{N}x{K} ta={int(ta)} tb={int(tb)}: {ms*1e3:8.1f} us  {tf:6.2f} TFLOP/s  (wall {wall*1e6:.1f} us)")


def bench_perm(h, dims, shuffle, reps=20):
    a = h.array(np.random.default_rng(0).standard_normal(dims))
    out_dims = [0] * len(dims)
    for i, s in enumerate(shuffle):
        out_dims[s] = dims[i]
    o = h.empty(out_dims)
    for _ in range(3):
        h.permute(o, a, dims, shuffle)
    h.prof_begin(capi.KFAM_PERMUTE)
    for _ in range(reps):
        h.permute(o, a, dims, shuffle)
    p = h.prof_end()
    ms = p["ms"] / reps
    gbs = 2 * 8 * a.size / (ms * 1e-3) / 1e9
    print(f"permute {dims} {shuffle}: {ms*1e3:8.1f} us  {gbs:7.1f} GB/s")


if __name__ == "__main__":
    h = capi.Handle(0)
    for shp in [(1024, 1024, 1024, False, False), (4096, 4096, 4096, False, False), (256, 5120, 256, True, False),
                (256, 256, 5120, True, False), (5120, 256, 256, False, False), (256, 256, 5120, False, True),
                (64, 64, 4096, False, False), (512, 512, 10240, True, False)]:
        bench_gemm(h, *shp)
    for dims, sh in [((64, 64, 64), (0, 2, 1)), ((256, 20, 256), (2, 1, 0)), ((1024, 1024), (1, 0)),
                     ((4096, 4096), (1, 0)), ((256, 5120), (1, 0)), ((256, 20, 256), (1, 0, 2)),
                     ((20,) * 6, (5, 4, 3, 2, 1, 0)), ((8192, 8192), (1, 0))]:
        bench_perm(h, dims, sh)
