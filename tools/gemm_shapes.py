"""GEMM microbenchmark on the TT-round / <x,y> shapes (kernel time from HIP events, per launch family)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402


def bench(h, M, N, K, ta, tb, reps=30):
    rng = np.random.default_rng(0)
    A = h.array(rng.standard_normal((K, M) if ta else (M, K)))
    B = h.array(rng.standard_normal((N, K) if tb else (K, N)))
    C = h.empty((M, N))
    for _ in range(3):
        h.gemm(C, M, N, 1.0, A, A.shape[1], ta, K, B, B.shape[1], tb)
    h.synchronize()
    h.prof_begin(capi.KFAM_GEMM | capi.KFAM_ELEMWISE)
    for _ in range(reps):
        h.gemm(C, M, N, 1.0, A, A.shape[1], ta, K, B, B.shape[1], tb)
    h.synchronize()
    p = h.prof_end()
    us = p["ms"] / reps * 1e3
    tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
    ref = (A.numpy().T if ta else A.numpy()) @ (B.numpy().T if tb else B.numpy())
    err = np.abs(C.numpy() - ref).max() / np.abs(ref).max()
    print(f"{M:5d}x{N:5d}x{K:5d} ta={int(ta)} tb={int(tb)}: {us:8.1f} us {tf:6.2f} TF/s  err {err:.1e}", flush=True)


if __name__ == "__main__":
    h = capi.Handle(0)
    for shp in [(256, 5120, 256, False, False), (256, 256, 5120, True, False), (256, 256, 5120, False, True),
                (5120, 256, 256, False, False), (256, 5120, 256, True, False), (20, 5120, 256, False, False),
                (1024, 1024, 1024, False, False), (4096, 4096, 4096, False, False), (512, 10240, 512, False, False),
                (512, 512, 10240, True, False)]:
        bench(h, *shp)
