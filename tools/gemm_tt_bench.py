"""Time the TT-shaped GEMMs of the bench step (back-to-back launches, wall / reps).

python tools/gemm_tt_bench.py [torch]   (XRS_GEMM_CFG selects a tile variant; "torch" also times
torch.matmul in fp64, i.e. the ROCm BLAS library, on the same shapes as a reference bar)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

SHAPES = [  # (M, N, K, ta, tb, what)
    (256, 5120, 256, 0, 0, "E X / G M / transform (NN wide)"),
    (256, 5120, 256, 1, 0, "dot E^T X (TN wide)"),
    (256, 256, 5120, 1, 0, "Gram M^T T (TN, K = n r)"),
    (256, 256, 5120, 0, 1, "Gram M T^T (NT, K = n r)"),
    (5120, 256, 256, 0, 0, "right chain M H (NN tall)"),
    (512, 10240, 512, 0, 0, "cfg5 NN wide"),
    (512, 512, 10240, 0, 1, "cfg5 Gram NT"),
]
TORCH = len(sys.argv) > 1 and sys.argv[1] == "torch"   # separate process: one HIP runtime per process
h = None if TORCH else capi.Handle(0)
rng = np.random.default_rng(0)
cfg = os.environ.get("XRS_GEMM_CFG", "default")
ONLY = os.environ.get("XRS_BENCH_ONLY")   # substring filter on the shape description
for M, N, K, ta, tb, what in ([] if TORCH else SHAPES):
    if ONLY and ONLY not in what:
        continue
    A = h.array(rng.standard_normal((K, M) if ta else (M, K)))
    B = h.array(rng.standard_normal((N, K) if tb else (K, N)))
    C = h.empty((M, N))
    call = lambda: h.gemm(C, M, N, 1.0, A, A.shape[1], bool(ta), K, B, B.shape[1], bool(tb))  # noqa: E731
    for _ in range(10):
        call()
    h.synchronize()
    reps = 100
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    h.synchronize()
    us = (time.perf_counter() - t0) / reps * 1e6
    print("cfg %-10s %-34s %5dx%5dx%5d ta%d tb%d: %7.1f us %6.1f TF/s" %
          (cfg, what, M, N, K, ta, tb, us, 2.0 * M * N * K / us / 1e6), flush=True)
    A.free(); B.free(); C.free()

if TORCH:
    import torch
    for M, N, K, ta, tb, what in SHAPES:
        a = torch.randn((K, M) if ta else (M, K), dtype=torch.float64, device="cuda")
        b = torch.randn((N, K) if tb else (K, N), dtype=torch.float64, device="cuda")
        op = lambda: (a.t() if ta else a) @ (b.t() if tb else b)  # noqa: E731
        for _ in range(10):
            op()
        torch.cuda.synchronize()
        reps = 100
        t0 = time.perf_counter()
        for _ in range(reps):
            op()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / reps * 1e6
        print("torch      %-34s %5dx%5dx%5d ta%d tb%d: %7.1f us %6.1f TF/s" %
              (what, M, N, K, ta, tb, us, 2.0 * M * N * K / us / 1e6), flush=True)
