"""How much does concurrency buy on the TT chain GEMM shape (256 x 5120 x 256, and the K = 5120 Gram)?
One launch per GEMM on one stream, a batched launch of c GEMMs, and c handles (streams) launching
alternately. Back-to-back launches, wall / reps."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

rng = np.random.default_rng(0)
hs = [capi.Handle(0) for _ in range(4)]
h = hs[0]
for (M, N, K, ta, tb, what) in [(256, 5120, 256, 0, 0, "NN wide"), (256, 256, 5120, 1, 0, "Gram TN")]:
    A = [hh.array(rng.standard_normal((K, M) if ta else (M, K))) for hh in hs]
    B = [hh.array(rng.standard_normal((N, K) if tb else (K, N))) for hh in hs]
    Cs = [hh.empty((M, N)) for hh in hs]
    fl = 2.0 * M * N * K
    def timeit(fn, work, reps=50):
        for _ in range(5):
            fn()
        for hh in hs:
            hh.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        for hh in hs:
            hh.synchronize()
        us = (time.perf_counter() - t0) / reps * 1e6
        return us, work * fl / us / 1e6
    us, tf = timeit(lambda: h.gemm(Cs[0], M, N, 1.0, A[0], A[0].shape[1], bool(ta), K, B[0], B[0].shape[1], bool(tb)), 1)
    print(f"{what}: single {us:.1f} us {tf:.1f} TF/s", flush=True)
    for c in (2, 3, 4):
        us, tf = timeit(lambda: h.gemm_batched(Cs[:c], M, N, 1.0, A[:c], A[0].shape[1], bool(ta), K, B[:c], B[0].shape[1], bool(tb)), c)
        print(f"{what}: batched x{c} {us:.1f} us {tf:.1f} TF/s", flush=True)
        def conc():
            for i in range(c):
                hs[i].gemm(Cs[i], M, N, 1.0, A[i], A[i].shape[1], bool(ta), K, B[i], B[i].shape[1], bool(tb))
        us, tf = timeit(conc, c)
        print(f"{what}: {c} streams {us:.1f} us {tf:.1f} TF/s", flush=True)
