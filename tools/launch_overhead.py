"""Host enqueue cost vs GPU time of back-to-back launches (is the TT step host-bound?).

python tools/launch_overhead.py  -> prints per-call host enqueue time and per-call wall time for
dependent GEMM chains of a few sizes (ctypes call included, as in the product path)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
rng = np.random.default_rng(0)
for (m, k, n) in [(32, 32, 32), (256, 256, 256), (5120, 256, 256), (256, 5120, 256)]:
    A = h.array(rng.standard_normal((m, k)))
    B = h.array(rng.standard_normal((k, n)))
    Cm = h.empty((m, n))
    for _ in range(20):
        h.gemm(Cm, m, n, 1.0, A, k, False, k, B, n, False)
    h.synchronize()
    reps = 400
    t0 = time.perf_counter()
    for _ in range(reps):
        h.gemm(Cm, m, n, 1.0, A, k, False, k, B, n, False)
    t1 = time.perf_counter()
    h.synchronize()
    t2 = time.perf_counter()
    print("gemm %5dx%5dx%5d: host enqueue %.2f us/call, wall %.2f us/call" %
          (m, k, n, (t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6), flush=True)
