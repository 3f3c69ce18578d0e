"""<x,y> at the bench's headline TT shape (order 10, n 20, rank 256): fp64 zipper (xrs_tt_dot) vs the fp32-MFMA
zipper (xrs_tt_dot_f32), host-timed per call, and the fp32 error against the fp64 value."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402

d, n, r = 10, 20, int(os.environ.get("RANK", "256"))
dims = [n] * d
ranks = bench.tt_ranks(d, n, r)
h = capi.Handle(0)
x = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, 0xBAADF00D))
y = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, 0xBAADF00D + 1))
x.move_core(0)
y.move_core(0)
f = bench.flops_dot(dims, ranks, ranks)
for name, fn in [("f64", x.dot), ("f32", x.dot_f32)]:
    for _ in range(3):
        fn(y)
    h.synchronize()
    K = 50
    t = time.perf_counter()
    for _ in range(K):
        v = fn(y)
    t = (time.perf_counter() - t) / K
    print(f"{name}: {t * 1e3:.4f} ms  {f / t / 1e12:.2f} TF/s  value {v!r}", flush=True)
d64, d32 = x.dot(y), x.dot_f32(y)
print("rel err (||x|| ||y||):", abs(d32 - d64) / (x.frob_norm() * y.frob_norm()))
