"""cfg3's certified round(128) (order 10, n 20, rank 128) repeated, the target of a kernel trace:
    rocprofv3 --kernel-trace -d DIR -o r --output-format csv -- python3 tools/round128_one.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xerus_amd import capi  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
h = capi.Handle(0)
d, n, r = 10, 20, 128
dims = [n] * d
cores = bench.random_cores(xe, dims, bench.tt_ranks(d, n, r), bench.SEED + 11)
x = capi.TTDevice.from_cores(h, cores)
x.move_core(0)
ts = []
for _ in range(reps):
    c = x.clone()
    h.synchronize()
    t0 = time.perf_counter()
    c.round(128, 8 * np.finfo(float).eps)
    h.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
    c.free()
print("round(128) ms:", " ".join(f"{t:.3f}" for t in ts), flush=True)
