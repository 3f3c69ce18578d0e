"""Host-side timing of the headline step's calls (is the step host-bound?).

python tools/host_timing.py -> median host time of x.dot_async(y) (enqueue only), x.round(r) (enqueue +
its check synchronisation), fut.result(), the synchronous x.dot(y), and the GEMM launch cost on the main
and on a side stream."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
d, n, r = 10, 20, 256
dims = [n] * d
ranks = bench.tt_ranks(d, n, r)
x = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, bench.SEED))
y = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, bench.SEED + 1))
x.move_core(0)
y.move_core(0)
T = {k: [] for k in ("dot_async", "round", "result", "sync_tail", "dot_sync", "round_after_sync")}
for it in range(25):
    t0 = time.perf_counter()
    fut = x.dot_async(y)
    t1 = time.perf_counter()
    x.round(r)
    t2 = time.perf_counter()
    fut.result()
    t3 = time.perf_counter()
    h.synchronize()
    t4 = time.perf_counter()
    x.dot(y)
    t5 = time.perf_counter()
    x.round(r)
    h.synchronize()
    t6 = time.perf_counter()
    if it >= 5:
        for k, v in zip(T, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            T[k].append(v * 1e6)
for k, v in T.items():
    print("%-18s median %8.1f us  min %8.1f us" % (k, statistics.median(v), min(v)), flush=True)
