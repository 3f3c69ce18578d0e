"""Diagnose the certified chain round on the cfg5 shape: python tools/debug_cfg5.py ORDER RANK
(set XRS_DEBUG_ROUND=1 for the per-edge certificate / orthogonality report on stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402
from xerus_amd import dist as xd  # noqa: E402

d, n, r = int(sys.argv[1]), 20, int(sys.argv[2])
ranks = bench.tt_ranks(d, n, r)
h = capi.Handle(0)
cores = bench.random_cores(xe, [n] * d, ranks, 5)
t = capi.TTDevice.from_cores(h, cores)
t0 = time.perf_counter()
t.move_core(0)
h.synchronize()
print("move_core(0) %.3f s, ranks kept %s" % (time.perf_counter() - t0, t.ranks == ranks[1:-1]), flush=True)
st = xd.ShardedTT(h, t, [n] * d, 1, 0)
comm = xd.TorchAllReduce()
for i in range(3):
    t0 = time.perf_counter()
    c = st.round(r, comm)
    h.synchronize()
    print("sharded round (1 rank): certified %s, %.2f ms" % (c, (time.perf_counter() - t0) * 1e3), flush=True)
t0 = time.perf_counter()
t.round(r)
h.synchronize()
print("TTDevice.round: %.2f ms, ranks kept %s" % ((time.perf_counter() - t0) * 1e3, t.ranks == ranks[1:-1]), flush=True)
