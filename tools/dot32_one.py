"""Runs the fp32 TT zipper (xrs_tt_dot_f32) REPS times at the bench's headline TT shape: the target of rocprofv3
kernel traces. python tools/dot32_one.py [REPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
d, n, r = 10, 20, 256
dims = [n] * d
ranks = bench.tt_ranks(d, n, r)
h = capi.Handle(0)
x = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, 0xBAADF00D))
y = capi.TTDevice.from_cores(h, bench.random_cores(xe, dims, ranks, 0xBAADF00D + 1))
x.move_core(0)
y.move_core(0)
for _ in range(reps):
    v = x.dot_f32(y)
h.synchronize()
print("done", v)
