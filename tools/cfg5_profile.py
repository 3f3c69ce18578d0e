"""cfg5 per-rank compute probe (diagnostics): BASELINE configs[4] (order 16, n = 20, rank 512, round(512)) as
rank 0 of a SHARDS-way mode-slice sharding, on one GPU with the null reduction hook.

With SHARDS = 1 this is the world-1 round. With SHARDS > 1 it runs exactly rank 0's kernels of a SHARDS-rank
round (its 20 / SHARDS mode slices) minus the all-reduces: the Grams are rank 0's partial sums, so the numbers
differ from the real round but every launch has the real round's shape -- the per-rank compute time of the
strong-scaling curve, whose non-shrinking part is the replicated r x r work. Run under
rocprofv3 --kernel-trace --stats to split it by kernel."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402
from xerus_amd import dist as xd  # noqa: E402

shards = int(os.environ.get("SHARDS", "1"))
reps = int(os.environ.get("REPS", "5"))
h = capi.Handle(0)
d, n, r = 16, 20, 512
ranks = bench.tt_ranks(d, n, r)
cores = bench.random_cores(xe, [n] * d, ranks, bench.SEED + 5)
st = xd.ShardedTT.from_full_cores(h, cores, shards, 0)
del cores
comm = xd.TorchAllReduce()   # no process group: the null hook
st.round(r, comm)            # canonicalises
for i in range(reps):
    h.synchronize()
    t0 = time.perf_counter()
    cert = st.round(r, comm)
    h.synchronize()
    print(f"cfg5 round({r}) rank 0 of {shards} shard(s): {(time.perf_counter() - t0) * 1e3:.3f} ms cert={cert}", flush=True)
st.local.free()
