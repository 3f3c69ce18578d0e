"""Per-rank time of the sharded cfg5 round (BASELINE configs[4]: order 16, rank 512, round(512)) on ONE GPU, with
the local slices certifying.

For N ranks a rank holds m = ceil(20 / N) slices of every mode. The probe rounds the TT whose every mode is one
random m-slice block repeated N times: rank 0's share is exactly that block, and the sum over ranks of every
Gram is N x rank 0's partial sum -- what xrs_comm_emulate's all-reduce enqueues (buf *= N). So the round is a
real, certified sharded round whose kernels are those of one rank of an N-way sharding (interior shapes
512 x m x 512, as cfg5's); only the end ranks differ (min(m^k, 512) instead of min(20^k, 512)) and the
collectives cost nothing (their volume is printed). N = 1 is cfg5 itself.

    python tools/cfg5_rank_probe.py [N ...]       (default 1 2 4 8; N = 0: the unsharded round)

MODE=trunc (r06): the truncating round(256) of the same TT (rank 512 -> 256, the certified truncation);
MODE=general: the cores graded (column j of every core scaled by 0.97^j) so that the certified truncation refuses
and round(256) takes the sharded general round (§3.2b). Each call rounds a fresh copy of the slices.
"""
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402
from xerus_amd import dist as xd  # noqa: E402

D, NG, R = 16, 20, 512
reps = int(os.environ.get("REPS", "6"))
MODE = os.environ.get("MODE", "chain")   # chain: round(512); trunc / general: round(256)
h = capi.Handle(0)
for world in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    if world == 0:   # the unsharded single-GPU round of cfg5 (xrs_tt_round), for comparison
        ranks = bench.tt_ranks(D, NG, R)
        x = capi.TTDevice.from_cores(h, bench.random_cores(xe, [NG] * D, ranks, bench.SEED + 5))
        x.round(R)
        ts = []
        for i in range(reps):
            h.synchronize()
            t0 = time.perf_counter()
            x.round(R)
            h.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"unsharded cfg5 round(512): {1e3 * min(ts):.3f} ms (median {1e3 * sorted(ts)[len(ts) // 2]:.3f}), "
              f"path {h.last_round_path()}", flush=True)
        x.free()
        continue
    m = NG if world == 1 else math.ceil(NG / world)
    ranks = bench.tt_ranks(D, m, R)
    cores = bench.random_cores(xe, [m] * D, ranks, bench.SEED + 5)
    if world > 1:
        # orthonormal factors left and right of the middle core (a different, well-conditioned tensor): the
        # m-slice TT's maximal-rank end edges are square products of random cores (e.g. 125 x 125 at m = 5),
        # too ill-conditioned for the certificates; cfg5's n = 20 end edges (20 x 20, 400 x 400) certify
        for k in range(D // 2):
            a, _, b = cores[k].shape
            cores[k] = np.linalg.qr(cores[k].reshape(a * m, b))[0].reshape(a, m, b)
        for k in range(D // 2 + 1, D):
            a, _, b = cores[k].shape
            cores[k] = np.linalg.qr(cores[k].reshape(a, m * b).T)[0].T.reshape(a, m, b)
    if MODE == "general":
        for k in range(D - 1):
            cores[k] = cores[k] * (0.97 ** np.arange(cores[k].shape[2]))[None, None, :]
    local = capi.TTDevice.from_cores(h, cores)
    comm = xd.EmulatedComm(h, world)
    ts, paths = [], set()
    st = xd.ShardedTT(h, local, [m * world] * D, world, 0)
    first = st.round_sharded(R, comm)   # canonicalises (as bench.py's cfg5: the timed rounds start right-canonical)
    target = R if MODE == "chain" else R // 2
    for i in range(reps):
        c = st if MODE == "chain" else xd.ShardedTT(h, st.local.clone(), st.dims, world, 0)
        c0 = comm.calls
        h.synchronize()
        t0 = time.perf_counter()
        paths.add(c.round_sharded(target, comm) or "uncertified")
        h.synchronize()
        ts.append(time.perf_counter() - t0)
        calls = comm.calls - c0
        if c is not st:
            c.local.free()
    r2 = sum(r * r for r in ranks[1:-1])
    print(f"N={world} [{MODE}]: m={m} local slices, ranks {ranks[1:-1]}, round({target}) {1e3 * min(ts):.3f} ms (median "
          f"{1e3 * sorted(ts)[len(ts) // 2]:.3f}), path {sorted(paths)} (first call {first}), all-reduces per round {calls} "
          f"(sum over ranks of r x r Grams: {8 * r2 / 1e6:.1f} MB per chain pass)", flush=True)
    comm.close()
    st.local.free()
