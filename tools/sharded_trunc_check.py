"""Sharded truncating round at the cfg5 per-rank shape (order 16, 10 local slices, rank 512 -> 256) with the
emulated 2-rank communicator (diagnostics): path taken and the rounded local cores' orthonormality."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402
from xerus_amd import dist as xd  # noqa: E402

D, M, R, W = 16, 10, 512, 2
h = capi.Handle(0)
ranks = bench.tt_ranks(D, M, R)
cores = bench.random_cores(xe, [M] * D, ranks, bench.SEED + 5)
for k in range(D // 2):
    a, _, b = cores[k].shape
    cores[k] = np.linalg.qr(cores[k].reshape(a * M, b))[0].reshape(a, M, b)
for k in range(D // 2 + 1, D):
    a, _, b = cores[k].shape
    cores[k] = np.linalg.qr(cores[k].reshape(a, M * b).T)[0].T.reshape(a, M, b)
comm = xd.EmulatedComm(h, W)
for target in (256, 256):
    st = xd.ShardedTT(h, capi.TTDevice.from_cores(h, cores), [M * W] * D, W, 0)
    path = st.round_sharded(target, comm)
    cs = st.local.cores()
    dev = max(float(np.abs(W * c.reshape(c.shape[0], -1) @ c.reshape(c.shape[0], -1).T - np.eye(c.shape[0])).max()) for c in cs[1:])
    print(f"round({target}): path {path!r}, ranks {st.ranks}, max |sum_ranks C C^T - I| = {dev:.2e}", flush=True)
    st.local.free()
comm.close()
