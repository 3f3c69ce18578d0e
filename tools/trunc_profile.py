"""Truncating-round timing probe (diagnostics): cfg3 round(64) and (x+y).round(128) a few times.

Run under rocprofv3 --kernel-trace --stats on the GPU box to see where a truncating round goes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import xerus_amd.xerus as xe  # noqa: E402
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
d, n, r = 10, 20, int(os.environ.get("RANK", "128"))
target = int(os.environ.get("TARGET", "64"))
reps = int(os.environ.get("REPS", "5"))
ranks = bench.tt_ranks(d, n, r)
graded = os.environ.get("GRADED")   # "0.8": decaying spectra (right rank index scaled by GRADED^j), raw cores
eps = float(os.environ.get("EPS", str(8 * np.finfo(float).eps)))
cores = bench.random_cores(xe, [n] * d, ranks, bench.SEED + 11)
if graded:
    for k in range(d - 1):
        cores[k] = cores[k] * (float(graded) ** np.arange(cores[k].shape[2]))[None, None, :]
if os.environ.get("SUM"):   # (x + y) with y a second random TT of the same ranks: block-diagonal cores, rank 2r
    c2 = bench.random_cores(xe, [n] * d, ranks, bench.SEED + 12)
    sc = []
    for k in range(d):
        X, Y = cores[k], c2[k]
        if k == 0:
            sc.append(np.concatenate([X, Y], axis=2))
        elif k == d - 1:
            sc.append(np.concatenate([X, Y], axis=0))
        else:
            Z = np.zeros((X.shape[0] + Y.shape[0], n, X.shape[2] + Y.shape[2]))
            Z[:X.shape[0], :, :X.shape[2]] = X
            Z[X.shape[0]:, :, X.shape[2]:] = Y
            sc.append(Z)
    cores = sc
x = capi.TTDevice.from_cores(h, cores)
if not graded and not os.environ.get("SUM"):
    x.move_core(0)
for i in range(reps):
    c = x.clone()
    h.synchronize()
    t0 = time.perf_counter()
    c.round(target if target > 0 else [2 ** 62] * (d - 1), eps)
    h.synchronize()
    print(f"round({target}) of rank {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms path={h.last_round_path()} ranks={c.ranks}",
          flush=True)
    c.free()
