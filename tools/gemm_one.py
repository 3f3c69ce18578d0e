"""Run one GEMM shape repeatedly (PMC collection target): python tools/gemm_one.py M N K ta tb reps"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

M, N, K, ta, tb, reps = (int(v) for v in sys.argv[1:7])
h = capi.Handle(0)
rng = np.random.default_rng(0)
A = h.array(rng.standard_normal((K, M) if ta else (M, K)))
B = h.array(rng.standard_normal((N, K) if tb else (K, N)))
C = h.empty((M, N))
for _ in range(reps):
    h.gemm(C, M, N, 1.0, A, A.shape[1], bool(ta), K, B, B.shape[1], bool(tb))
h.synchronize()
