"""Runs one fp32 GEMM shape (xrs_gemm_f32) REPS times: the target of rocprofv3 PMC / trace passes
(tools/sgemm_pmc.sh). python tools/sgemm_one.py M N K TA TB [REPS]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

M, N, K, ta, tb = (int(a) for a in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 100
h = capi.Handle(0)
rng = np.random.default_rng(0)
A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
dA, dB, dC = h.array_f32(A), h.array_f32(B), capi.Float32Array(h, (M, N))
for _ in range(reps):
    h.gemm_f32(dC, M, N, 1.0, dA, A.shape[1], bool(ta), K, dB, B.shape[1], bool(tb))
h.synchronize()
print("done", M, N, K, ta, tb, reps, os.environ.get("XRS_SGEMM", "auto"))
