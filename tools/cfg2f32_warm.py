"""cfg2_f32 (1024^3 fp32 GEMM, bench.py's event timing) after 20 / 200 / 1000 untimed launches (diagnostics)."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import bench
from xerus_amd import capi
h = capi.Handle(0)
n = 1024
rng = np.random.default_rng(1)
A32, B32 = rng.standard_normal((n, n)).astype(np.float32), rng.standard_normal((n, n)).astype(np.float32)
A, B, C = h.array_f32(A32), h.array_f32(B32), capi.Float32Array(h, (n, n))
for warm in (20, 200, 1000, 20, 200, 1000):
    ev = bench._events(h, capi.KFAM_GEMM, lambda: h.gemm_f32(C, n, n, 1.0, A, n, False, n, B, n, False), 50, warm=warm)
    print(f"warm {warm}: {ev['us_per_launch']:.2f} us", flush=True)
