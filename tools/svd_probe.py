"""Jacobi SVD kernel timing probe (diagnostics): one workgroup vs the multi-workgroup block kernel."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
rng = np.random.default_rng(0)
for p in [64, 128, 256, 512]:
    U0, _ = np.linalg.qr(rng.standard_normal((p, p)))
    V0, _ = np.linalg.qr(rng.standard_normal((p, p)))
    A0 = (U0 * np.logspace(0, -6, p)) @ V0.T
    for kind, M in (("graded", A0), ("cholT", np.linalg.cholesky(A0 @ A0.T).T.copy())):
      A = h.array(M)
      for kernel in (1, 2):
        ts = []
        for _ in range(4):
            h.synchronize()
            t0 = time.perf_counter()
            S, Vt, sw = h.svd_rows_vt(A, kernel)
            ts.append((time.perf_counter() - t0) * 1e3)
            S.free(), Vt.free()
        print(f"{kind} p=q={p} kernel={kernel}: {min(ts):.3f} ms sweeps={sw}", flush=True)
