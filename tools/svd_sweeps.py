"""Jacobi sweep counts and times on the truncating round's SVD inputs (diagnostics): the columns of the
Cholesky factor L of B B^T (B = r x 20r) for a flat (random) and a graded (0.8^j) spectrum, p = q = r."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
rng = np.random.default_rng(0)
for r in [64, 128, 256]:
    B = rng.standard_normal((r, 20 * r))
    for kind, Bk in (("flat", B), ("graded", (0.8 ** np.arange(r))[:, None] * B)):
        L = np.linalg.cholesky(Bk @ Bk.T)
        A = h.array(L.T.copy())   # rows of L^T = columns of L, as the round's wide edges
        for kernel in (1, 2):
            ts = []
            for _ in range(3):
                h.synchronize()
                t0 = time.perf_counter()
                S, Vt, sw = h.svd_rows_vt(A, kernel)
                ts.append((time.perf_counter() - t0) * 1e3)
                S.free(), Vt.free()
            print(f"{kind} r={r} kernel={kernel}: {min(ts):.3f} ms sweeps={sw} ({min(ts) / max(sw, 1) * 1e3:.1f} us/sweep)", flush=True)
