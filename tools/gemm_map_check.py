"""Correctness sweep of the LDS-DMA GEMM's split-K / batched shapes against numpy (diagnostics)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
rng = np.random.default_rng(1)
worst = 0.0
for (cnt, M, N, K, ta, tb) in [(1, 256, 256, 5120, 1, 0), (1, 512, 512, 5120, 1, 0), (2, 256, 256, 5120, 1, 0),
                               (3, 512, 512, 5120, 1, 0), (5, 512, 512, 2560, 0, 1), (4, 256, 256, 1280, 1, 0),
                               (13, 512, 512, 5120, 0, 1), (3, 256, 5120, 256, 0, 0), (6, 512, 512, 10240, 0, 1)]:
    As = [rng.standard_normal((K, M) if ta else (M, K)) for _ in range(cnt)]
    Bs = [rng.standard_normal((N, K) if tb else (K, N)) for _ in range(cnt)]
    dA = [h.array(a) for a in As]
    dB = [h.array(b) for b in Bs]
    dC = [h.empty((M, N)) for _ in range(cnt)]
    if cnt == 1:
        h.gemm(dC[0], M, N, 1.0, dA[0], As[0].shape[1], bool(ta), K, dB[0], Bs[0].shape[1], bool(tb))
    else:
        h.gemm_batched(dC, M, N, 1.0, dA, As[0].shape[1], bool(ta), K, dB, Bs[0].shape[1], bool(tb))
    errs = []
    for a, b, c in zip(As, Bs, dC):
        E = (a.T if ta else a) @ (b.T if tb else b)
        errs.append(float(np.abs(c.numpy() - E).max() / np.abs(E).max()))
    worst = max(worst, max(errs))
    print(f"count {cnt} {M}x{N}x{K} ta{ta} tb{tb}: max rel err {max(errs):.2e}", flush=True)
    if M == N and cnt == 1:
        dS = h.empty((M, N))
        h.gemm_sym(dS, M, 1.0, dA[0], As[0].shape[1], bool(ta), K, dA[0], As[0].shape[1], not bool(ta))
        a = As[0]
        E = (a.T @ a) if ta else (a @ a.T)
        print(f"   sym Gram: max rel err {np.abs(dS.numpy() - E).max() / np.abs(E).max():.2e}", flush=True)
print("worst", worst)
