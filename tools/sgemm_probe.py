"""fp32-MFMA GEMM (xrs_gemm_f32) timing per tile configuration (XRS_SGEMM="cfg,splits", read per call) on the
shapes that matter: BASELINE configs[1] (1024^3) and the fp32 TT zipper's products. Dispatch begin / end
events (hipExtLaunchKernelGGL), mean over 30 launches, interleaved rounds (cdna_hip_programming.md rule 24).

    python tools/sgemm_probe.py [rounds]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

PEAK = 157.3
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
h = capi.Handle(0)
rng = np.random.default_rng(0)

cases = [
    ("1024^3 NN", 1024, 1024, 1024, False, False, ["", "1,2", "6,2", "13,1", "13,2", "6,1"]),
    ("256x5120x256 TN (E^T X)", 256, 5120, 256, True, False, ["", "11,1"]),
    ("5120x256x256 NN (X F)", 5120, 256, 256, False, False, ["", "12,1"]),
    ("256x256x5120 TN (T^T Y)", 256, 256, 5120, True, False, ["", "10,16"]),
    ("256x256x5120 NT (T Y^T)", 256, 256, 5120, False, True, ["", "10,16"]),
]
for name, M, N, K, ta, tb, cfgs in cases:
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    dA, dB = h.array_f32(A), h.array_f32(B)
    dC = capi.Float32Array(h, (M, N))
    res = {c: [] for c in cfgs}
    for _ in range(rounds):
        for c in cfgs:
            if c:
                os.environ["XRS_SGEMM"] = c
            else:
                os.environ.pop("XRS_SGEMM", None)
            fn = lambda: h.gemm_f32(dC, M, N, 1.0, dA, A.shape[1], ta, K, dB, B.shape[1], tb)  # noqa: E731
            fn()
            h.synchronize()
            h.prof_begin(capi.KFAM_GEMM)
            for _ in range(30):
                fn()
            p = h.prof_end()
            res[c].append(p["ms"] / max(1, p["launches"]) * 1e3)
    os.environ.pop("XRS_SGEMM", None)
    expect = A.astype(np.float64).T if ta else A.astype(np.float64)
    expect = expect @ (B.astype(np.float64).T if tb else B.astype(np.float64))
    err = np.linalg.norm(dC.numpy() - expect) / np.linalg.norm(expect)
    print(f"{name}: rel err {err:.2e}", flush=True)
    for c in cfgs:
        us = min(res[c])
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        print(f"   cfg {c or 'auto':>5}: {us:8.2f} us (median {np.median(res[c]):8.2f})  {tf:7.2f} TF/s  frac {tf / PEAK:.3f}", flush=True)
    for d in (dA, dB, dC):
        d.free()
