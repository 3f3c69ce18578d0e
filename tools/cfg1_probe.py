"""cfg1 probe (diagnostics): A(i,j) = B(i,k,l) * C(k,j,l) at 64^3 through the C++ host API, timed over 200
evaluations, plus a check against numpy; run under rocprofv3 --kernel-trace --stats for the kernel split."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import xerus_amd.xerus as xe  # noqa: E402

rng = np.random.default_rng(2)
Bn, Cn = rng.standard_normal((64, 64, 64)), rng.standard_normal((64, 64, 64))
B, C = xe.Tensor.from_ndarray(Bn), xe.Tensor.from_ndarray(Cn)
i, j, k, l = xe.indices(4)
A = xe.Tensor()
A(i, j) << B(i, k, l) * C(k, j, l)
ref = np.einsum("ikl,kjl->ij", Bn, Cn)
got = A.to_ndarray()
print("rel err", np.linalg.norm(got - ref) / np.linalg.norm(ref), flush=True)
for reps in (200, 200):
    xe.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        A(i, j) << B(i, k, l) * C(k, j, l)
    xe.synchronize()
    print(f"{(time.perf_counter() - t0) / reps * 1e6:.1f} us per evaluation", flush=True)
