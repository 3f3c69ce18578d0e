"""Square dense SVD through the bidiagonal path (syev.hip svd_bidiag) on a set of spectra: accuracy against
numpy and wall time per call. Run it twice to compare paths: XRS_SVD_BIDIAG=2 (strict: a failed a-posteriori
check raises) / 1 (default, Jacobi fallback) / 0 (Jacobi only).

    XRS_SVD_BIDIAG=2 python tools/svd_bidiag_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402


def cases(rng):
    for n in (16, 33, 64, 100, 128):
        yield f"gauss{n}", rng.standard_normal((n, n))
    n = 128
    U, _ = np.linalg.qr(rng.standard_normal((n, n)))
    V, _ = np.linalg.qr(rng.standard_normal((n, n)))
    yield "graded1e-12", (U * np.logspace(0, -12, n)) @ V.T
    yield "flat", (U * (1.0 + 1e-6 * rng.standard_normal(n))) @ V.T
    yield "twin", (U * np.repeat(np.linspace(1, 2, n // 2), 2)) @ V.T
    yield "rank100", rng.standard_normal((n, 100)) @ rng.standard_normal((100, n))
    yield "scaled1e150", rng.standard_normal((n, n)) * 1e150
    yield "scaled1e-200", rng.standard_normal((n, n)) * 1e-200
    for m in (256, 512):
        yield f"gauss{m}", rng.standard_normal((m, m))
        U, _ = np.linalg.qr(rng.standard_normal((m, m)))
        V, _ = np.linalg.qr(rng.standard_normal((m, m)))
        yield f"graded{m}", (U * np.logspace(0, -12, m)) @ V.T
    for m, k in ((128, 2560), (2560, 128), (64, 1000), (300, 100), (48, 500), (32, 500)):
        yield f"g{m}x{k}", rng.standard_normal((m, k))


def main():
    h = capi.Handle(0)
    rng = np.random.default_rng(5)
    mode = os.environ.get("XRS_SVD_BIDIAG", "1")
    only = sys.argv[1:]
    for name, A in cases(rng):
        if only and name not in only:
            continue
        dA = h.array(A)
        try:
            U, S, Vt = h.svd(dA)
        except Exception as e:  # strict mode: the check's numbers are in the message
            print(f"mode {mode} {name:12s} FAILED {e}", flush=True)
            continue
        Uh, Sh, Vh = U.numpy(), S.numpy(), Vt.numpy()
        Sr = np.linalg.svd(A, compute_uv=False)
        k = Sh.size
        sc = 1.0 / np.abs(A).max()
        res = np.linalg.norm(((Uh * Sh) @ Vh - A) * sc) / np.linalg.norm(A * sc)
        ou = np.abs(Uh.T @ Uh - np.eye(k)).max()   # (k = min(m, n))
        ov = np.abs(Vh @ Vh.T - np.eye(k)).max()
        se = np.abs(Sh - Sr).max() / Sr[0]
        h.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            h.svd(dA)
        h.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        print(f"mode {mode} {name:12s} res {res:.2e} orthU {ou:.2e} orthV {ov:.2e} sigma {se:.2e} mono {bool(np.all(np.diff(Sh) <= 0))} "
              f"{ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
