"""The square dense SVD's bidiagonal path (syev.hip svd_bidiag: Householder bidiagonalisation, the Golub-Kahan
tridiagonal's top eigenpairs, back-transformation, a first-order CholeskyQR step on the halves, a-posteriori
check) against the LAPACK-call oracle. XRS_SVD_BIDIAG=2 (strict) makes a failed check raise, so these cases prove the path itself
delivers dgesdd-level results on spectra without large clusters; spectra with them (graded over many decades,
flat, rank-deficient) take the default mode's Jacobi fallback, covered below and by
tests/test_factorisations_gpu.py.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_STRICT = r"""
import sys, json
import numpy as np
sys.path.insert(0, %r)
from xerus_amd import capi
from oracle import xerus_ref as ref
h = capi.Handle(0)
rng = np.random.default_rng(11)
out = []
def spectra():
    for n in (16, 31, 64, 96, 128):
        yield "gauss%%d" %% n, rng.standard_normal((n, n))
    n = 128
    U, _ = np.linalg.qr(rng.standard_normal((n, n)))
    V, _ = np.linalg.qr(rng.standard_normal((n, n)))
    yield "graded", (U * np.logspace(0, -1, n)) @ V.T   # (gaps above dstein's cluster tolerance 1e-3 ||T||)
    yield "tiny", rng.standard_normal((n, n)) * 1e-200
    for m, q in ((128, 1500), (1500, 128), (64, 700), (300, 100), (24, 400)):   # (the QR factor's route)
        yield "g%%dx%%d" %% (m, q), rng.standard_normal((m, q))
for name, A in spectra():
    Uh, Sh, Vh = (x.numpy() for x in h.svd(h.array(A)))
    Sr = ref.svd(A)[1]
    k = Sh.size
    assert Uh.shape == (A.shape[0], k) and Vh.shape == (k, A.shape[1])
    sc = 1.0 / np.abs(A).max()
    out.append(dict(name=name, res=float(np.linalg.norm(((Uh * Sh) @ Vh - A) * sc) / np.linalg.norm(A * sc)),
                    ou=float(np.abs(Uh.T @ Uh - np.eye(k)).max()), ov=float(np.abs(Vh @ Vh.T - np.eye(k)).max()),
                    se=float(np.abs(Sh - Sr).max() / Sr[0]), mono=bool(np.all(np.diff(Sh) <= 0))))
print(json.dumps(out))
"""


def test_svd_bidiag_strict():
    env = dict(os.environ, XRS_SVD_BIDIAG="2")
    p = subprocess.run([sys.executable, "-c", _STRICT % ROOT], env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    import json

    for r in json.loads(p.stdout.strip().splitlines()[-1]):
        assert r["res"] <= 1e-14 and r["ou"] <= 1e-14 and r["ov"] <= 1e-14, r
        assert r["se"] <= 1e-12 and r["mono"], r


@pytest.mark.parametrize("kind", ["rank_deficient", "identity", "zero", "twin", "graded12"])
def test_svd_square_fallback_cases(handle, ref, kind):
    """Spectra the bidiagonal path may hand to the Jacobi fallback: the default mode still meets dgesdd's bars."""
    n = 96
    rng = np.random.default_rng(3)
    if kind == "rank_deficient":
        A = rng.standard_normal((n, 7)) @ rng.standard_normal((7, n))
    elif kind == "identity":
        A = np.eye(n)
    elif kind == "zero":
        A = np.zeros((n, n))
    else:
        U, _ = np.linalg.qr(rng.standard_normal((n, n)))
        V, _ = np.linalg.qr(rng.standard_normal((n, n)))
        s = np.repeat(np.linspace(1, 2, n // 2), 2) if kind == "twin" else np.logspace(0, -12, n)
        A = (U * s) @ V.T
    Uh, Sh, Vh = (x.numpy() for x in handle.svd(handle.array(A)))
    Sr = ref.svd(A)[1]
    assert np.all(np.diff(Sh) <= 0)
    assert np.abs(Sh - Sr).max() <= 1e-12 * max(Sr[0], 1.0)
    assert np.linalg.norm((Uh * Sh) @ Vh - A) <= 1e-14 * np.linalg.norm(A)
    if kind == "zero":   # (Jacobi route: orthonormal rows of Vt only for S > 0, as before this path existed)
        assert not Sh.any()
        return
    assert np.abs(Uh.T @ Uh - np.eye(n)).max() <= 1e-14
    assert np.abs(Vh @ Vh.T - np.eye(n)).max() <= 1e-14
