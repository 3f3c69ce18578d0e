"""The Householder tridiagonalisation (xrs_sym_tridiag: k_sytrd / k_sytrd_l512, csrc/syev.hip)
against LAPACK (numpy / scipy): T = Q^T A Q has A's eigenvalues. Bar: eigenvalues of T equal eigvalsh(A) to
1e-13 ||A|| (backward stable: u ||A|| times a small multiple). Orders around the band and panel edges."""
import numpy as np
import pytest
from scipy.linalg import eigvalsh_tridiagonal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3, 16, 17, 18, 31, 32, 33, 47, 64, 100, 127, 128, 129, 200, 255, 256])
def test_tridiag_eigenvalues(handle, n):
    rng = np.random.default_rng(n)
    B = rng.standard_normal((n, 3 * n))
    A = B @ B.T / n + np.diag(rng.standard_normal(n))
    A = 0.5 * (A + A.T)
    d, e = handle.sym_tridiag(handle.array(A))
    got = np.sort(eigvalsh_tridiagonal(d, e)) if n > 1 else d
    want = np.linalg.eigvalsh(A)
    nrm = np.linalg.norm(A, 2)
    assert np.abs(got - want).max() <= 1e-13 * nrm, (np.abs(got - want).max() / nrm)


def test_tridiag_lower_triangle_only(handle):
    n = 90
    rng = np.random.default_rng(5)
    A = rng.standard_normal((n, n))
    A = A + A.T
    Al = np.tril(A) + np.triu(np.full_like(A, 3.0), 1)
    d, e = handle.sym_tridiag(handle.array(Al))
    assert np.abs(np.sort(eigvalsh_tridiagonal(d, e)) - np.linalg.eigvalsh(A)).max() <= 1e-13 * np.linalg.norm(A, 2)


def test_tridiag_structured(handle):
    """Diagonal, already tridiagonal and exactly repeated-eigenvalue matrices (zero columns: tau = 0)."""
    for A in (np.diag(np.arange(1.0, 81.0)), np.diag(np.ones(70)) + np.diag(np.ones(69), 1) + np.diag(np.ones(69), -1),
              np.eye(64) * 2.0):
        d, e = handle.sym_tridiag(handle.array(A))
        assert np.abs(np.sort(eigvalsh_tridiagonal(d, e)) - np.linalg.eigvalsh(A)).max() <= 1e-13 * np.linalg.norm(A, 2)
