"""The certified truncating round's eigensolver (xrs_sym_eig_top, csrc/syev.hip) vs LAPACK dsyevd (numpy):
the kk largest eigenpairs of symmetric matrices up to 256, with flat, graded and clustered-free spectra.
Bars: eigenvalues to 1e-13 ||A||, eigenvectors orthonormal to 1e-12 and residual ||A u - lam u|| to 1e-12 ||A||
(the round additionally checks the orthonormality of every new core and falls back on failure)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _spd(n, spectrum, seed):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    return (Q * spectrum) @ Q.T


@pytest.mark.parametrize("n,kk,kind", [(2, 1, "flat"), (5, 5, "flat"), (33, 7, "flat"), (64, 64, "flat"), (64, 32, "graded"),
                                       (100, 50, "flat"), (128, 64, "flat"), (128, 48, "graded"), (128, 20, "wishart"),
                                       (129, 60, "flat"), (200, 100, "wishart"), (256, 128, "wishart"), (256, 256, "flat")])
def test_sym_eig_top(handle, n, kk, kind):
    rng = np.random.default_rng(n * 7 + kk)
    if kind == "flat":
        A = _spd(n, 1.0 + rng.random(n) * 3.0, n)
    elif kind == "graded":   # gaps >= 7e-4 ||A|| among the kept ones (inverse iteration: orthogonality ~ u ||A|| / gap)
        A = _spd(n, 0.9 ** np.arange(n), n + 1)
    else:   # the round's P = B B^T of a random wide edge
        B = rng.standard_normal((n, 20 * n))
        A = B @ B.T
    A = 0.5 * (A + A.T)
    lam, Ut, st = handle.sym_eig_top(handle.array(A), kk)
    assert st == 0
    lam, U = lam.numpy(), Ut.numpy().T
    want = np.linalg.eigvalsh(A)[::-1][:kk]
    nrm = np.linalg.norm(A, 2)
    assert np.abs(lam - want).max() <= 1e-13 * nrm
    assert np.abs(U.T @ U - np.eye(kk)).max() <= 1e-12
    assert np.linalg.norm(A @ U - U * lam, axis=0).max() <= 1e-12 * nrm


def test_sym_eig_top_lower_triangle_only(handle):
    """Only the lower triangle is read (the round's Grams are mirrored anyway)."""
    A = _spd(40, np.linspace(1, 5, 40), 3)
    Al = np.tril(A) + np.triu(np.full_like(A, 7.0), 1)
    lam, Ut, st = handle.sym_eig_top(handle.array(Al), 10)
    assert st == 0
    assert np.abs(lam.numpy() - np.linalg.eigvalsh(A)[::-1][:10]).max() <= 1e-13 * 5


@pytest.mark.parametrize("n,kk", [(24, 12), (96, 40), (200, 120)])
def test_sym_eig_top_clusters(handle, n, kk):
    """Exactly repeated and 1e-9-close eigenvalues inside the kept set (inverse iteration alone gives
    non-orthogonal vectors there; k_cluster_orth orthonormalises each cluster): eigenvalues, orthonormality
    and residuals at the same bars, and the kept subspace equals LAPACK's when the cut lies in a gap."""
    rng = np.random.default_rng(n)
    spec = np.concatenate([np.repeat([9.0, 7.0, 5.0], 4), 5.0 - 1e-9 * np.arange(1, 4), 1.0 + rng.random(n - 15)])
    A = _spd(n, spec, n + 3)
    A = 0.5 * (A + A.T)
    lam, Ut, st = handle.sym_eig_top(handle.array(A), kk)
    assert st == 0
    lam, U = lam.numpy(), Ut.numpy().T
    w, Z = np.linalg.eigh(A)
    nrm = np.linalg.norm(A, 2)
    assert np.abs(lam - w[::-1][:kk]).max() <= 1e-13 * nrm
    assert np.abs(U.T @ U - np.eye(kk)).max() <= 1e-12
    assert np.linalg.norm(A @ U - U * lam, axis=0).max() <= 1e-12 * nrm
    P = Z[:, ::-1][:, :kk]
    if w[::-1][kk - 1] - w[::-1][kk] > 1e-3:   # the projector onto the kept subspace is unique
        assert np.abs(U @ U.T - P @ P.T).max() <= 1e-11
