"""GPU parity of QC/CQ/QR/RQ/SVD (through the C-ABI) against the LAPACK-call oracle.

Factors are not unique (pivot order, signs), so parity is judged on invariants, as the reference's own
tests do (fullTensor_factorisations.cxx:26-276): reconstruction, orthogonality, singular values, and
the exact rank of the reference's rank rule (blasLapackWrapper.cpp:268-272).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


SHAPES = [(8, 5), (5, 8), (6, 6), (1, 4), (4, 1), (400, 128), (5120, 256), (2560, 128), (2560, 20), (20, 256),
          (128, 2560), (256, 5120), (700, 300), (3, 3000)]


@pytest.mark.parametrize("m,n", SHAPES)
def test_qc_random(handle, ref, m, n):
    A = np.random.default_rng(m * 31 + n).standard_normal((m, n))
    Q, Cm, r = handle.qc(handle.array(A))
    Qh, Ch = Q.numpy(), Cm.numpy()
    _, _, rr = ref.qc(A)
    assert r == rr == min(m, n)
    assert _rel(Qh @ Ch, A) <= TOL
    assert np.linalg.norm(Qh.T @ Qh - np.eye(r)) <= TOL * max(1, r)


@pytest.mark.parametrize("m,n", SHAPES)
def test_cq_random(handle, ref, m, n):
    A = np.random.default_rng(m * 17 + n).standard_normal((m, n))
    Cm, Q, r = handle.cq(handle.array(A))
    Ch, Qh = Cm.numpy(), Q.numpy()
    _, _, rr = ref.cq(A)
    assert r == rr == min(m, n)
    assert _rel(Ch @ Qh, A) <= TOL
    assert np.linalg.norm(Qh @ Qh.T - np.eye(r)) <= TOL * max(1, r)


@pytest.mark.parametrize("m,n,k", [(600, 200, 50), (300, 120, 1), (40, 30, 7), (2000, 256, 128), (256, 2000, 100)])
@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_qc_cq_rank_deficient_matches_reference_rule(handle, ref, m, n, k, sign):
    rng = np.random.default_rng(m + n + k)
    A = sign * (rng.standard_normal((m, k)) @ rng.standard_normal((k, n)))
    Q, Cm, r = handle.qc(handle.array(A))
    _, _, rr = ref.qc(A)
    assert r == rr
    assert _rel(Q.numpy() @ Cm.numpy(), A) <= 1e-11
    Cc, Qc, r2 = handle.cq(handle.array(A))
    _, _, rr2 = ref.cq(A)
    assert r2 == rr2
    assert _rel(Cc.numpy() @ Qc.numpy(), A) <= 1e-11


@pytest.mark.parametrize("m,n", [(8, 5), (5, 8), (400, 128), (5120, 256), (128, 2560), (33, 700), (2000, 250),
                                 (1500, 33), (100, 3000), (1200, 300), (300, 1200), (6000, 512), (512, 4000)])
def test_qr_rq(handle, m, n):
    A = np.random.default_rng(m + 3 * n).standard_normal((m, n))
    k = min(m, n)
    Q, R = handle.qr(handle.array(A))
    Qh, Rh = Q.numpy(), R.numpy()
    assert _rel(Qh @ Rh, A) <= TOL
    assert np.linalg.norm(Qh.T @ Qh - np.eye(k)) <= TOL * k
    R2, Q2 = handle.rq(handle.array(A))
    R2h, Q2h = R2.numpy(), Q2.numpy()
    assert _rel(R2h @ Q2h, A) <= TOL
    assert np.linalg.norm(Q2h @ Q2h.T - np.eye(k)) <= TOL * k


@pytest.mark.parametrize("m,n", [(3000, 600), (2100, 1030), (1100, 1100)])
def test_qr_rq_above_512(handle, m, n):
    """Orders above 512: the blocked CholeskyQR2 (chol_full, explicit inverses) -- tall QR and wide RQ."""
    A = np.random.default_rng(m + n).standard_normal((m, n))
    Q, R = handle.qr(handle.array(A))
    Qh, Rh = Q.numpy(), R.numpy()
    assert _rel(Qh @ Rh, A) <= TOL
    assert np.abs(Qh.T @ Qh - np.eye(n)).max() <= 1e-13
    assert np.allclose(np.tril(Rh, -1), 0.0)
    R2, Q2 = handle.rq(handle.array(np.ascontiguousarray(A.T)))
    R2h, Q2h = R2.numpy(), Q2.numpy()
    assert _rel(R2h @ Q2h, A.T) <= TOL
    assert np.abs(Q2h @ Q2h.T - np.eye(n)).max() <= 1e-13


@pytest.mark.parametrize("m,n", [(8, 5), (5, 8), (64, 64), (128, 128), (30, 200), (200, 30), (1, 5), (5, 1),
                                 (256, 256), (512, 512), (300, 512), (512, 300), (100, 100), (90, 64)])
def test_svd(handle, ref, m, n):
    A = np.random.default_rng(m * 5 + n).standard_normal((m, n))
    U, S, Vt = handle.svd(handle.array(A))
    Uh, Sh, Vh = U.numpy(), S.numpy(), Vt.numpy()
    _, Sr, _ = ref.svd(A)
    k = min(m, n)
    assert np.all(np.diff(Sh) <= 0)
    assert np.max(np.abs(Sh - Sr)) <= 1e-12 * Sr[0]
    assert _rel((Uh * Sh[None, :]) @ Vh, A) <= TOL
    assert np.linalg.norm(Uh.T @ Uh - np.eye(k)) <= TOL * k
    assert np.linalg.norm(Vh @ Vh.T - np.eye(k)) <= TOL * k
    # LAPACK-level accuracy (dgesdd measured 1e-15 .. 3e-15 here): the reference's 1e-14 TT tests need it
    assert _rel((Uh * Sh[None, :]) @ Vh, A) <= 1e-14
    assert np.abs(Uh.T @ Uh - np.eye(k)).max() <= 1e-14
    assert np.abs(Vh @ Vh.T - np.eye(k)).max() <= 1e-14


def test_svd_rank_deficient(handle, ref):
    rng = np.random.default_rng(9)
    A = rng.standard_normal((40, 6)) @ rng.standard_normal((6, 50))
    U, S, Vt = handle.svd(handle.array(A))
    Sh = S.numpy()
    _, Sr, _ = ref.svd(A)
    assert ref.svd_rank(Sh, 0, ref.EPSILON) == ref.svd_rank(Sr, 0, ref.EPSILON) == 6
    assert np.max(np.abs(Sh - Sr)) <= 1e-12 * Sr[0]


@pytest.mark.parametrize("m,n,scale", [(3000, 200, 1e-6), (2000, 256, 1e6), (1000, 96, 1e-3)])
def test_qr_graded_columns(handle, m, n, scale):
    """Columns graded over `scale` (kappa ~ 1/scale or scale): CholeskyQR2 path + its certification and fallback."""
    rng = np.random.default_rng(m + n)
    A = rng.standard_normal((m, n)) * np.logspace(0, np.log10(scale), n)[None, :]
    Q, R = handle.qr(handle.array(A))
    Qh, Rh = Q.numpy(), R.numpy()
    assert _rel(Qh @ Rh, A) <= 1e-12
    assert np.linalg.norm(Qh.T @ Qh - np.eye(n)) <= TOL * n


@pytest.mark.parametrize("p,q", [(17, 40), (100, 100), (128, 128), (129, 129), (200, 256), (256, 256), (300, 400),
                                 (512, 512), (250, 500)])
@pytest.mark.parametrize("kernel", [1, 2])
def test_svd_rows_vt_kernels(handle, p, q, kernel):
    """The truncating round's Jacobi SVD (one workgroup vs the multi-workgroup block kernel) against LAPACK:
    singular values to ~u*S0, orthonormal Vt, A Vt^T Vt = A. Graded spectrum as in a TT edge."""
    rng = np.random.default_rng(p * 7 + q)
    U0, _ = np.linalg.qr(rng.standard_normal((p, p)))
    V0, _ = np.linalg.qr(rng.standard_normal((q, p)))
    s0 = np.logspace(0, -9, p)
    A = (U0 * s0) @ V0.T
    S, Vt, sweeps = handle.svd_rows_vt(handle.array(A), kernel)
    S, Vt = S.numpy(), Vt.numpy()
    assert 0 < sweeps <= 40
    assert np.all(np.diff(S) <= 0)
    assert np.max(np.abs(S - s0)) <= 1e-14 * s0[0] * np.sqrt(p)
    assert np.linalg.norm(Vt @ Vt.T - np.eye(p)) <= 1e-13 * p
    assert _rel((A @ Vt.T) @ Vt, A) <= 1e-14 * np.sqrt(p)


@pytest.mark.parametrize("kernel", [1, 2])
def test_svd_rows_vt_rank_deficient(handle, kernel):
    rng = np.random.default_rng(5)
    A = rng.standard_normal((200, 7)) @ rng.standard_normal((7, 300))
    S, Vt, sweeps = handle.svd_rows_vt(handle.array(A), kernel)
    S = S.numpy()
    ref = np.linalg.svd(A, compute_uv=False)
    assert sweeps > 0
    assert np.max(np.abs(S[:7] - ref[:7])) <= 1e-13 * ref[0]
    assert np.max(np.abs(S[7:])) <= 1e-12 * ref[0]
    Vt7 = Vt.numpy()[:7]
    assert np.linalg.norm(Vt7 @ Vt7.T - np.eye(7)) <= 1e-13


@pytest.mark.parametrize("m,n,k", [(600, 600, 300), (1024, 700, 650), (700, 1024, 600)])
def test_qc_cq_rank_deficient_above_512(handle, ref, m, n, k):
    """Rank-revealing QC / CQ of rank-deficient matrices with min(m, n) > 512: shifted CholeskyQR3 breaks
    down, the exact dgeqp3 emulation runs on the matrix itself; the rank is the reference's rule
    (blasLapackWrapper.cpp:268-272, oracle: LAPACK dgeqp3)."""
    rng = np.random.default_rng(m + n + k)
    # exactly rank k: k random columns and n - k zero columns, interleaved by a random permutation (a
    # product of random factors puts |R_kk| / R_00 of the deficient part at ~5e-15 for these sizes, i.e.
    # inside the noise band of the 16 eps threshold, where LAPACK's own rank is a rounding accident)
    A0 = np.zeros((m, n))
    A0[:, rng.permutation(n)[:k]] = rng.standard_normal((m, k))
    # The reference cuts only when its R_00 is positive (|R_kk| < 16 eps R_00, R_00 signed), i.e. for one of
    # A and -A: both signs are run, so the cut and the no-cut branch of the rule are each exercised once.
    qc_ranks, cq_ranks = set(), set()
    for sign in (1.0, -1.0):
        A = sign * A0
        Q, Cm, r = handle.qc(handle.array(A))
        assert r == ref.qc(A)[2]
        qc_ranks.add(r)
        assert _rel(Q.numpy() @ Cm.numpy(), A) <= 1e-11
        Cc, Qc, r2 = handle.cq(handle.array(A))
        assert r2 == ref.cq(A)[2]
        cq_ranks.add(r2)
        assert _rel(Cc.numpy() @ Qc.numpy(), A) <= 1e-11
        Qh = Qc.numpy()
        assert np.abs(Qh @ Qh.T - np.eye(r2)).max() <= 1e-12
    for ranks in (qc_ranks, cq_ranks):
        assert ranks == {k, min(m, n)}, ranks


@pytest.mark.parametrize("m,n", [(600, 600), (900, 700), (700, 1024), (1024, 1024), (3000, 600)])
def test_svd_above_512(handle, ref, m, n):
    """The API SVD for 512 < min(m, n) <= 1024 (QR preconditioning + block Jacobi on the triangular factor):
    singular values vs dgesdd, reconstruction and orthogonality at LAPACK level."""
    A = np.random.default_rng(m * 3 + n).standard_normal((m, n))
    A[:, : min(m, n) // 3] *= 1e-4   # a graded part
    U, S, Vt = handle.svd(handle.array(A))
    Uh, Sh, Vh = U.numpy(), S.numpy(), Vt.numpy()
    Sr = ref.svd(A)[1]
    k = min(m, n)
    assert np.all(np.diff(Sh) <= 0)
    assert np.max(np.abs(Sh - Sr)) <= 1e-12 * Sr[0]
    assert _rel((Uh * Sh[None, :]) @ Vh, A) <= 1e-13
    assert np.abs(Uh.T @ Uh - np.eye(k)).max() <= 1e-12
    assert np.abs(Vh @ Vh.T - np.eye(k)).max() <= 1e-12
