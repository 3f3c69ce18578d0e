"""ALS / ASD (algorithms/als.cpp) and the dense solves (blasWrapper::solve) on the GPU vs the oracle.

The ALS runs are deterministic given the start: both sides start from the same cores (read back from the
GPU TT) and run the same sweep schedule; the represented tensors are gauge-invariant, so the full tensors
and the returned energies are compared. The full-rank case must reach the dense solution.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tensor(xe, arr):
    return xe.Tensor.from_ndarray(np.require(np.asarray(arr, dtype=np.float64), requirements="C"))


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _laplace_cores(d, n, shift=0.0):
    L = 2 * np.eye(n) - np.eye(n, k=1) - np.eye(n, k=-1) + shift * np.eye(n)
    I = np.eye(n)
    cs = []
    for k in range(d):
        if k == 0:
            c = np.zeros((1, n, n, 2)); c[0, :, :, 0] = L; c[0, :, :, 1] = I
        elif k == d - 1:
            c = np.zeros((2, n, n, 1)); c[0, :, :, 0] = I; c[1, :, :, 0] = L
        else:
            c = np.zeros((2, n, n, 2)); c[0, :, :, 0] = I; c[1, :, :, 0] = L; c[1, :, :, 1] = I
        cs.append(c)
    return cs


def _operator(xe, cores):
    d = len(cores)
    dims = [c.shape[1] for c in cores] + [c.shape[2] for c in cores]
    A = xe.TTOperator(dims)
    for k, c in enumerate(cores):
        A.set_component(k, _tensor(xe, c))
    return A


def _oracle_tt(ref, tt):
    o = ref.TT([tt.get_component(k).to_ndarray() for k in range(tt.degree())])
    o.canonicalized, o.core_position = tt.canonicalized, tt.corePosition
    return o


@pytest.mark.parametrize("variant,spd,asd", [("ALS_SPD", True, False), ("ALS", False, False), ("ASD_SPD", True, True)])
def test_als_matches_oracle(xe, ref, variant, spd, asd):
    d, n = 4, 4
    rng = np.random.default_rng(11)
    cores = _laplace_cores(d, n, shift=0.0 if spd else 0.3)
    if not spd:   # a nonsymmetric operator: perturb the mode coupling
        cores = [c + 0.1 * rng.standard_normal(c.shape) * (c != 0) for c in cores]
    A = _operator(xe, cores)
    b = xe.TTTensor.random([n] * d, [2, 2, 2])
    x = xe.TTTensor.random([n] * d, [2, 3, 2])
    ob, ox = _oracle_tt(ref, b), _oracle_tt(ref, x)
    en = getattr(xe, variant)(A, x, b, 6)
    oen = ref.als(cores, ox, ob, spd=spd, num_half_sweeps=6, asd=asd)
    assert x.ranks() == ox.ranks
    assert _rel(xe.Tensor(x).to_ndarray(), ox.full()) <= 1e-9
    assert en == pytest.approx(oen, rel=1e-9, abs=1e-12)
    assert x.canonicalized and x.corePosition == 0


@pytest.mark.parametrize("variant,spd", [("DMRG_SPD", True), ("DMRG", False)])
def test_dmrg_matches_oracle(xe, ref, variant, spd):
    """Two-site DMRG (als.cpp:43-69, 556-563): merged two-site local solves, SVD splits truncated to the
    initial ranks; same ranks, tensor and energy as the oracle's restatement (oracle/xerus_ref.py:dmrg)."""
    d, n = 5, 4
    rng = np.random.default_rng(13)
    cores = _laplace_cores(d, n, shift=0.0 if spd else 0.3)
    if not spd:
        cores = [c + 0.1 * rng.standard_normal(c.shape) * (c != 0) for c in cores]
    A = _operator(xe, cores)
    b = xe.TTTensor.random([n] * d, [2, 2, 2, 2])
    x = xe.TTTensor.random([n] * d, [2, 3, 3, 2])
    ob, ox = _oracle_tt(ref, b), _oracle_tt(ref, x)
    en = getattr(xe, variant)(A, x, b, 5)
    oen = ref.dmrg(cores, ox, ob, spd=spd, num_half_sweeps=5)
    assert x.ranks() == ox.ranks
    assert _rel(xe.Tensor(x).to_ndarray(), ox.full()) <= 1e-9
    assert en == pytest.approx(oen, rel=1e-9, abs=1e-12)
    assert x.canonicalized and x.corePosition == 0


def test_dmrg_spd_reaches_dense_solution(xe, ref):
    """DMRG_SPD with ranks that hold the solution converges to the dense solve of the Laplace system."""
    d, n = 4, 4
    cores = _laplace_cores(d, n, shift=0.5)
    A = _operator(xe, cores)
    b = xe.TTTensor.random([n] * d, [2, 2, 2])
    x = xe.TTTensor.random([n] * d, [4, 16, 4])
    xe.DMRG_SPD(A, x, b, 1e-13)
    N = n ** d
    M = ref.op_full(cores).reshape(N, N)
    xs = np.linalg.solve(M, xe.Tensor(b).to_ndarray().reshape(N))
    assert _rel(xe.Tensor(x).to_ndarray().reshape(N), xs) <= 1e-9


def test_als_local_system_above_512(xe, ref):
    """ALS (non-SPD: local operator x A^T A x, only approximately symmetric) with interior local systems of
    order 12 * 4 * 12 = 576 > 512: solved through the general (QR) path, same result as the oracle."""
    d, n = 6, 4
    rng = np.random.default_rng(17)
    cores = [c + 0.1 * rng.standard_normal(c.shape) * (c != 0) for c in _laplace_cores(d, n, shift=0.3)]
    A = _operator(xe, cores)
    b = xe.TTTensor.random([n] * d, [2, 2, 2, 2, 2])
    x = xe.TTTensor.random([n] * d, [3, 12, 12, 12, 3])
    ob, ox = _oracle_tt(ref, b), _oracle_tt(ref, x)
    en = xe.ALS(A, x, b, 2)
    oen = ref.als(cores, ox, ob, spd=False, num_half_sweeps=2)
    assert x.ranks() == ox.ranks
    assert _rel(xe.Tensor(x).to_ndarray(), ox.full()) <= 1e-8
    assert en == pytest.approx(oen, rel=1e-8, abs=1e-12)


def test_als_spd_full_rank_reaches_dense_solution(xe, ref):
    d, n = 4, 4
    cores = _laplace_cores(d, n)
    A = _operator(xe, cores)
    b = xe.TTTensor.random([n] * d, [2, 2, 2])
    x = xe.TTTensor.random([n] * d, [4, 16, 4])   # maximal ranks: the boundary components fold away
    xe.ALS_SPD(A, x, b, 1e-13)
    N = n ** d
    M = ref.op_full(cores).reshape(N, N)
    xs = np.linalg.solve(M, xe.Tensor(b).to_ndarray().reshape(N))
    assert _rel(xe.Tensor(x).to_ndarray().reshape(N), xs) <= 1e-10


def test_als_approximation_without_operator(xe, ref):
    d, n = 5, 3
    b = xe.TTTensor.random([n] * d, [2, 3, 3, 2])
    x = xe.TTTensor.random([n] * d, [2, 2, 2, 2])
    ob, ox = _oracle_tt(ref, b), _oracle_tt(ref, x)
    en = xe.ALS_SPD(x, b, 4)
    oen = ref.als(None, ox, ob, spd=True, num_half_sweeps=4)
    assert _rel(xe.Tensor(x).to_ndarray(), ox.full()) <= 1e-10
    assert en == pytest.approx(oen, rel=1e-10)


# ---------------------------------------------------------------------------------------- dense solves
@pytest.mark.parametrize("n,p", [(64, 1), (600, 3), (1100, 2)])
def test_solve_spd_blocked_cholesky(xe, n, p):
    rng = np.random.default_rng(n)
    G = rng.standard_normal((n, n))
    M = G @ G.T / n + np.eye(n)
    B = rng.standard_normal((n, p)) if p > 1 else rng.standard_normal(n)
    X = xe.solve(_tensor(xe, M), _tensor(xe, B), 1 if p > 1 else 0).to_ndarray()   # extraDegree: the rhs columns
    assert X.shape == B.shape
    assert _rel(M @ X, B) <= 1e-12


@pytest.mark.parametrize("m,n", [(200, 200), (300, 120), (120, 300)])
def test_solve_general_and_least_squares(xe, m, n):
    rng = np.random.default_rng(m + n)
    M = rng.standard_normal((m, n))
    B = rng.standard_normal((m, 2))
    X = xe.solve(_tensor(xe, M), _tensor(xe, B), 1).to_ndarray()
    want = np.linalg.lstsq(M, B, rcond=None)[0]
    assert _rel(X, want) <= 1e-10
    X2 = xe.solve_least_squares(_tensor(xe, M), _tensor(xe, B), 1).to_ndarray()
    assert _rel(X2, want) <= 1e-10


@pytest.mark.parametrize("m,n", [(600, 600), (700, 560), (560, 700)])
def test_solve_general_above_512(xe, m, n):
    """min(m, n) > 512: nonsymmetric square, tall least-squares and wide minimum-norm systems through the
    shifted-CholeskyQR3 QR / LQ solve (the reference: dgesv / dgelsd, no size limit)."""
    rng = np.random.default_rng(m * 7 + n)
    M = rng.standard_normal((m, n))
    B = rng.standard_normal((m, 3))
    want = np.linalg.lstsq(M, B, rcond=None)[0]
    X = xe.solve(_tensor(xe, M), _tensor(xe, B), 1).to_ndarray()
    assert _rel(X, want) <= 1e-9
    X2 = xe.solve_least_squares(_tensor(xe, M), _tensor(xe, B), 1).to_ndarray()
    assert _rel(X2, want) <= 1e-9


def test_solve_tensor_modes(xe):
    """A (i, j, k, l) X (k, l) = B (i, j): the leading B.degree() modes of A are contracted (tensor.cpp:1654)."""
    rng = np.random.default_rng(2)
    G = rng.standard_normal((12, 12))
    M = G @ G.T + 12 * np.eye(12)
    B = rng.standard_normal((3, 4))
    X = xe.solve(_tensor(xe, M.reshape(3, 4, 3, 4)), _tensor(xe, B)).to_ndarray()
    assert X.shape == (3, 4)
    assert _rel(M @ X.reshape(12), B.reshape(12)) <= 1e-12
