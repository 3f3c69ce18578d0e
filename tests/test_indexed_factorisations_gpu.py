"""The indexed factorisation front end on the GPU: (U(i,r), S(r,s), Vt(s,j)) << SVD(A(i,j), ...), QR, RQ, QC,
CQ, the SVD soft threshold and TTTensor.soft_threshold.

Ports of the reference's unit tests (src/unitTests/fullTensor_factorisations.cxx: SVD_Identity :25,
SVD_zero :54, SVD_Random_512x512 :69, SVD_soft_thresholding :111, SVD_Random_Order_Six :140,
QR_AND_RQ_Random_Order_Six :170, QC :248) with their tolerances, plus oracle parity of the singular
values / kept ranks (oracle/xerus_ref.py, dgesdd) and of the TT soft threshold
(ttNetwork.cpp:688-713 -> tensorNetwork.cpp:678-818 with _softThreshold).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _T(xe, a):
    return xe.Tensor.from_ndarray(np.ascontiguousarray(a, dtype=np.float64))


def _orth_dev(xe, U, k, S):
    """frob_norm(U(i^k, m) * U(i^k, n) - I(m, n)) with U's LAST mode the rank."""
    i, m, n = xe.indices(3)
    G = xe.Tensor()
    G(m, n) << U(i ** k, m) * U(i ** k, n)
    return np.linalg.norm(G.to_ndarray() - np.eye(S.dimensions[0]))


def _orth_dev_rows(xe, V, k, S):
    i, m, n = xe.indices(3)
    G = xe.Tensor()
    G(m, n) << V(m, i ** k) * V(n, i ** k)
    return np.linalg.norm(G.to_ndarray() - np.eye(S.dimensions[0]))


def test_svd_identity(xe):
    """fullTensor_factorisations.cxx:25-51"""
    A = np.zeros((2, 2, 2, 2))
    for idx in [(0, 0, 0, 0), (0, 1, 0, 1), (1, 0, 1, 0), (1, 1, 1, 1)]:
        A[idx] = 1.0
    tA = _T(xe, A)
    res1, res2, res3 = xe.Tensor([2, 2, 4]), xe.Tensor([4, 4]), xe.Tensor([4, 2, 2])
    i, j, k, l, m, n = xe.indices(6)
    (res1(i, j, m), res2(m, n), res3(n, k, l)) << xe.SVD(tA(i, j, k, l))
    assert np.allclose(res2.to_ndarray().reshape(2, 2, 2, 2), A, atol=1e-15)
    assert _orth_dev(xe, res1, 2, res2) < 1e-12
    assert _orth_dev_rows(xe, res3, 2, res2) < 1e-12
    (res1(m, i, j), res2(n, m), res3(k, n, l)) << xe.SVD(tA(i, j, k, l))
    assert np.allclose(res2.to_ndarray().reshape(2, 2, 2, 2), A, atol=1e-15)
    assert list(res1.dimensions) == [4, 2, 2] and list(res3.dimensions) == [2, 4, 2]


def test_svd_zero(xe):
    """fullTensor_factorisations.cxx:54-66: the zero tensor has rank 1 with sigma 0."""
    tA = xe.Tensor([2, 2, 2, 2])
    res1, res2, res3 = xe.Tensor(), xe.Tensor(), xe.Tensor()
    i, j, k, l, m, n = xe.indices(6)
    (res1(i, j, m), res2(m, n), res3(n, k, l)) << xe.SVD(tA(i, j, k, l))
    assert res2.dimensions[0] == 1
    assert abs(res2[0]) < 1e-15
    assert _orth_dev(xe, res1, 2, res2) < 1e-12
    assert _orth_dev_rows(xe, res3, 2, res2) < 1e-12


@pytest.mark.parametrize("dims", [(8, 8, 8, 8, 8, 8), (9, 7, 5, 5, 9, 7)])
def test_svd_random_order_six(xe, ref, dims):
    """fullTensor_factorisations.cxx:69-108 (512 x 512) and :140-167; reconstruction 1e-14, orthogonality
    1e-12, singular values vs dgesdd of the same matricisation."""
    rng = np.random.default_rng(sum(dims))
    A = rng.standard_normal(dims)
    tA = _T(xe, A)
    res1, res2, res3, res4 = xe.Tensor(), xe.Tensor(), xe.Tensor(), xe.Tensor()
    i, j, k, l, m, n, o, p = xe.indices(8)
    (res1(i, j, k, o), res2(o, p), res3(p, l, m, n)) << xe.SVD(tA(i, j, k, l, m, n))
    res4(i, j, k, l, m, n) << res1(i, j, k, o) * res2(o, p) * res3(p, l, m, n)
    assert xe.approx_equal(res4, tA, 1e-14)
    assert _orth_dev(xe, res1, 3, res2) < 1e-12
    assert _orth_dev_rows(xe, res3, 3, res2) < 1e-12
    s_ref = ref.svd(A.reshape(int(np.prod(dims[:3])), -1))[1]
    s = np.diag(res2.to_ndarray())
    assert np.max(np.abs(s - s_ref[: len(s)])) <= 1e-12 * s_ref[0]

    # permuted base: A(l,k,m,i,j,n) -> rows (i,j,k), columns (l,m,n)
    (res1(i, j, k, o), res2(o, p), res3(p, l, m, n)) << xe.SVD(tA(l, k, m, i, j, n))
    res4(l, k, m, i, j, n) << res1(i, j, k, o) * res2(o, p) * res3(p, l, m, n)
    assert xe.approx_equal(res4, tA, 1e-14)
    # rank index not last / first in the outputs (:98-103)
    (res1(i, o, k, j), res2(p, o), res3(l, n, m, p)) << xe.SVD(-1 * tA(l, i, m, k, j, n))
    res4(l, k, m, i, j, n) << res1(k, o, i, j) * res2(p, o) * res3(l, n, m, p)
    assert xe.approx_equal(-1 * res4, tA, 1e-14)


def test_svd_max_rank_eps(xe, ref):
    """SVD(A, maxRank, eps): the cut of calculate_svd (tensor.cpp:1462-1474), ranks identical to the oracle."""
    rng = np.random.default_rng(5)
    U0, _ = np.linalg.qr(rng.standard_normal((60, 40)))
    V0, _ = np.linalg.qr(rng.standard_normal((50, 40)))
    s0 = 0.7 ** np.arange(40)
    A = (U0 * s0) @ V0.T
    tA = _T(xe, A.reshape(6, 10, 5, 10))
    U, S, Vt = xe.Tensor(), xe.Tensor(), xe.Tensor()
    i, j, k, l, r1, r2 = xe.indices(6)
    s_ref = ref.svd(A)[1]
    for max_rank, eps in [(2 ** 62, 1e-6), (12, 1e-12), (30, 0.01), (2 ** 62, 8 * np.finfo(float).eps)]:
        (U(i, j, r1), S(r1, r2), Vt(r2, k, l)) << xe.SVD(tA(i, j, k, l), max_rank, eps)
        want = ref.svd_rank(s_ref, max_rank, eps)
        assert S.dimensions[0] == want, (max_rank, eps)
        assert list(U.dimensions) == [6, 10, want] and list(Vt.dimensions) == [want, 5, 10]
        s = np.diag(S.to_ndarray())
        assert np.max(np.abs(s - s_ref[:want])) <= 1e-13 * s_ref[0]


def test_svd_soft_thresholding(xe):
    """fullTensor_factorisations.cxx:111-138 (Tensor:SVD_soft_thresholding)."""
    rng = np.random.default_rng(111)
    A = 10 * rng.standard_normal((3, 5, 2, 7, 3, 12))
    tA = _T(xe, A)
    U, S, V, Us, Ss, Vs, Ax = (xe.Tensor() for _ in range(7))
    i, j, k, l, m, n, o, p = xe.indices(8)
    (U(i, j, k, o), S(o, p), V(p, l, m, n)) << xe.SVD(tA(i, j, k, l, m, n))
    (Us(i, j, k, o), Ss(o, p), Vs(p, l, m, n)) << xe.SVD(tA(i, j, k, l, m, n), softThreshold=7.3)
    U.resize_mode(U.degree() - 1, Ss.dimensions[0])
    V.resize_mode(0, Ss.dimensions[0])
    assert xe.approx_equal(U, Us, 1e-12)
    assert xe.approx_equal(V, Vs, 1e-12)
    Sd, Ssd = S.to_ndarray(), Ss.to_ndarray()
    for x in range(S.dimensions[0]):
        if x < Ss.dimensions[0]:
            assert abs(Ssd[x, x] - max(0.0, Sd[x, x] - 7.3)) <= 3e-13 * max(1.0, Sd[x, x])
        else:
            assert Sd[x, x] <= 7.3
    Ax(i, j, k, l, m, n) << U(i, j, k, o) * S(o, p) * V(p, l, m, n)
    assert xe.approx_equal(tA, Ax, 1e-12)
    i2 = xe.Index()
    G = xe.Tensor()
    G(o, p) << U(i, j, k, o) * U(i, j, k, p)
    assert np.linalg.norm(G.to_ndarray() - np.eye(S.dimensions[0])) < 1e-12
    G(o, p) << V(o, l, m, n) * V(p, l, m, n)
    assert np.linalg.norm(G.to_ndarray() - np.eye(S.dimensions[0])) < 1e-12
    del i2
    # a threshold inside the spectrum: the ranks drop to the values above it (:158-163)
    tau = float(np.median(np.diag(Sd)))
    (Us(i, j, k, o), Ss(o, p), Vs(p, l, m, n)) << xe.SVD(tA(i, j, k, l, m, n), softThreshold=tau)
    keep = int(np.sum(np.diag(Sd)[1:] >= tau)) + 1
    assert Ss.dimensions[0] == keep < S.dimensions[0]
    assert np.allclose(np.diag(Ss.to_ndarray()), np.maximum(0.0, np.diag(Sd)[:keep] - tau), rtol=0, atol=3e-13 * Sd[0, 0])
    # preventZero keeps sigma_0 at >= EPSILON sigma_0 when the threshold exceeds it
    (Us(i, j, k, o), Ss(o, p), Vs(p, l, m, n)) << xe.SVD(tA(i, j, k, l, m, n), softThreshold=1e6, preventZero=True)
    assert Ss.dimensions[0] == 1
    assert Ss[0] == pytest.approx(8 * np.finfo(float).eps * Sd[0, 0], rel=1e-12)


def test_qr_rq_random_order_six(xe):
    """fullTensor_factorisations.cxx:170-245 (QR_AND_RQ_Random_Order_Six), incl. a fixed index."""
    rng = np.random.default_rng(170)
    A = rng.standard_normal((7, 5, 9, 7, 5, 9))
    tA = _T(xe, A)
    Q, R, Q2, R2, Q3, R3, Q4, res4 = (xe.Tensor() for _ in range(8))
    i, j, k, l, m, n, o, p, q, r = xe.indices(10)

    def orth(X, rows):
        return np.linalg.norm(X - np.eye(X.shape[0])) if rows else 0.0

    (Q(i, j, k, l), R(l, m, n, r)) << xe.QR(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q(i, j, k, o) * R(o, m, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    G = xe.Tensor()
    G(l, m) << Q(i, j, k, l) * Q(i, j, k, m)
    assert orth(G.to_ndarray(), True) < 1e-12
    (Q(i, j, k, l), R(l, m, n, r)) << xe.QR(tA(i, n, k, m, j, r))
    res4(i, n, k, m, j, r) << Q(i, j, k, o) * R(o, m, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    (Q2(i, k, l), R2(l, m, j, n, r)) << xe.QR(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q2(i, k, o) * R2(o, m, j, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    (Q3(i, m, j, k, l), R3(l, n, r)) << xe.QR(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q3(i, m, j, k, o) * R3(o, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    (Q(i, l, j, k, m), R(l, n, r)) << xe.QR(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q(i, o, j, k, m) * R(o, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    G(l, q) << Q(i, l, j, k, m) * Q(i, q, j, k, m)
    assert orth(G.to_ndarray(), True) < 1e-12

    (R(i, j, k, l), Q(l, m, n, r)) << xe.RQ(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << R(i, j, k, o) * Q(o, m, n, r)
    assert xe.approx_equal(res4, tA, 5e-15)
    G(p, q) << Q(p, m, n, r) * Q(q, m, n, r)
    assert orth(G.to_ndarray(), True) < 1e-12
    (R(i, j, k, l), Q(l, m, n, r)) << xe.RQ(tA(i, n, k, m, j, r))
    res4(i, n, k, m, j, r) << R(i, j, k, o) * Q(o, m, n, r)
    assert xe.approx_equal(res4, tA, 5e-15)
    (R2(i, m, j, k, l), Q2(l, n, r)) << xe.RQ(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << R2(i, m, j, k, l) * Q2(l, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    (R3(i, k, l), Q3(l, m, j, n, r)) << xe.RQ(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << R3(i, k, o) * Q3(o, m, j, n, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    (R(l, i, k), Q(n, m, j, l, r)) << xe.RQ(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << R(o, i, k) * Q(n, m, j, o, r)
    assert xe.approx_equal(res4, tA, 2e-15)
    G(p, q) << Q(n, m, j, q, r) * Q(n, m, j, p, r)
    assert orth(G.to_ndarray(), True) < 1e-12
    # a fixed index in the base (:239-243)
    (R3(i, k, l), Q4(l, j, n, r)) << xe.RQ(tA(i, j, k, 3, n, r))
    res4(i, j, k, n, r) << R3(i, k, o) * Q4(o, j, n, r)
    assert np.linalg.norm(A[:, :, :, 3, :, :] - res4.to_ndarray()) < 1e-12


def test_qc_cq(xe, ref):
    """fullTensor_factorisations.cxx:248-285 (QC) and the CQ counterpart; the rank of a rank-deficient base
    is the oracle's pivoted-QR rank rule (blasLapackWrapper.cpp:268-272)."""
    rng = np.random.default_rng(248)
    A = rng.standard_normal((2, 2, 2, 2, 2, 2))
    tA = _T(xe, A)
    B = _T(xe, np.arange(6, dtype=float).reshape(2, 3))
    Q, R, Q2, R2, Q3, R3, res4 = (xe.Tensor() for _ in range(7))
    i, j, k, l, m, n, o, p, q, r = xe.indices(10)
    (Q(i, j), R(j, k)) << xe.QC(B(i, k))
    assert Q.dimensions[1] == ref.qc(np.arange(6, dtype=float).reshape(2, 3))[2] == 2
    (Q(i, j, k, l), R(l, m, n, r)) << xe.QC(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q(i, j, k, o) * R(o, m, n, r)
    assert xe.approx_equal(res4, tA, 1e-15)
    (Q2(i, k, l), R2(l, m, j, n, r)) << xe.QC(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q2(i, k, o) * R2(o, m, j, n, r)
    assert xe.approx_equal(res4, tA, 1e-12)
    (Q3(i, m, j, k, l), R3(l, n, r)) << xe.QC(tA(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << Q3(i, m, j, k, o) * R3(o, n, r)
    assert xe.approx_equal(res4, tA, 1e-15)
    # rank-deficient base: rank 3 of a 12 x 10 matricisation
    D = (rng.standard_normal((12, 3)) @ rng.standard_normal((3, 10))).reshape(3, 4, 2, 5)
    tD = _T(xe, D)
    C, Qc = xe.Tensor(), xe.Tensor()
    (Q(i, j, l), C(l, m, n)) << xe.QC(tD(i, j, m, n))
    assert Q.dimensions[2] == ref.qc(D.reshape(12, 10))[2]
    res4(i, j, m, n) << Q(i, j, o) * C(o, m, n)
    assert xe.approx_equal(res4, tD, 1e-13)
    (C(i, j, l), Qc(l, m, n)) << xe.CQ(tD(i, j, m, n))
    assert C.dimensions[2] == ref.cq(D.reshape(12, 10))[2]
    res4(i, j, m, n) << C(i, j, o) * Qc(o, m, n)
    assert xe.approx_equal(res4, tD, 1e-13)
    G = xe.Tensor()
    G(l, q) << Qc(l, m, n) * Qc(q, m, n)
    assert np.linalg.norm(G.to_ndarray() - np.eye(Qc.dimensions[0])) < 1e-12


def test_factorisation_errors(xe):
    """prepare_split's preconditions (indexedTensor_tensor_factorisations.cpp:46-116) throw."""
    tA = _T(xe, np.ones((3, 4)))
    U, S, Vt = xe.Tensor(), xe.Tensor(), xe.Tensor()
    i, j, k, r1, r2, r3 = xe.indices(6)
    with pytest.raises(Exception):   # j of the base in neither output
        (U(i, r1), S(r1, r2), Vt(r2, k)) << xe.SVD(tA(i, j))
    with pytest.raises(Exception):   # two new indices on the left
        (U(i, r1, r3), S(r1, r2), Vt(r2, j)) << xe.SVD(tA(i, j))
    with pytest.raises(Exception):   # three outputs for QR
        (U(i, r1), S(r1, r2), Vt(r2, j)) << xe.QR(tA(i, j))


@pytest.mark.parametrize("dims,ranks,tau", [([2] * 10, [2] * 9, 0.3), ([4, 5, 3, 6, 4], [4, 8, 7, 4], 0.5),
                                            ([20] * 6, [30] * 5, 2.0)])
def test_tt_soft_threshold(xe, ref, dims, ranks, tau):
    """TTNetwork::soft_threshold (ttNetwork.cpp:688-713; TT:soft_thresholding's operation) vs the oracle:
    same ranks, same represented tensor (1e-10) -- the thresholded values are the tensor's own singular
    values edge by edge, so the result is gauge-invariant."""
    xe.seed(0xBAADF00D)
    x = xe.TTTensor.random(dims, ranks)
    cores = [x.get_component(k).to_ndarray() for k in range(len(dims))]
    ox = ref.TT([c.copy() for c in cores], True, 0)
    taus = [tau * (1 + 0.1 * e) for e in range(len(dims) - 1)]   # distinct: checks the reversed order
    x.soft_threshold(taus)
    ox.soft_threshold(taus)
    assert x.ranks() == ox.ranks
    full = ox.full()
    got = xe.Tensor(x).to_ndarray() if np.prod(dims) <= 4_000_000 else None
    if got is not None:
        assert np.linalg.norm(got - full) <= 1e-10 * max(np.linalg.norm(full), 1e-300)
    assert x.canonicalized and x.corePosition == 0
