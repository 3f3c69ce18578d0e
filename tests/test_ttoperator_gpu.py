"""TTOperator and its application (TTStack contraction) on the GPU against the oracle and dense products.

Reference: TTNetwork<true> (ttNetwork.cpp:57-221), TTStack::contract_stack (ttStack.cpp:197-309), the
stack's assignment and canonicalisation (ttNetwork.cpp:1075-1093, ttStack.cpp:160-168). The reference's
own operator tests (ttArithmetic.cxx, ttOperator tests) are property tests on dense equivalents; these
follow them: the contracted result against the dense operator product, ranks against the oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tensor(xe, arr):
    return xe.Tensor.from_ndarray(np.require(np.asarray(arr, dtype=np.float64), requirements="C"))


def _op_cores(op):
    d = op.degree() // 2
    return [op.get_component(k).to_ndarray() for k in range(d)]


def _tt_cores(tt):
    return [tt.get_component(k).to_ndarray() for k in range(tt.degree())]


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _apply_dense(Af, xf):
    d = xf.ndim
    return np.tensordot(Af, xf, axes=(list(range(d, 2 * d)), list(range(d))))


DIMS = [([3, 4, 2, 3], [2, 3, 3, 2], [2, 3, 2], [3, 4, 3]),
        ([5, 5, 5], [5, 5, 5], [3, 3], [4, 6]),
        ([2, 3, 4, 3, 2], [3, 2, 2, 3, 2], [2, 2, 2, 2], [2, 3, 3, 2])]


@pytest.mark.parametrize("n,m,ra,rx", DIMS)
def test_operator_random_full_matches_components(xe, ref, n, m, ra, rx):
    A = xe.TTOperator.random(n + m, ra)
    assert A.degree() == 2 * len(n) and A.dimensions == n + m
    Af = xe.Tensor(A).to_ndarray()
    assert Af.shape == tuple(n + m)
    np.testing.assert_allclose(Af, ref.op_full(_op_cores(A)), rtol=0, atol=1e-12 * np.abs(Af).max())
    assert A.canonicalized and A.corePosition == 0
    assert A.frob_norm() == pytest.approx(np.linalg.norm(Af), rel=1e-12)


@pytest.mark.parametrize("n,m,ra,rx", DIMS)
def test_apply_matches_dense_and_oracle(xe, ref, n, m, ra, rx):
    A = xe.TTOperator.random(n + m, ra)
    x = xe.TTTensor.random(m, rx)
    i, j = xe.Index(), xe.Index()
    y = xe.TTTensor()
    y(i & 0) << A(i / 2, j / 2) * x(j & 0)
    Af, xf = xe.Tensor(A).to_ndarray(), xe.Tensor(x).to_ndarray()
    yd = _apply_dense(Af, xf)
    assert y.dimensions == n
    assert _rel(xe.Tensor(y).to_ndarray(), yd) <= 1e-12
    # the stack's contraction, then move_core to the operator's core position (ttStack.cpp:163-166)
    o = ref.TT(ref.op_apply_cores(_op_cores(A), _tt_cores(x)))
    o.move_core(A.corePosition)
    assert y.ranks() == o.ranks
    assert y.canonicalized and y.corePosition == A.corePosition


def test_apply_raw_cores_bitwise_order(handle, ref):
    """xrs_tt_operator_apply through the C-ABI: each product core against the oracle's einsum (fused rank
    index operator-major), and the transposed form."""
    rng = np.random.default_rng(3)
    d, n, m, ra, rx = 3, [3, 2, 4], [2, 3, 2], [1, 2, 3, 1], [1, 3, 2, 1]
    A = [rng.standard_normal((ra[k], n[k], m[k], ra[k + 1])) for k in range(d)]
    X = [rng.standard_normal((rx[k], m[k], rx[k + 1])) for k in range(d)]
    Z = [rng.standard_normal((rx[k], n[k], rx[k + 1])) for k in range(d)]
    for tr, V in ((False, X), (True, Z)):
        got = handle.tt_operator_apply(n, m, ra, [handle.array(a) for a in A], rx, [handle.array(v) for v in V], transpose=tr)
        want = ref.op_apply_cores(A, V, transpose=tr)
        for g, w in zip(got, want):
            assert g.shape == w.shape
            np.testing.assert_allclose(g, w, rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("n,m,ra,rx", DIMS[:2])
def test_transposed_application(xe, ref, n, m, ra, rx):
    A = xe.TTOperator.random(n + m, ra)
    x = xe.TTTensor.random(n, rx)
    i, j = xe.Index(), xe.Index()
    y = xe.TTTensor()
    y(j & 0) << x(i & 0) * A(i / 2, j / 2)
    Af, xf = xe.Tensor(A).to_ndarray(), xe.Tensor(x).to_ndarray()
    d = len(n)
    yd = np.tensordot(xf, Af, axes=(list(range(d)), list(range(d))))
    assert y.dimensions == m
    assert _rel(xe.Tensor(y).to_ndarray(), yd) <= 1e-12


def test_operator_product_and_transpose(xe):
    n, m, p = [3, 2, 4], [2, 3, 2], [2, 2, 3]
    A = xe.TTOperator.random(n + m, [2, 3])
    B = xe.TTOperator.random(m + p, [3, 2])
    i, j, k = xe.Index(), xe.Index(), xe.Index()
    C = xe.TTOperator()
    C(i / 2, k / 2) << A(i / 2, j / 2) * B(j / 2, k / 2)
    Af, Bf = xe.Tensor(A).to_ndarray(), xe.Tensor(B).to_ndarray()
    Cd = np.tensordot(Af, Bf, axes=([3, 4, 5], [0, 1, 2]))
    assert C.dimensions == n + p
    assert _rel(xe.Tensor(C).to_ndarray(), Cd) <= 1e-12
    At = xe.TTOperator(A)
    At.transpose()
    assert At.dimensions == m + n
    np.testing.assert_allclose(xe.Tensor(At).to_ndarray(), np.transpose(Af, [3, 4, 5, 0, 1, 2]), rtol=0, atol=1e-13)


def test_identity_and_scalar_products(xe):
    n = [3, 4, 3, 2]
    I = xe.TTOperator.identity(n + n)
    x = xe.TTTensor.random(n, [2, 3, 2])
    y = xe.TTTensor.random(n, [3, 2, 2])
    i, j = xe.Index(), xe.Index()
    z = xe.TTTensor()
    z(i & 0) << I(i / 2, j / 2) * x(j & 0)
    assert _rel(xe.Tensor(z).to_ndarray(), xe.Tensor(x).to_ndarray()) <= 1e-13
    A = xe.TTOperator.random(n + n, [2, 2, 2])
    Af, xf, yf = xe.Tensor(A).to_ndarray(), xe.Tensor(x).to_ndarray(), xe.Tensor(y).to_ndarray()
    want = float(np.sum(yf * _apply_dense(Af, xf)))
    got = (A(i / 2, j / 2) * x(j & 0)) * y(i & 0)
    assert got == pytest.approx(want, rel=1e-11)
    got2 = (y(i & 0) * A(i / 2, j / 2)) * x(j & 0)
    assert got2 == pytest.approx(want, rel=1e-11)


def test_operator_tt_svd_and_round(xe, ref):
    rng = np.random.default_rng(9)
    n, m = [3, 2, 3], [2, 3, 2]
    A0 = xe.TTOperator.random(n + m, [2, 3])
    Af = xe.Tensor(A0).to_ndarray()
    Af = Af + 1e-10 * rng.standard_normal(Af.shape)
    A = xe.TTOperator(_tensor(xe, Af), 1e-6)
    # the reference's operator TT-SVD = the TT-SVD of the mode-interleaved tensor (ttNetwork.cpp:128-146)
    inter = np.transpose(Af, [0, 3, 1, 4, 2, 5]).reshape([n[k] * m[k] for k in range(3)])
    o = ref.tt_svd(inter, 1e-6, [0, 0])
    assert A.ranks() == o.ranks == [2, 3]
    assert _rel(xe.Tensor(A).to_ndarray(), Af) <= 1e-8
    # a canonical sum is re-canonicalised with the rank-revealing QC (ttNetwork.cpp:841-843). Whether that
    # QC drops the duplicated ranks depends on the sign of its pivoted R_00 (the reference's rule is signed,
    # blasLapackWrapper.cpp:268-272), i.e. on the gauge of A's cores: the oracle runs the reference's sum +
    # move_core on the SAME cores, and the ranks must agree (per edge: kept when R_00 > 0, doubled otherwise)
    S = A + A
    cores = [np.asarray(A.get_component(k).to_ndarray()) for k in range(3)]
    oa = ref.TT([c.reshape(c.shape[0], -1, c.shape[-1]) for c in cores])
    os_ = ref.tt_add(oa, oa)
    os_.move_core(A.corePosition)
    assert S.ranks() == os_.ranks
    assert S.ranks()[0] in (2, 4) and S.ranks()[1] in (3, 6)   # (per edge: the sign of that edge's R_00)
    assert _rel(xe.Tensor(S).to_ndarray(), 2 * Af) <= 1e-8
    # a non-canonical summand keeps the block-diagonal ranks; round() then cuts them
    B = xe.TTOperator(A)
    B.set_component(1, B.get_component(1))   # set_component away from the core drops canonicalized (:491)
    assert not B.canonicalized
    S2 = B + A
    assert S2.ranks() == [4, 6]
    S2.round(1e-12)
    assert S2.ranks() == [2, 3]
    assert _rel(xe.Tensor(S2).to_ndarray(), 2 * Af) <= 1e-8
