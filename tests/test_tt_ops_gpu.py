"""Ports of the reference's TT unit tests that need the TT operations around rounding (entrywise / dyadic
products, kronecker / dirac, fix_mode / resize_mode, chop) -- each test cites its source
(src/unitTests/*.cxx:line), keeps its inputs' shapes, operations and tolerances, and checks the TT results
against the dense Tensor computed the same way, as the reference does. The reference's sparse-Tensor and
TensorNetwork legs are out of scope (dense only); random draws come from the library's own
mt19937_64 stream (seeded per test), the dimensions of the reference's randomised loops from numpy.

approx_equal(a, b, eps) is the reference's: ||a - b|| <= eps (||a|| + ||b||) / 2 (tensor.cpp:1646-1651).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EPSILON = 8 * np.finfo(float).eps   # xerus EPSILON (basic.h)


def nd(x, xe):
    return (x if isinstance(x, np.ndarray) else xe.Tensor(x).to_ndarray() if not hasattr(x, "to_ndarray") else x.to_ndarray())


class _Approx:
    """truthy when ||a - b|| <= eps (||a|| + ||b||) / 2; repr shows the ratio (failure messages)"""

    def __init__(self, a, b, eps):
        a, b = np.asarray(a), np.asarray(b)
        self.shape = (a.shape, b.shape)
        self.ratio = np.linalg.norm(a - b) / max((np.linalg.norm(a) + np.linalg.norm(b)) / 2, 1e-300) if a.shape == b.shape else np.inf
        self.eps = eps

    def __bool__(self):
        return bool(self.ratio <= self.eps)

    def __repr__(self):
        return f"approx(ratio {self.ratio:.3e} vs eps {self.eps:.1e}, shapes {self.shape})"


def approx(a, b, eps=EPSILON):
    return _Approx(a, b, eps)


def full(xe, t):
    return xe.Tensor(t).to_ndarray()


def op_apply(A, X, d):
    """dense C(i&0) = A(i/2, j/2) * X(j&0)"""
    return np.tensordot(A, X, axes=(list(range(d, 2 * d)), list(range(d))))


# ---------------------------------------------------------------------------------------- ttOther.cxx
def test_entrywise_product(xe):
    """TT:entrywise_product (ttOther.cxx:6-34)."""
    xe.seed(0xBAADF00D)
    A = xe.TTTensor.random([2] * 10, [2] * 9)
    B = xe.TTTensor.random([2] * 10, [2] * 9)
    Af, Bf = xe.Tensor(A), xe.Tensor(B)
    Ao, Bo = xe.TTOperator(Af), xe.TTOperator(Bf)
    C = xe.entrywise_product(A, B)
    Co = xe.entrywise_product(Ao, Bo)
    Cf = xe.entrywise_product(Af, Bf).to_ndarray()
    assert np.array_equal(Cf, Af.to_ndarray() * Bf.to_ndarray())
    assert np.linalg.norm(Cf - full(xe, Co)) / np.linalg.norm(Cf) < 1e-13
    assert np.linalg.norm(Cf - full(xe, C)) / np.linalg.norm(Cf) < 1e-13
    # rank 2 x 2 per edge; both inputs are canonical, so the product is moved to core 0 by the rank-revealing
    # QC, which cuts the end edges to their structural maximum (n_0 = n_9 = 2)
    assert C.ranks() == xe.TTTensor.reduce_to_maximal_ranks([4] * 9, [2] * 10)
    D1 = xe.entrywise_product(A, A)
    Do1 = xe.entrywise_product(Ao, Ao)
    Df = xe.entrywise_product(Af, Af).to_ndarray()
    assert approx(Df, full(xe, D1), 1e-13)
    assert approx(Df, full(xe, Do1), 1e-13)


def test_entrywise_product_soft_thresholding_file(xe):
    """TT:soft_thresholding (ttOther.cxx:36-56): despite its name the same products, at 1e-14."""
    xe.seed(0xBAADF00D + 1)
    A = xe.TTTensor.random([2] * 10, [2] * 9)
    B = xe.TTTensor.random([2] * 10, [2] * 9)
    Af, Bf = xe.Tensor(A), xe.Tensor(B)
    Ao, Bo = xe.TTOperator(Af), xe.TTOperator(Bf)
    Cf = xe.entrywise_product(Af, Bf).to_ndarray()
    assert np.linalg.norm(Cf - full(xe, xe.entrywise_product(Ao, Bo))) / np.linalg.norm(Cf) < 1e-14
    assert np.linalg.norm(Cf - full(xe, xe.entrywise_product(A, B))) / np.linalg.norm(Cf) < 1e-14


def test_non_operator_pseudo_inverse(xe):
    """TT:Non-operator Pseudo Inverse (ttOther.cxx:58-85): chop at the middle, SVD of the middle core with
    the singular values inverted above 1e-10, pInv = left * U S^+ V * right; A^+ A A^+ = A^+ and
    A A^+ A = A to 1e-10 (the order-4 TT as a 100 x 100 matrix)."""
    d = 2
    xe.seed(0xBAADF00D + 2)
    op = xe.TTTensor.random([10] * (2 * d), [4] * (2 * d - 1))
    tmp = xe.TTTensor(op)
    tmp.move_core(d)
    left, right = tmp.chop(d)
    assert left.dimensions == [10, 10, 4] and right.dimensions == [4, 10]
    core = tmp.get_component(d)
    U, S, V = xe.calculate_svd(core, 1)                  # core(i, j^2): U (4, r), S (r, r), V (r, 10, 4)
    s = S.to_ndarray()
    sd = np.diag(s).copy()
    sd[sd > 1e-10] = 1.0 / sd[sd > 1e-10]
    L, R = left.to_tensor().to_ndarray(), right.to_tensor().to_ndarray()
    # pInv(j, i^(d-1), k^d) = L(k^d, r1) U(r1, r2) S(r2, r3) V(r3, j, r4) R(r4, i^(d-1))
    P = np.einsum("abr,rs,s,sjt,ti->jiab", L, U.to_ndarray(), sd, V.to_ndarray(), R)
    Pm = P.reshape(100, 100)
    Am = full(xe, op).reshape(100, 100)
    assert np.linalg.norm(Pm @ Am @ Pm - Pm) < 1e-10
    assert np.linalg.norm(Am @ Pm @ Am - Am) < 1e-10
    # chop reassembles the TT: left * core * right
    T = np.einsum("abr,rjt,ti->abji", L, core.to_ndarray(), R)
    assert approx(T, full(xe, tmp), 1e-14)


# ---------------------------------------------------------------------------------------- ttCreation.cxx
@pytest.mark.parametrize("dims", [[2], [2, 2], [2, 7], [2] * 8, [7, 5, 3, 1, 4, 2, 8, 1]])
def test_tttensor_creation(xe, dims):
    """TT:TTTensor_Creation (ttCreation.cxx:27-60): TT-SVD at eps 1e-14 reproduces the tensor to 1e-14."""
    xe.seed(27 + len(dims))
    A = xe.Tensor.random(dims)
    tt = xe.TTTensor(A, 1e-14)
    assert approx(full(xe, tt), A.to_ndarray(), 1e-14)


@pytest.mark.parametrize("dims", [[2, 2], [2, 7], [2, 7, 3, 1], [2] * 8, [7, 5, 6, 3, 1, 4, 2, 1]])
def test_ttoperator_creation(xe, dims):
    """TT:TTOperator_Creation (ttCreation.cxx:62-95)."""
    xe.seed(62 + len(dims))
    A = xe.Tensor.random(dims)
    tt = xe.TTOperator(A, 1e-14)
    assert approx(full(xe, tt), A.to_ndarray(), 1e-14)


def test_creation_with_epsilon(xe):
    """TT:creation_with_epsilon (ttCreation.cxx:97-111): TT-SVD with eps 0.03 and round(0.03) of the exact
    TT cut the middle rank below 25 with error below (number of dropped ranks) * eps."""
    eps = 0.03
    xe.seed(97)
    A = xe.Tensor.random([5, 5, 5, 5])
    ttA = xe.TTTensor(A, eps)
    ttB = xe.TTTensor(A, 0.0)
    ttB.round(eps)
    num_decrease = 5 - ttA.rank(0) + 25 - ttA.rank(1) + 5 - ttA.rank(2)
    a = A.to_ndarray()
    assert np.linalg.norm(a - full(xe, ttA)) / np.linalg.norm(a) < num_decrease * eps
    assert ttA.ranks()[1] < 25
    assert np.linalg.norm(a - full(xe, ttB)) / np.linalg.norm(a) < num_decrease * eps
    assert ttB.ranks()[1] < 25


def test_creation_from_full_tensor_5x5x5x5(xe):
    """TT:creation_from_fullTensor_5x5x5x5 (ttCreation.cxx:113-123)."""
    xe.seed(113)
    A = xe.Tensor.random([5, 5, 5, 5])
    B = full(xe, xe.TTTensor(A))
    assert approx(A.to_ndarray(), B, 1e-14)
    assert np.linalg.norm(A.to_ndarray() - B) < 1e-13 * 5 ** 4


def test_named_constructors(xe):
    """TT:named_constructors (ttCreation.cxx:125-181): ranks survive move_core sweeps; identity, ones."""
    dims, opdims = [2] * 10, [2] * 20
    ranks = [4] * 9
    ranks[4] = 1
    xe.seed(125)
    X = xe.TTTensor.random(dims, ranks)
    found = X.ranks()
    X.move_core(X.degree() - 1)
    X.move_core(0)
    assert X.ranks() == found
    Xop = xe.TTOperator.random(opdims, ranks)
    found = Xop.ranks()
    Xop.move_core(X.degree() - 1)
    Xop.move_core(0)
    assert Xop.ranks() == found
    ident = xe.TTOperator.identity(opdims)
    assert ident.ranks() == [1] * 9
    i, j = xe.indices(2)
    X2 = xe.TTTensor()
    X2(j & 0) << ident(j / 2, i / 2) * X(i & 0)
    assert xe.frob_norm(X2 - X) < 1e-14 * 1024
    ones = xe.TTTensor.ones(dims)
    assert ones.ranks() == [1] * 9
    assert np.linalg.norm(full(xe, ones) - np.ones(dims)) < 1e-14 * 1024
    opones = xe.TTOperator.ones(dims)
    assert opones.ranks() == [1] * 4
    assert np.linalg.norm(full(xe, opones) - np.ones(dims)) < 1e-14 * 1024


def test_dyadic_product(xe):
    """TT:dyadic_product (ttCreation.cxx:183-221): products of order-1 TTs / operators are canonical with the
    core at 0 and ||O S|| = prod ||o_i s_i||; sums of dyadic products stay canonical."""
    xe.seed(183)
    o = [xe.TTOperator.random([10, 10], []) for _ in range(3)]
    s = [xe.TTTensor.random([10], []) for _ in range(3)]
    O = xe.dyadic_product(o)
    S = xe.dyadic_product(s)
    assert O.canonicalized and O.corePosition == 0
    assert S.canonicalized and S.corePosition == 0
    i, j = xe.indices(2)
    r = 1.0
    for oi, si in zip(o, s):
        y = xe.TTTensor()
        y(i & 0) << oi(i / 2, j / 2) * si(j & 0)
        r *= y.frob_norm()
    Y = xe.TTTensor()
    Y(i & 0) << O(i / 2, j / 2) * S(j & 0)
    assert abs(Y.frob_norm() - r) < 1e-12
    # dense check of the structure: O S = (o1 s1) x (o2 s2) x (o3 s3)
    dense = [op_apply(full(xe, oi), full(xe, si), 1) for oi, si in zip(o, s)]
    assert approx(full(xe, Y), np.einsum("a,b,c->abc", *dense), 1e-13)
    S = xe.dyadic_product(S, xe.TTTensor.ones([10])) + xe.dyadic_product(xe.TTTensor.ones([10]), S)
    assert S.canonicalized and S.corePosition == 0
    e0 = np.zeros(10)
    e0[0] = 1.0
    e1 = np.zeros(10)
    e1[1] = 1.0
    Sd = full(xe, S)
    S = S * (1 / np.sqrt(2))
    S = xe.dyadic_product(S, xe.TTTensor(xe.Tensor.from_ndarray(e0))) + xe.dyadic_product(xe.TTTensor(xe.Tensor.from_ndarray(e1)), S)
    assert S.canonicalized and S.corePosition == 0
    expect = (np.multiply.outer(Sd, e0) + np.multiply.outer(e1, Sd)) / np.sqrt(2)
    assert approx(full(xe, S), expect, 1e-13)


# ---------------------------------------------------------------------------------------- consistency.cxx
def _dims_sequence(seed, n=6):
    rng = np.random.default_rng(seed)
    return [int(v) for v in rng.integers(1, 4, size=n)]


def test_consistency_entrywise_product(xe):
    """Consistency:entrywise_product (consistency.cxx:755-879): dense vs TT / TTOperator entrywise products,
    nested and scaled, orders 0..5, approx_equal at 1e-14."""
    dims1 = []
    extra = _dims_sequence(755)
    xe.seed(755)
    for d in range(1, 7):
        dimsX = dimsY = list(dims1)
        dimsA = dimsB = dims1 + dims1
        A, B = xe.Tensor.random(dimsA), xe.Tensor.random(dimsB)
        X, Y = xe.Tensor.random(dimsX), xe.Tensor.random(dimsY)
        ttA, ttB = xe.TTOperator(A, 0.33), xe.TTOperator(B, 0.33)
        ttX, ttY = xe.TTTensor(X, 0.33), xe.TTTensor(Y, 0.33)
        A, B, X, Y = xe.Tensor(ttA), xe.Tensor(ttB), xe.Tensor(ttX), xe.Tensor(ttY)
        a, b, x, y = A.to_ndarray(), B.to_ndarray(), X.to_ndarray(), Y.to_ndarray()
        ep = xe.entrywise_product
        assert approx(x * x, full(xe, ep(ttX, ttX)), 1e-14)
        assert approx(x * y, full(xe, ep(ttX, ttY)), 1e-14)
        assert approx(x * y * x, full(xe, ep(ep(ttX, ttY), ttX)), 1e-14)
        assert approx((3.7 * x) * y * x * (-3 * y), full(xe, ep(ep(ep(3.7 * ttX, ttY), ttX), -3 * ttY)), 1e-14)
        assert approx(a * a, full(xe, ep(ttA, ttA)), 1e-14)
        assert approx(a * b, full(xe, ep(ttA, ttB)), 1e-14)
        assert approx((3.7 * a) * b * (-1.2 * a), full(xe, ep(ep(3.7 * ttA, ttB), -1.2 * ttA)), 1e-14)
        assert np.array_equal(ep(X, Y).to_ndarray(), x * y)   # the dense product itself
        dims1.append(extra[d - 1])


def test_consistency_named_constructors(xe):
    """Consistency:named_constructors (consistency.cxx:881-938): ones, identity, kronecker and dirac (by
    position and by multi-index) as TT / TTOperator against the dense constructors, orders 0..5."""
    dims1 = []
    extra = _dims_sequence(881)
    rng = np.random.default_rng(882)
    for d in range(1, 7):
        dimsX, dimsA = list(dims1), dims1 + dims1
        assert approx(xe.Tensor.ones(dimsA).to_ndarray(), full(xe, xe.TTOperator.ones(dimsA)))
        assert approx(xe.Tensor.ones(dimsX).to_ndarray(), full(xe, xe.TTTensor.ones(dimsX)))
        assert approx(xe.Tensor.identity(dimsA).to_ndarray(), full(xe, xe.TTOperator.identity(dimsA)))
        assert approx(xe.Tensor.kronecker(dimsA).to_ndarray(), full(xe, xe.TTOperator.kronecker(dimsA)))
        assert approx(xe.Tensor.kronecker(dimsX).to_ndarray(), full(xe, xe.TTTensor.kronecker(dimsX)))
        posA = int(rng.integers(0, int(np.prod(dimsA))))
        posX = int(rng.integers(0, int(np.prod(dimsX))))
        assert approx(xe.Tensor.dirac(dimsA, posA).to_ndarray(), full(xe, xe.TTOperator.dirac(dimsA, posA)))
        assert approx(xe.Tensor.dirac(dimsX, posX).to_ndarray(), full(xe, xe.TTTensor.dirac(dimsX, posX)))
        mA, mX = xe.position_to_multiIndex(posA, dimsA), xe.position_to_multiIndex(posX, dimsX)
        assert list(mA) == (list(np.unravel_index(posA, dimsA)) if dimsA else [])
        assert approx(xe.Tensor.dirac(dimsA, mA).to_ndarray(), full(xe, xe.TTOperator.dirac(dimsA, mA)))
        assert approx(xe.Tensor.dirac(dimsX, mX).to_ndarray(), full(xe, xe.TTTensor.dirac(dimsX, mX)))
        dims1.append(extra[d - 1])


def _consistency_setup(xe, d, dims1, dims2):
    dimsX, dimsY = list(dims1), list(dims2)
    dimsA, dimsB = dims1 + dims1, dims2 + dims1
    A, B = xe.Tensor.random(dimsA), xe.Tensor.random(dimsB)
    X, Y = xe.Tensor.random(dimsX), xe.Tensor.random(dimsY)
    ttA, ttB = xe.TTOperator(A, 0.75), xe.TTOperator(B, 0.75)
    ttX, ttY = xe.TTTensor(X, 0.6), xe.TTTensor(Y, 0.6)
    return ttA, ttB, ttX, ttY, xe.Tensor(ttA), xe.Tensor(ttB), xe.Tensor(ttX), xe.Tensor(ttY)


def _consistency_products(xe, d, A, B, X, Y, ttA, ttB, ttX, ttY):
    i, j, k = xe.indices(3)
    a, b, x, y = (t.to_ndarray() for t in (A, B, X, Y))
    ttC = xe.TTTensor()
    ttC(i & 0) << ttA(i / 2, j / 2) * ttX(j & 0)
    assert approx(op_apply(a, x, d), full(xe, ttC), 1e-14)
    ttC(i & 0) << ttB(i / 2, j / 2) * ttX(j & 0)
    assert approx(op_apply(b, x, d), full(xe, ttC), 1e-14)
    ttC(j & 0) << ttY(i & 0) * ttB(i / 2, j / 2)
    assert approx(np.tensordot(y, b, axes=(list(range(d)), list(range(d)))), full(xe, ttC), 1e-14)


def test_consistency_fix_mode(xe):
    """Consistency:fix_mode (consistency.cxx:421-586): TTTensor::fix_mode against the dense fix_mode (the
    TTOperators are rebuilt from their fixed dense tensors, as in the reference), require_correct_format
    holds afterwards, then operator x tensor products of the fixed objects; orders 1..6."""
    seq1, seq2 = _dims_sequence(421), _dims_sequence(422)
    rng = np.random.default_rng(423)
    xe.seed(421)
    dims1, dims2 = [], []
    for d in range(1, 7):
        dims1.append(seq1[d - 1])
        dims2.append(seq2[d - 1])
        ttA, ttB, ttX, ttY, A, B, X, Y = _consistency_setup(xe, d, dims1, dims2)
        slate = int(rng.integers(0, d))
        pX, pY = int(rng.integers(0, dims1[slate])), int(rng.integers(0, dims2[slate]))
        A.fix_mode(slate + d, pX)
        A.fix_mode(slate, pX)
        B.fix_mode(slate + d, pX)
        B.fix_mode(slate, pY)
        X.fix_mode(slate, pX)
        Y.fix_mode(slate, pY)
        ttA, ttB = xe.TTOperator(A), xe.TTOperator(B)   # (TTOperator::fix_mode is not available)
        with pytest.raises(Exception):
            xe.TTOperator(A).fix_mode(0, 0)
        ttX.fix_mode(slate, pX)
        ttY.fix_mode(slate, pY)
        ttX.require_correct_format()
        ttY.require_correct_format()
        assert approx(A.to_ndarray(), full(xe, ttA), 1e-14)
        assert approx(B.to_ndarray(), full(xe, ttB), 1e-14)
        assert approx(X.to_ndarray(), full(xe, ttX), 1e-14)
        assert approx(Y.to_ndarray(), full(xe, ttY), 1e-14)
        if d > 1:
            _consistency_products(xe, d - 1, A, B, X, Y, ttA, ttB, ttX, ttY)


def test_consistency_resize_mode(xe):
    """Consistency:resize_mode (consistency.cxx:588-753): resize_mode of TTTensor / TTOperator modes (grow or
    cut at a position) against the dense resize_mode, then operator x tensor products; orders 1..6."""
    seq1, seq2 = _dims_sequence(588), _dims_sequence(589)
    rng = np.random.default_rng(590)
    xe.seed(588)
    dims1, dims2 = [], []
    for d in range(1, 7):
        dims1.append(seq1[d - 1])
        dims2.append(seq2[d - 1])
        ttA, ttB, ttX, ttY, A, B, X, Y = _consistency_setup(xe, d, dims1, dims2)
        dim = int(rng.integers(0, d))
        n1, n2 = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        p1 = int(rng.integers(dims1[dim] - min(n1, dims1[dim]), dims1[dim] + 1))
        p2 = int(rng.integers(dims2[dim] - min(n2, dims2[dim]), dims2[dim] + 1))
        for T in (A, ttA):
            T.resize_mode(dim + d, n1, p1)
            T.resize_mode(dim, n1, p1)
        for T in (B, ttB):
            T.resize_mode(dim + d, n1, p1)
            T.resize_mode(dim, n2, p2)
        X.resize_mode(dim, n1, p1)
        ttX.resize_mode(dim, n1, p1)
        Y.resize_mode(dim, n2, p2)
        ttY.resize_mode(dim, n2, p2)
        for T in (ttA, ttB, ttX, ttY):
            T.require_correct_format()
        assert approx(A.to_ndarray(), full(xe, ttA), 1e-14)
        assert approx(B.to_ndarray(), full(xe, ttB), 1e-14)
        assert approx(X.to_ndarray(), full(xe, ttX), 1e-14)
        assert approx(Y.to_ndarray(), full(xe, ttY), 1e-14)
        _consistency_products(xe, d, A, B, X, Y, ttA, ttB, ttX, ttY)


def test_entrywise_product_feeds_round(xe):
    """The entrywise product is the canonical input of round() (rank r^2): (x o x).round(r^2) keeps the tensor,
    a truncating round matches the oracle's truncation error of the same product cores."""
    from oracle import xerus_ref as ref
    from ttutil import tt_diff_norm

    xe.seed(1209)
    x = xe.TTTensor.random([6] * 6, [5] * 5)
    y = xe.TTTensor.random([6] * 6, [4] * 5)
    z = xe.entrywise_product(x, y)
    assert z.ranks() == xe.TTTensor.reduce_to_maximal_ranks([20] * 5, [6] * 6)   # (canonical inputs: moved to core 0)
    zc = [z.get_component(k).to_ndarray() for k in range(6)]
    zz = xe.TTTensor(z)
    zz.round(8)
    o = ref.TT([c.copy() for c in zc])
    o.round(8)
    assert zz.ranks() == o.ranks
    e_gpu, nrm = tt_diff_norm([zz.get_component(k).to_ndarray() for k in range(6)], zc)
    e_ref, _ = tt_diff_norm(o.cores, zc)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm
