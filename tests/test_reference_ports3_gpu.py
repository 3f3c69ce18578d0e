"""Ports of the reference's TensorNetwork and Consistency unit tests (src/unitTests/tensorNetwork.cxx,
consistency.cxx) through the Python binding of the C++ host API, with the reference's values and tolerances.

The reference runs several of these on lazy TensorNetwork objects and sparse copies. Sparse tensors are out
of scope and the binding's TensorNetwork holds results, not index expressions, so each
expression is evaluated on dense Tensors: the same indexed-expression machinery (the contraction-order
heuristic of network.cpp, the traces, fixed indices and index spans), the same expected values.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def approx(a, b, eps):
    a, b = np.asarray(a), np.asarray(b)
    return np.linalg.norm(a - b) <= eps * (np.linalg.norm(a) + np.linalg.norm(b)) / 2


def entrywise(res, want, eps=4 * np.finfo(float).eps):
    """misc::approx_entrywise_equal(Tensor, vector) (tensor.cpp): each entry within eps relative"""
    got = res.to_ndarray().ravel()
    want = np.asarray(want, dtype=float)
    return got.size == want.size and bool(np.all(np.abs(got - want) <= eps * np.maximum(np.abs(got), np.abs(want)) + 0.0))


def filled(xe, dims):
    """the reference's hand-filled tensors: entry k of the row-major order = 2^k"""
    size = int(np.prod(dims))
    return xe.Tensor.from_ndarray((2.0 ** np.arange(size)).reshape(dims))


def test_traces(xe):
    """TensorNetwork:traces (tensorNetwork.cxx:68-150): traces, partial traces and fixed indices in products of
    2x2, 2x2x2 and 2x2x2x2 tensors (entries 2^k), every expected value of the reference."""
    A, B, C = filled(xe, [2, 2]), filled(xe, [2, 2, 2]), filled(xe, [2, 2, 2, 2])
    sA, sB, sC = (xe.Tensor.from_ndarray(T.to_ndarray()) for T in (A, B, C))   # (the reference's sparse copies)
    i, j, k, l, p = xe.indices(5)
    res = xe.Tensor()
    res() << A(i, i) * sA(j, j)
    assert entrywise(res, [9 * 9])
    res(j) << B(i, i, j) * sA(k, k)
    assert entrywise(res, [9 * 65, 9 * 130])
    res(j) << sB(i, j, i) * A(k, k)
    assert entrywise(res, [9 * 33, 9 * 132])
    res() << B(j, i, i) * sB(k, k, j)
    assert entrywise(res, [9 * 65 + 144 * 130])
    res(j, k) << C(i, i, j, k) * sA(l, l)
    assert entrywise(res, [4097 * 9, 8194 * 9, 16388 * 9, 32776 * 9])
    res(j, k) << sC(i, j, i, k) * sA(l, l)
    assert entrywise(res, [1025 * 9, 2050 * 9, 16400 * 9, 32800 * 9])
    res(p, k, j) << sB(l, p, l) * C(i, j, i, k)
    assert entrywise(res, [33 * 1025, 33 * 16400, 33 * 2050, 33 * 32800, 132 * 1025, 132 * 16400, 132 * 2050, 132 * 32800])
    res(p, k, j) << B(l, p, l) * sC(j, i, i, k)
    assert entrywise(res, [33 * 65, 33 * 16640, 33 * 130, 33 * 33280, 132 * 65, 132 * 16640, 132 * 130, 132 * 33280])
    res(p, k, j) << sB(l, p, l) * C(j, i, k, i)
    assert entrywise(res, [33 * 33, 33 * 8448, 33 * 132, 33 * 33792, 132 * 33, 132 * 8448, 132 * 132, 132 * 33792])
    res(k) << sB(l, l, 1) * C(0, k, i, i)
    assert entrywise(res, [130 * 9, 130 * 144])
    res(k) << B(l, l, 0) * sC(1, k, i, i)
    assert entrywise(res, [65 * 2304, 65 * 36864])
    res(j) << sB(l, l, 0) * C(j, 0, i, i)
    assert entrywise(res, [65 * 9, 65 * 2304])
    res(j) << sB(l, l, 1) * sC(j, 1, i, i)
    assert entrywise(res, [130 * 144, 130 * 36864])
    res() << C(i, i, j, j) * sA(k, k)
    assert entrywise(res, [(1 + 8 + 4096 + 32768) * 9])
    res() << C(i, j, i, j) * sA(k, k)
    assert entrywise(res, [(1 + 32 + 1024 + 32768) * 9])
    res() << C(i, j, j, i) * sA(k, k)
    assert entrywise(res, [(1 + 64 + 512 + 32768) * 9])


def test_contraction_single_node_trace(xe):
    """TensorNetwork:contraction_single_node_trace (tensorNetwork.cxx:152-160): E() = A(i1,i2,i2) * B(i1)
    with a size-1 mode is a normal number (and equals the dense trace)."""
    xe.seed(152)
    A, B = xe.Tensor.random([1, 10, 10]), xe.Tensor.random([1])
    i1, i2 = xe.indices(2)
    E = xe.Tensor()
    E() << A(i1, i2, i2) * B(i1)
    v = E[0]
    assert np.isfinite(v) and v != 0.0
    want = np.einsum("aii,a->", A.to_ndarray(), B.to_ndarray())
    assert abs(v - want) <= 1e-14 * (abs(want) + np.abs(A.to_ndarray()).sum())


def test_contraction_single_network_trace(xe):
    """TensorNetwork:contraction_single_network_trace (tensorNetwork.cxx:162-175): the double trace
    ATN(i1,i1,i2,i2) of a 2x2x2x2 tensor, once into a network converted to a Tensor, once into a Tensor."""
    xe.seed(162)
    A = xe.Tensor.random([2, 2, 2, 2])
    i1, i2 = xe.indices(2)
    E = xe.Tensor()
    E() << A(i1, i1, i2, i2)
    want = np.einsum("iijj->", A.to_ndarray())
    assert np.isfinite(E[0]) and E[0] != 0.0
    assert abs(E[0] - want) <= 1e-14 * np.abs(A.to_ndarray()).sum()
    E2 = xe.TensorNetwork(E).to_tensor()
    assert E2[0] == E[0]


def test_index_reshuffle2(xe):
    """TensorNetwork:index_reshuffle2 (tensorNetwork.cxx:177-191): spans n^(1), n^(2) around a contraction
    over a size-1 rank mode; the result modes are ordered as the left-hand side says."""
    n1, n2, n3, n4, r1, r2 = xe.indices(6)
    A = xe.Tensor.from_ndarray(np.arange(6, dtype=float).reshape(2, 1, 3) + 1)
    B = xe.Tensor.from_ndarray(np.arange(20, dtype=float).reshape(1, 4, 5, 1) + 1)
    R = xe.Tensor()
    R(n1 ^ 1, n2, r2, n3 ^ 1, n4) << A(n1 ^ 1, r1, n3 ^ 1) * B(r1, n2, n4, r2)
    assert list(R.dimensions) == [2, 4, 1, 3, 5]
    want = np.einsum("arc,rbds->abscd", A.to_ndarray(), B.to_ndarray())
    assert np.allclose(R.to_ndarray(), want, rtol=1e-15, atol=0)
    B2 = xe.Tensor.from_ndarray(np.arange(42, dtype=float).reshape(1, 6, 7, 1) + 1)
    R2 = xe.Tensor()
    R2(n1 ^ 2, n2, r2, n3 ^ 2, n4) << R(n1 ^ 2, r1, n3 ^ 2) * B2(r1, n2, n4, r2)
    assert list(R2.dimensions) == [2, 4, 6, 1, 3, 5, 7]


@pytest.mark.parametrize("case", range(10))
def test_triple_indices(xe, case):
    """TensorNetwork:triple_indices (tensorNetwork.cxx:193-218): an index appearing three times in a product
    is an error (FAILTEST), whatever the left-hand side."""
    A = xe.Tensor.random([2, 2, 2])
    B, C, D, F = (xe.Tensor.random([2, 2]) for _ in range(4))
    i1, i2, i3, i4 = xe.indices(4)
    E = xe.Tensor()
    exprs = [
        lambda: E() << A(i1, i1, i2) * B(i2, i2),
        lambda: E(i2) << A(i1, i1, i2) * B(i2, i2),
        lambda: E() << A(i1, i2, i2) * B(i2, i1),
        lambda: E(i2) << A(i1, i2, i2) * B(i2, i1),
        lambda: E() << A(i2, i2, i2) * B(i1, i1),
        lambda: E(i2) << A(i2, i2, i2) * B(i1, i1),
        lambda: E() << A(i1, i2, i2) * B(i1, i3) * C(i3, i2),
        lambda: E() << B(i1, i2) * C(i2, i3) * D(i3, i2),
        lambda: E() << B(i1, i2) * C(i2, i3) * D(i1, i2),
        lambda: E() << B(i1, i2) * C(i2, i3) * D(i3, i4) * F(i4, i2),
    ]
    with pytest.raises(RuntimeError):
        exprs[case]()


def test_contraction_multi_node_trace_and_reshuffle(xe):
    """TensorNetwork:contraction_multi_node_trace / index_reshuffle (tensorNetwork.cxx:220-243): the outer
    product of two 1x10 tensors traced over (i1,i1),(i2,i2), directly and after a mode reshuffle."""
    xe.seed(220)
    A, B = xe.Tensor.random([1, 10]), xe.Tensor.random([1, 10])
    i1, i2, i3, i4 = xe.indices(4)
    tmp = xe.Tensor()
    tmp(i1, i2, i3, i4) << A(i1, i3) * B(i2, i4)
    E = xe.Tensor()
    E() << tmp(i1, i1, i2, i2)
    assert np.isfinite(E[0]) and E[0] != 0.0
    want = np.einsum("iijj->", np.einsum("ac,bd->abcd", A.to_ndarray(), B.to_ndarray()))
    assert abs(E[0] - want) <= 1e-13 * abs(want)
    tmp2 = xe.Tensor()
    tmp2(i1, i2, i3, i4) << tmp(i3, i4, i1, i2)
    E() << tmp2(i1, i1, i2, i2)
    assert np.isfinite(E[0]) and E[0] != 0.0


def test_save_network(xe):
    """TensorNetwork:Save_Network (tensorNetwork.cxx:245-317): chains of 2x2 matrices 1..24 contracted in
    several index layouts, all equal to {20596523, 21531582, 46728183, 48849590}."""
    mats = [xe.Tensor.from_ndarray(np.arange(4 * q + 1, 4 * q + 5, dtype=float).reshape(2, 2)) for q in range(6)]
    A, B, C, D, E, F = mats
    i, j, k, l, m, n, o = xe.indices(7)
    want = [20596523, 21531582, 46728183, 48849590]
    res1, res2, res3 = xe.Tensor(), xe.Tensor(), xe.Tensor()
    res2(i, l) << A(i, j) * B(j, k) * C(k, l)
    res1 = xe.Tensor.from_ndarray(res2.to_ndarray())
    res2(l, o) << D(l, m) * E(m, n) * F(n, o)
    res3(i, o) << res1(i, l) * res2(l, o)
    assert entrywise(res3, want)
    r1A, r2A = xe.Tensor(), xe.Tensor()
    for _ in range(2):
        r1A(i, j, m, n, k, l) << A(i, j) * E(m, n) * C(k, l)
        r2A(l, m, j, k, n, o) << D(l, m) * B(j, k) * F(n, o)
        res3(i, o) << r1A(i, j, m, n, k, l) * r2A(l, m, j, k, n, o)
        assert entrywise(res3, want)
    for _ in range(2):
        r1A(i, l, m, n, j, k) << A(i, j) * E(m, n) * C(k, l)
        r2A(l, o, m, n, j, k) << D(l, m) * B(j, k) * F(n, o)
        res3(i, o) << r1A(i, l, m, n, j, k) * r2A(l, o, m, n, j, k)
        assert entrywise(res3, want)


def _grow(rng, lo, hi):
    return int(rng.integers(lo, hi + 1))


def test_consistency_sum_and_difference(xe):
    """Consistency:sum_and_difference (consistency.cxx:29-166): TT-SVDs (eps 0.2) of random tensors and
    operators of orders 0..6 equal their dense conversions; sums, differences and scaled combinations of TT
    tensors / operators equal the dense ones to 1e-14."""
    rng = np.random.default_rng(29)
    xe.seed(29)
    dims1 = []
    for d in range(7):
        dimsX, dimsA = list(dims1), dims1 + dims1
        X, Y = xe.Tensor.random(dimsX), xe.Tensor.random(dimsX)
        A, B = xe.Tensor.random(dimsA), xe.Tensor.random(dimsA)
        ttX, ttY = xe.TTTensor(X, 0.2), xe.TTTensor(Y, 0.2)
        ttA, ttB = xe.TTOperator(A, 0.2), xe.TTOperator(B, 0.2)
        X, Y, A, B = (xe.Tensor(t).to_ndarray() for t in (ttX, ttY, ttA, ttB))
        full = lambda t: xe.Tensor(t).to_ndarray()  # noqa: E731
        for dense, tt in ((X + X, ttX + ttX), (X + Y, ttX + ttY), (X - Y, ttX - ttY), (X + Y + X, ttX + ttY + ttX),
                          (3.7 * X + Y + X - 3 * Y, 3.7 * ttX + ttY + ttX - 3 * ttY)):
            assert approx(dense, full(tt), 1e-14), d
        for dense, tt in ((A + A, ttA + ttA), (A + B, ttA + ttB), (A - B, ttA - ttB),
                          (3.7 * A + B - 1.2 * A, 3.7 * ttA + ttB - 1.2 * ttA)):
            assert approx(dense, full(tt), 1e-14), d
        dims1.append(_grow(rng, 1, 3))


def test_consistency_fixed_indices(xe):
    """Consistency:fixed_indices (consistency.cxx:169-290), dense part: X(0, i&2, 1) + X(0, i&2, 0) and
    X(0, i&2, 1) * X(0, i&2, 0) (entrywise over the spanned middle modes) against numpy, and the operator
    chain B(k/2, 1, j^(d-2), 0) * A(0, j^(d-2), 0, i/2) * X(i&0) with fixed indices inside both operators,
    orders 2..6 (dims 2..3)."""
    rng = np.random.default_rng(169)
    xe.seed(169)
    dims1 = [_grow(rng, 2, 3), _grow(rng, 2, 3)]
    dims2 = [_grow(rng, 2, 3), _grow(rng, 2, 3)]
    i, j, k = xe.indices(3)
    for d in range(2, 7):
        X = xe.Tensor.from_ndarray(xe.Tensor(xe.TTTensor(xe.Tensor.random(dims1), 0.6)).to_ndarray())
        A = xe.Tensor.from_ndarray(xe.Tensor(xe.TTOperator(xe.Tensor.random(dims1 + dims1), 0.75)).to_ndarray())
        B = xe.Tensor.from_ndarray(xe.Tensor(xe.TTOperator(xe.Tensor.random(dims2 + dims1), 0.75)).to_ndarray())
        x, a, b = X.to_ndarray(), A.to_ndarray(), B.to_ndarray()
        C = xe.Tensor()
        C(i & 0) << X(0, i & 2, 1) + X(0, i & 2, 0)
        assert approx(C.to_ndarray(), x[0, ..., 1] + x[0, ..., 0], 1e-14), d
        C(i & 0) << X(0, i & 2, 1) * X(0, i & 2, 0)
        want = np.tensordot(x[0, ..., 1], x[0, ..., 0], axes=d - 2) if d > 2 else x[0, 1] * x[0, 0]
        assert approx(C.to_ndarray(), want, 1e-14), d
        C(k & 0) << B(k / 2, 1, j ^ (d - 2), 0) * A(0, j ^ (d - 2), 0, i / 2) * X(i & 0)
        bb = b[(slice(None),) * d + (1,) + (slice(None),) * (d - 2) + (0,)]      # k/2 (d modes), j^(d-2)
        aa = a[(0,) + (slice(None),) * (d - 2) + (0,) + (slice(None),) * d]      # j^(d-2), i/2 (d modes)
        t = np.tensordot(aa, x, axes=d)                                            # j^(d-2)
        want = np.tensordot(bb, t, axes=d - 2) if d > 2 else bb * t
        assert approx(C.to_ndarray(), want, 1e-13), d
        dims1.append(_grow(rng, 2, 3))
        dims2.append(_grow(rng, 2, 3))


def test_consistency_operator_times_tensor(xe):
    """Consistency:operator_times_tensor (consistency.cxx:293-419): A x, B x, y^T B and B A x for TT operators
    (TT-SVD eps 0.75) and TT tensors (eps 0.6) of orders 0..6 equal the dense products to 1e-14 (the
    three-factor product as two TT products)."""
    rng = np.random.default_rng(293)
    xe.seed(293)
    dims1, dims2 = [], []
    i, j, k = xe.indices(3)
    for d in range(7):
        ttA = xe.TTOperator(xe.Tensor.random(dims1 + dims1), 0.75)
        ttB = xe.TTOperator(xe.Tensor.random(dims2 + dims1), 0.75)
        ttX = xe.TTTensor(xe.Tensor.random(dims1), 0.6)
        ttY = xe.TTTensor(xe.Tensor.random(dims2), 0.6)
        A, B, X, Y = (xe.Tensor(t) for t in (ttA, ttB, ttX, ttY))
        for lhs_dense, rhs_dense, tt in (((A, X), None, (ttA, ttX)), ((B, X), None, (ttB, ttX))):
            C = xe.Tensor()
            C(i & 0) << lhs_dense[0](i / 2, j / 2) * lhs_dense[1](j & 0)
            ttC = xe.TTTensor()
            ttC(i & 0) << tt[0](i / 2, j / 2) * tt[1](j & 0)
            assert approx(C.to_ndarray(), xe.Tensor(ttC).to_ndarray(), 1e-14), d
        C = xe.Tensor()
        C(j & 0) << B(i / 2, j / 2) * Y(i & 0)
        ttC = xe.TTTensor()
        ttC(j & 0) << ttY(i & 0) * ttB(i / 2, j / 2)
        assert approx(C.to_ndarray(), xe.Tensor(ttC).to_ndarray(), 1e-14), d
        C(k & 0) << B(k / 2, i / 2) * A(i / 2, j / 2) * X(j & 0)
        ttAX = xe.TTTensor()
        ttAX(i & 0) << ttA(i / 2, j / 2) * ttX(j & 0)
        ttC = xe.TTTensor()
        ttC(k & 0) << ttB(k / 2, i / 2) * ttAX(i & 0)
        assert approx(C.to_ndarray(), xe.Tensor(ttC).to_ndarray(), 1e-14), d
        dims1.append(_grow(rng, 1, 3))
        dims2.append(_grow(rng, 1, 3))
