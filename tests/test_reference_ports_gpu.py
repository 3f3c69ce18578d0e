"""The reference's own unit tests for the hot path, re-expressed against the MI355X build.

Each test names the reference test it ports (src/unitTests/*.cxx:line) and keeps its inputs, operations
and tolerances; the reference's indexed assignments `B(i) = TT(i)` / `ttC(i&0) = ttA(i&0) + ttB(i&0)`
are written with the Python module's equivalents (Tensor(tt), tt + tt). Runs through the C++ host API
(xerus_amd.xerus), i.e. the HIP kernels behind the C-ABI.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _approx_equal(a, b, eps):
    """approx_equal (tensor.cpp:1738-1743): ||a-b|| <= eps (||a|| + ||b||) / 2."""
    return np.linalg.norm(a - b) <= eps * (np.linalg.norm(a) + np.linalg.norm(b)) / 2


def _dense(xe, tt):
    return xe.Tensor(tt).to_ndarray()


def test_product_1000x1000_bitexact(xe, handle):
    """Tensor:Product_1000x1000 (fullTensor_product.cxx:400-418): the expression engine emits exactly one
    GEMM with the reference's transpose flags -- memcmp-equal to a direct xrs_gemm call."""
    from xerus_amd import capi

    n = 1000
    ii, jj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    A = (ii + jj).astype(np.float64)
    B = ((n - ii) * (n - jj)).astype(np.float64)
    tA, tB = xe.Tensor.from_ndarray(A), xe.Tensor.from_ndarray(B)
    dA, dB = handle.array(A), handle.array(B)
    i, J, K = xe.indices(3)
    for ta, tb, lhs, rhs in [(False, False, (i, J), (J, K)), (False, True, (i, J), (K, J)), (True, True, (J, i), (K, J))]:
        C = handle.empty((n, n))
        handle.gemm(C, n, n, 1.0, dA, n, ta, n, dB, n, tb)
        res = xe.Tensor()
        res(i, K) << tA(*lhs) * tB(*rhs)
        got, want = res.to_ndarray(), C.numpy()
        assert got.tobytes() == want.tobytes(), (ta, tb, np.abs(got - want).max())


def test_tt_rounding(xe):
    """TT:TTTensor_Rounding (ttRounding.cxx:27-103): TT-SVD with eps 1e-14, round(1e-14) (the eps-only
    overload) and round(maxRank) reproduce the dense tensor to 1e-14, incl. an order-8 2^8 tensor and
    one with unit modes."""
    cases = [([2], 1), ([2, 2], 2), ([2, 7], 2), ([2] * 8, 512), ([5, 6, 3, 1, 4, 2, 8, 1], 576)]
    for dims, max_rank in cases:
        A = xe.Tensor.random(dims)
        a = A.to_ndarray()
        tt = xe.TTTensor(A, 1e-14)
        assert _approx_equal(_dense(xe, tt), a, 1e-14), dims
        tt.round(1e-14)
        assert _approx_equal(_dense(xe, tt), a, 1e-14), dims
        tt.round(max_rank)
        assert _approx_equal(_dense(xe, tt), a, 1e-14), dims


def test_tt_no_rounding(xe):
    """TT:no_rounding (ttRounding.cxx:106-117): round(2) of a rank-2 TT is the identity; a + 0.0*c has
    rank 4 and round(2) recovers the rank-2 tensor to 1e-14."""
    dims, ranks = [2] * 7, [2] * 6
    a = xe.TTTensor.random(dims, ranks)
    b = a.__copy__()
    a.round(2)
    assert _approx_equal(_dense(xe, a), _dense(xe, b), xe.EPSILON)
    c = xe.TTTensor.random(dims, ranks)
    a = a + 0.0 * c
    a.round(2)
    assert a.ranks() == ranks
    assert _approx_equal(_dense(xe, a), _dense(xe, b), 1e-14)


def test_tt_special_sum_diff(xe):
    """TT:special_sum_diff (ttArithmetic.cxx:143-200): sums and differences with the zero TT, order 4 and
    order 1, against the dense results (absolute Frobenius bounds of the reference)."""
    for dims, tol_sum, tol_b in [([10, 10, 10, 10], 5e-13, 3.1e-13), ([10], 3.1e-13, 3.1e-13)]:
        A = xe.Tensor(dims)              # the zero tensor
        B = xe.Tensor.random(dims)
        a, b = A.to_ndarray(), B.to_ndarray()
        ttA, ttB = xe.TTTensor(A), xe.TTTensor(B)
        dB = _dense(xe, ttB)
        for ttC, C, Bexp in [(ttA + ttB, a + b, dB), (ttB + ttA, b + a, dB), (ttA - ttB, a - b, -dB), (ttB - ttA, b - a, dB)]:
            got = _dense(xe, ttC)
            assert np.linalg.norm(got - C) < tol_sum
            assert np.linalg.norm(got - Bexp) < tol_b


def test_tt_full_contraction(xe):
    """TT:full_contraction (ttArithmetic.cxx:408-433), TTTensor part: frob norms and the full contraction
    value_t(ttA(i&0) * ttB(i&0)) against the dense tensors."""
    A, B = xe.Tensor.random([10] * 4), xe.Tensor.random([10] * 4)
    a, b = A.to_ndarray(), B.to_ndarray()
    ttA, ttB = xe.TTTensor(A), xe.TTTensor(B)
    i = xe.Index()

    def close(x, y, eps):   # misc::approx_equal on scalars
        return abs(x - y) <= eps * (abs(x) + abs(y)) / 2

    assert close(np.linalg.norm(a), xe.frob_norm(ttA), 3e-13)
    assert close(np.linalg.norm(b), xe.frob_norm(ttB), 2e-13)
    assert close(np.linalg.norm(a - b), xe.frob_norm(ttA - ttB), 1e-12)
    C = float(A(i / 1) * B(i & 0))
    ttC = float(ttA(i & 0) * ttB(i & 0))
    assert close(C, ttC, 1e-12)
    assert close(C, float(np.sum(a * b)), 1e-12)


def test_tt_dot_generic_network_order12(xe, ref):
    """value_t(x(i&0) * y(i&0)) contracted as the reference does it -- the 28-node TensorNetwork in the
    heuristics' order (tests/test_contraction_order_cpu.py pins that order), one permutation + GEMM per
    pair -- agrees with the zipper and with the oracle at the cfg4 shape (order 12, n 20, rank 256)."""
    dims, ranks = [20] * 12, [256] * 11
    rng = ref.Rng(47)
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    tx, ty = xe.TTTensor(len(dims)), xe.TTTensor(len(dims))
    for k in range(len(dims)):
        tx.set_component(k, xe.Tensor.from_ndarray(x.cores[k]))
        ty.set_component(k, xe.Tensor.from_ndarray(y.cores[k]))
    want = ref.dot(x, y)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    net = xe.tt_dot_network(tx, ty)
    zip_ = xe.dot(tx, ty)
    assert abs(net - want) <= 1e-12 * nx * ny
    assert abs(zip_ - want) <= 1e-12 * nx * ny


def _approx(a, b, eps=4 * np.finfo(float).eps):
    """misc::approx_equal (include/xerus/misc/math.h:71-73)."""
    return abs(a - b) <= eps * 0.5 * (abs(a) + abs(b))


def test_contractions_of_4_to_degree_0(xe):
    """TensorNetwork:contractions_of_4_to_degree_0 (tensorNetwork.cxx:27-46): the ring A-D, B-C closed over
    two size-1 links contracts to (A.D)(B.C) in every factor order, to 1e-20 (the same contraction order
    is found whatever order the factors are written in)."""
    xe.seed(0xBAADF00D)
    A, B, C, D = (xe.Tensor.random([100, 1]) for _ in range(4))
    E = xe.Tensor()
    i1, i2, i3, i4 = xe.indices(4)
    E() << A(i1, i2) * D(i1, i2)
    a1 = E[0]
    E() << B(i3, i4) * C(i3, i4)
    a2 = E[0]
    E() << A(i1, i2) * B(i3, i2) * C(i3, i4) * D(i1, i4)
    assert _approx(E[0], a1 * a2, 1e-20)
    E() << B(i3, i2) * C(i3, i4) * D(i1, i4) * A(i1, i2)
    assert _approx(E[0], a1 * a2, 1e-20)
    E() << B(i3, i2) * D(i1, i4) * C(i3, i4) * A(i1, i2)
    assert _approx(E[0], a1 * a2, 1e-20)


def test_contractions_of_3_to_degree_0(xe):
    """TensorNetwork:contractions_of_3_to_degree_0 (tensorNetwork.cxx:48-66): a closed 3-ring in three
    factor orders (the 3-node closed-form order, tensorNetwork.cpp:1269-1313), equal to 4 eps."""
    xe.seed(0xBAADF00D)
    A = xe.Tensor.random([1, 10])
    B = xe.Tensor.random([10, 100])
    C = xe.Tensor.random([100, 1])
    assert B.is_dense()
    E = xe.Tensor()
    i1, i2, i3 = xe.indices(3)
    E() << A(i1, i2) * B(i2, i3) * C(i3, i1)
    a1 = E[0]
    E() << B(i2, i3) * C(i3, i1) * A(i1, i2)
    a2 = E[0]
    E() << C(i3, i1) * B(i2, i3) * A(i1, i2)
    a3 = E[0]
    assert _approx(a1, a2)
    assert _approx(a2, a3)
    want = float((A.to_ndarray() @ B.to_ndarray() @ C.to_ndarray())[0, 0])
    assert abs(a1 - want) <= 1e-13 * np.sqrt(100 * 10)
