"""Ports of the reference's dense-Tensor unit tests (src/unitTests/fullTensor_add_sub.cxx, fullTensor_arithmetic.cxx,
fullTensor_factor.cxx, fullTensor_utilities.cxx, fullTensor_solve.cxx, tensor.cxx) through the Python binding of the
C++ host API, with the reference's values and tolerances. (fullTensor_product / _trace / _assignment are the
golden known-answer cases of tests/golden/known_products.json, run by test_api_gpu.py.) Sparse legs are out of
scope; Tensor::modify_diagonal_entries (a host callback) is not part of the binding.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def T(xe, arr):
    return xe.Tensor.from_ndarray(np.require(np.asarray(arr, dtype=np.float64), requirements="C"))


def entrywise(res, want, eps=4 * np.finfo(float).eps):
    """misc::approx_entrywise_equal(Tensor, vector): every entry within eps relative"""
    got = res.to_ndarray().ravel()
    want = np.asarray(want, dtype=float).ravel()
    return got.size == want.size and bool(np.all(np.abs(got - want) <= eps * np.maximum(np.abs(got), np.abs(want))))


def approx(a, b, eps):
    a, b = np.asarray(a), np.asarray(b)
    return np.linalg.norm(a - b) <= eps * (np.linalg.norm(a) + np.linalg.norm(b)) / 2


# ------------------------------------------------------------------------------------ fullTensor_add_sub.cxx
def test_sum_matrix_2x2(xe):
    """Tensor:sum_matrix_2x2 (fullTensor_add_sub.cxx:29-49)"""
    B, C = T(xe, [[1, 2], [3, 4]]), T(xe, [[5, 6], [7, 8]])
    i, J = xe.indices(2)
    res = xe.Tensor([2, 2])
    res(i, J) << B(i, J) + C(i, J)
    assert entrywise(res, [6, 8, 10, 12])
    res(i, J) << B(i, J) + C(J, i)
    assert entrywise(res, [6, 9, 9, 12])


def test_sum_lhs_equals_rhs(xe):
    """Tensor:sum_lhs_equals_rhs (fullTensor_add_sub.cxx:51-71): B(i,J) = B(i,J) + C(i,J), then B + B^T"""
    B, C = T(xe, [[1, 2], [3, 4]]), T(xe, [[5, 6], [7, 8]])
    i, J = xe.indices(2)
    B(i, J) << B(i, J) + C(i, J)
    assert entrywise(B, [6, 8, 10, 12])
    B(i, J) << B(i, J) + B(J, i)
    assert entrywise(B, [12, 18, 18, 24])


def test_sum_matrix_1024(xe):
    """Tensor:sum_matrix_1000x1000 (fullTensor_add_sub.cxx:73-92): 1024^2 index-function tensors, sums in both
    orders to 1e-14"""
    a = np.add.outer(np.arange(1024.0), np.arange(1024.0))
    b = np.multiply.outer(np.arange(1024.0), np.arange(1024.0))
    A, B, C = T(xe, a), T(xe, b), T(xe, a + b)
    i, J = xe.indices(2)
    res = xe.Tensor([1024, 1024])
    res(i, J) << A(i, J) + B(i, J)
    assert approx(res.to_ndarray(), C.to_ndarray(), 1e-14)
    res(J, i) << A(J, i) + B(i, J)
    assert approx(res.to_ndarray(), (a + b.T).T, 1e-14)   # res(J,i) = A(J,i) + B(i,J): res^T = A^T + B
    assert approx(res.to_ndarray(), C.to_ndarray(), 1e-14)   # (A, B symmetric: the reference's own check)


def test_sum_dyadic_fails(xe):
    """Tensor:sum_dyadic (fullTensor_add_sub.cxx:94-109): B(i) + C(J) into res(i,J) is an error (FAILTEST)"""
    B, C = T(xe, [1, 2]), T(xe, [5, 9])
    i, J = xe.indices(2)
    res = xe.Tensor([2, 2])
    with pytest.raises(RuntimeError):
        res(i, J) << B(i) + C(J)


def test_sum_threefold(xe):
    """Tensor:sum_threefold_sum (fullTensor_add_sub.cxx:111-131)"""
    B, C, D = T(xe, [1, 2]), T(xe, [5, 9]), T(xe, [7, 13])
    (i,) = xe.indices(1)
    res = xe.Tensor([2])
    res(i) << B(i) + C(i) + D(i)
    assert entrywise(res, [13, 24])


# --------------------------------------------------------------------------------- fullTensor_arithmetic.cxx
@pytest.mark.parametrize("case", range(8))
def test_arithmetic_negatives(xe, case):
    """Tensor:Arithmetic_Negatives (fullTensor_arithmetic.cxx:25-43): mismatched dimensions / spans in products
    and sums are errors (FAILTEST)"""
    B = xe.Tensor([2, 2])
    B2, B3, B4, B5 = xe.Tensor([3, 3]), xe.Tensor([3, 2]), xe.Tensor([2, 3]), xe.Tensor([2, 2, 2])
    C = xe.Tensor([2])
    i, j = xe.indices(2)
    exprs = [lambda: C(i) << B(i, j) * B2(j, j), lambda: C(i) << B(i, j) * B3(j, j),
             lambda: C(i) << B(i, j) * B4(j, j), lambda: C(i) << B(i, j) * B5(j, j, j),
             lambda: B(i, j) << B(i, j) + B2(j, j), lambda: B(i, j) << B(i, j) + B3(j, j),
             lambda: B(i, j) << B(i, j) + B4(j, j), lambda: B(i, j) << B(i, j) + B5(j, j, j)]
    with pytest.raises(RuntimeError):
        exprs[case]()


# ------------------------------------------------------------------------------------- fullTensor_factor.cxx
def test_factors(xe):
    """Tensor:Factors (fullTensor_factor.cxx:25-55): lazy scalar factors through SVD and QR of 3 A / 7 B"""
    xe.seed(25)
    A = xe.Tensor.random([2, 7, 5, 5, 2, 7])
    B = xe.Tensor.random([2, 7, 5, 5, 2, 7])
    A3, B7 = 3 * A, 7 * B
    assert not A.has_factor() and not B.has_factor()
    assert A3.has_factor() and B7.has_factor()
    i, j, k, l, m, n, o, p, r = xe.indices(9)
    res1, res2, res3, res4 = xe.Tensor(), xe.Tensor(), xe.Tensor(), xe.Tensor()
    (res1(i, j, k, o), res2(o, p), res3(p, l, m, n)) << xe.SVD(A3(i, j, k, l, m, n))   # (3 A as a lazy factor)
    res4(i, j, k, l, m, n) << 3.7 * res1(i, j, k, o) * (res2(o, p) / 3.7) * res3(p, l, m, n)
    assert approx(res4.to_ndarray(), A3.to_ndarray(), 1e-11)
    Q, R = xe.Tensor(), xe.Tensor()
    (Q(i, j, k, l), R(l, m, n, r)) << xe.QR(B7(i, j, k, m, n, r))
    res4(i, j, k, m, n, r) << (Q(i, j, k, o) / 12.5) * (12.5 * R(o, m, n, r) / 7)
    assert approx(res4.to_ndarray(), B.to_ndarray(), 1e-12)


def test_value_t_product(xe):
    """Tensor:value_t_Product (fullTensor_factor.cxx:57-79)"""
    A = T(xe, np.full((4, 2, 2, 7), 73.0))
    B, C, D = xe.Tensor(), xe.Tensor(), xe.Tensor()
    (j,) = xe.indices(1)
    B(j & 0) << A(j & 0) * 2.0
    C(j & 0) << 3 * A(j & 0)
    D(j & 0) << A(j & 0) / 73.0
    A(j & 0) << A(j & 0) / 2
    n = 4 * 2 * 2 * 7
    assert entrywise(B, [146] * n) and entrywise(C, [219] * n) and entrywise(D, [1] * n) and entrywise(A, [36.5] * n)


# ---------------------------------------------------------------------------------- fullTensor_utilities.cxx
def test_remove_slate(xe):
    """Tensor:remove_slate (fullTensor_utilities.cxx:25-42) with resize_mode's cut position"""
    A = T(xe, np.arange(1, 28, dtype=float).reshape(3, 3, 3))
    A.remove_slate(0, 1)
    assert entrywise(A, list(range(1, 10)) + list(range(19, 28)), 1e-14)
    A.resize_mode(0, 3, 1)
    assert entrywise(A, list(range(1, 10)) + [0] * 9 + list(range(19, 28)), 1e-14)
    A.remove_slate(1, 0)
    assert entrywise(A, [4, 5, 6, 7, 8, 9] + [0] * 6 + [22, 23, 24, 25, 26, 27], 1e-14)
    A.resize_mode(1, 3, 1)
    assert entrywise(A, [4, 5, 6, 0, 0, 0, 7, 8, 9] + [0] * 9 + [22, 23, 24, 0, 0, 0, 25, 26, 27], 1e-14)


def test_fix_mode(xe):
    """Tensor:fix_mode (fullTensor_utilities.cxx:44-55)"""
    A = T(xe, np.arange(1, 28, dtype=float).reshape(3, 3, 3))
    A.fix_mode(0, 1)
    assert entrywise(A, list(range(10, 19)), 1e-14)
    A.fix_mode(1, 2)
    assert entrywise(A, [12, 15, 18], 1e-14)


def test_dimension_reduction_and_expansion(xe):
    """Tensor:dimension_reduction / dimension_expansion (fullTensor_utilities.cxx:58-118)"""
    base = np.arange(1, 9, dtype=float).reshape(2, 2, 2)
    for mode, want in ((0, [1, 2, 3, 4]), (1, [1, 2, 5, 6]), (2, [1, 3, 5, 7])):
        A = T(xe, base)
        A.resize_mode(mode, 1)
        assert entrywise(A, want, 1e-13) and A.dimensions[mode] == 1 and A.size == 4
    for mode, want in ((0, [1, 2, 3, 4, 5, 6, 7, 8, 0, 0, 0, 0]), (1, [1, 2, 3, 4, 0, 0, 5, 6, 7, 8, 0, 0]),
                       (2, [1, 2, 0, 3, 4, 0, 5, 6, 0, 7, 8, 0])):
        A = T(xe, base)
        A.resize_mode(mode, 3)
        assert entrywise(A, want, 1e-13) and A.dimensions[mode] == 3 and A.size == 12


# -------------------------------------------------------------------------------------- fullTensor_solve.cxx
def test_solve_ax_equals_b(xe):
    """Tensor:solve_Ax_equals_b (fullTensor_solve.cxx:26-76): x(k,i) = b(j) / A(j,k,i), regular and singular A"""
    i, j, k = xe.indices(3)
    a1 = np.zeros((4, 2, 2))
    a1[0, 0, 0] = a1[1, 0, 1] = a1[2, 1, 0] = a1[3, 1, 1] = 1
    b1 = T(xe, [73, -73, 128, 93])
    x1 = xe.Tensor([2, 2])
    x1(k, i) << b1(j) / T(xe, a1)(j, k, i)
    got = x1.to_ndarray()
    assert abs(73 - got[0, 0]) < 1e-14 and abs(-73 - got[0, 1]) < 1e-14
    assert abs(128 - got[1, 0]) < 1e-14 and abs(93 - got[1, 1]) < 1e-14
    a2 = np.zeros((4, 2, 2))
    a2[0, 0, 0] = a2[1, 0, 1] = 1
    b2 = T(xe, [73, -73, 0, 0])
    x2 = xe.Tensor([2, 2])
    x2(k, i) << b2(j) / T(xe, a2)(j, k, i)
    got = x2.to_ndarray()
    assert abs(73 - got[0, 0]) < 1e-14 and abs(-73 - got[0, 1]) < 1e-14
    assert got[1, 0] < 1e-14 and got[1, 1] < 1e-14


def test_solve_vs_least_squares(xe):
    """Tensor:solve vs least squares (fullTensor_solve.cxx:78-133), dense legs: the 500 x 500 second-difference
    matrix (A[0] = 1): Cholesky; A[0] = -0.9: LDL; A[1] = -0.9: LU; least squares.

    The reference asserts ||A x - b|| < 1e-10 for its draw of b. The system has kappa ~ 1e6, so that residual
    is a backward error of order u ||A|| ||x|| and depends on the draw: here each leg must meet 1e-10 or stay
    within 4x of LAPACK's residual (numpy.linalg.solve / lstsq) on the same A and b."""
    N = 500
    a = 2 * np.eye(N) - np.eye(N, k=1) - np.eye(N, k=-1)
    a[0, 0] = 1
    xe.seed(78)
    B = xe.Tensor.random([N])
    b = B.to_ndarray()
    i, j = xe.indices(2)

    def check(A, X, leg, lsq=False):
        r = xe.Tensor()
        r(i) << A(i, j) * X(j) - B(i)
        an = A.to_ndarray()
        xl = np.linalg.lstsq(an, b, rcond=None)[0] if lsq else np.linalg.solve(an, b)
        lapack = np.linalg.norm(an @ xl - b)
        assert r.frob_norm() < max(1e-10, 4 * lapack), (leg, r.frob_norm(), lapack)

    A = T(xe, a)
    check(A, xe.solve(A, B), "cholesky")
    A[0] = -0.9
    check(A, xe.solve(A, B), "ldl")
    A[1] = -0.9
    check(A, xe.solve(A, B), "lu")
    check(A, xe.solve_least_squares(A, B), "least squares", lsq=True)


def test_solve_transposed(xe):
    """Tensor:solve_transposed (fullTensor_solve.cxx:150-184), dense legs: x(i) = r(j) / A(i,j) equals
    r(j) / At(j,i) with At = A^T to 1e-12 (identity plus 300 random off-diagonal entries)"""
    N = 100
    rng = np.random.default_rng(150)
    a = np.eye(N).ravel()
    a[rng.integers(1, N * N, size=3 * N)] = rng.standard_normal(3 * N)
    A = T(xe, a.reshape(N, N))
    i, j = xe.indices(2)
    At = xe.Tensor()
    At(i, j) << A(j, i)
    r = T(xe, np.arange(N, dtype=float))
    x3, x4 = xe.Tensor(), xe.Tensor()
    x3(i) << r(j) / A(i, j)
    x4(i) << r(j) / At(j, i)
    assert np.linalg.norm(x3.to_ndarray() - x4.to_ndarray()) < 1e-12
    want = np.linalg.solve(a.reshape(N, N).T, np.arange(N, dtype=float))   # r(j) = A(i,j) x(i): A^T x = r
    assert np.linalg.norm(x3.to_ndarray() - want) <= 1e-12 * np.linalg.norm(want)


def test_solve_matrix(xe):
    """Tensor:solve_matrix (fullTensor_solve.cxx:186-223): random A (m... x n...), B = A X_real with extra modes
    p...; solve_least_squares and the indexed X(j^n, k^p) = B(i^m, k^p) / A(i^m, j^n) leave residuals < 1e-10"""
    rng = np.random.default_rng(186)
    xe.seed(186)
    for run in range(10):
        degM, degN, degP = (int(v) for v in (rng.integers(1, 4), rng.integers(1, 4), rng.integers(0, 4)))
        mDims = [int(v) for v in rng.integers(1, 11, size=degM)]
        nDims = [int(v) for v in rng.integers(1, 11, size=degN)]
        pDims = [int(v) for v in rng.integers(1, 11, size=degP)]
        A = xe.Tensor.random(mDims + nDims) * float(rng.standard_normal())
        realX = xe.Tensor.random(nDims + pDims)
        i, j, k = xe.indices(3)
        B = xe.Tensor()
        B(i ^ degM, k ^ degP) << A(i ^ degM, j ^ degN) * realX(j ^ degN, k ^ degP)
        B = B * float(rng.standard_normal())
        X = xe.solve_least_squares(A, B, degP)
        res = xe.Tensor()
        res(i ^ degM, k ^ degP) << A(i ^ degM, j ^ degN) * X(j ^ degN, k ^ degP) - B(i ^ degM, k ^ degP)
        assert res.frob_norm() < 1e-10, (run, res.frob_norm())
        X2 = xe.Tensor()
        X2(j ^ degN, k ^ degP) << B(i ^ degM, k ^ degP) / A(i ^ degM, j ^ degN)
        res(i ^ degM, k ^ degP) << A(i ^ degM, j ^ degN) * X2(j ^ degN, k ^ degP) - B(i ^ degM, k ^ degP)
        assert res.frob_norm() < 1e-10, (run, res.frob_norm())


# ------------------------------------------------------------------------------------------------ tensor.cxx
def test_one_norm(xe):
    """Tensor:one_norm (tensor.cxx:56-70)"""
    (i,) = xe.indices(1)
    A = xe.Tensor.ones([100, 100])
    assert abs(A.one_norm() - 100.0 * 100) <= 1e-12 * 1e4
    assert abs(xe.one_norm(A) - 100.0 * 100) <= 1e-12 * 1e4
    assert abs(A.frob_norm() - 100.0) <= 1e-12 * 100
    A = xe.Tensor.identity([100, 100])
    assert abs(A.one_norm() - 100.0) <= 1e-12 * 100
    assert abs(A.frob_norm() - 10.0) <= 1e-12 * 10
