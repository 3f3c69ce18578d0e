"""Ports of the reference's TT arithmetic unit tests (src/unitTests/ttArithmetic.cxx): sums, differences,
operator products (TTStack contraction), transposes and dyadic products of TTTensor / TTOperator against
the dense Tensor computed the same way, with the reference's tolerances. Index expressions the Python
binding does not parse (transposed operator factors, chains of three) are written with TTOperator.transpose()
and two products; the arithmetic is the reference's. Random draws: the library's mt19937_64 stream (seeded
per test), dimensions of the randomised loops from numpy.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def full(xe, t):
    return xe.Tensor(t).to_ndarray()


def approx(a, b, eps):
    a, b = np.asarray(a), np.asarray(b)
    return np.linalg.norm(a - b) <= eps * (np.linalg.norm(a) + np.linalg.norm(b)) / 2


def op_mat(a, d):
    """the 2d-mode operator tensor as a matrix (rows: first d modes)"""
    rows = int(np.prod(a.shape[:d]))
    return a.reshape(rows, -1)


def apply(xe, A, x):
    i, j = xe.indices(2)
    y = xe.TTTensor()
    y(i & 0) << A(i / 2, j / 2) * x(j & 0)
    return y


def apply_t(xe, A, x):
    """x^T A: y(j&0) = x(i&0) * A(i/2, j/2)"""
    i, j = xe.indices(2)
    y = xe.TTTensor()
    y(j & 0) << x(i & 0) * A(i / 2, j / 2)
    return y


def op_prod(xe, A, B):
    i, j, k = xe.indices(3)
    C = xe.TTOperator()
    C(i / 2, k / 2) << A(i / 2, j / 2) * B(j / 2, k / 2)
    return C


def transposed(xe, A):
    T = xe.TTOperator(A)
    T.transpose()
    return T


def test_sum(xe):
    """TT:sum (ttArithmetic.cxx:27-55): dims from intDist(1, 10); TT and TTOperator sums to 3.1e-13."""
    rng = np.random.default_rng(27)
    dims = [int(v) for v in rng.integers(1, 11, size=4)]
    xe.seed(27)
    A, B = xe.Tensor.random(dims), xe.Tensor.random(dims)
    C = A.to_ndarray() + B.to_ndarray()
    ttC = xe.TTTensor(A) + xe.TTTensor(B)
    toC = xe.TTOperator(A) + xe.TTOperator(B)
    assert np.linalg.norm(full(xe, ttC) - C) < 3.1e-13
    assert np.linalg.norm(full(xe, toC) - C) < 3.1e-13


def test_difference(xe):
    """TT:difference (ttArithmetic.cxx:57-72)."""
    xe.seed(57)
    A, B = xe.Tensor.random([10] * 4), xe.Tensor.random([10] * 4)
    ttC = xe.TTTensor(A) - xe.TTTensor(B)
    assert np.linalg.norm(full(xe, ttC) - (A.to_ndarray() - B.to_ndarray())) < 1e-12


def test_real_difference(xe):
    """TT:real_difference (ttArithmetic.cxx:74-114): x - x, (x + y) - (y + x), 73 x + y - (y + 73 x) vanish;
    the ranks of a sum are the sums of ranks."""
    xe.seed(74)
    ttA = xe.TTTensor.random([10] * 5, [4] * 4)
    ttB = xe.TTTensor.random([10] * 5, [4] * 4)
    fn = lambda t: t.frob_norm()  # noqa: E731
    assert fn(ttA - ttA) < 1e-11
    assert fn(ttB - ttB) < 1e-11
    assert fn((ttA + ttB) - (ttA + ttB)) < 1e-11
    assert (ttA + ttB).ranks() == [8] * 4
    assert (ttB + ttA).ranks() == [8] * 4
    assert fn((ttA + ttB) - (ttB + ttA)) < 1e-11
    assert fn((73 * ttA + ttB) - (ttB + 73 * ttA)) < 1e-9
    ttA = xe.TTTensor.random([10] * 5, [2, 5, 7, 2])
    assert fn(ttA - ttA) < 1e-11
    assert fn(ttB - ttB) < 1e-11
    assert fn((ttA + ttB) - (ttA + ttB)) < 1e-11
    assert fn((ttA + ttB) - (ttB + ttA)) < 1e-11
    assert fn((73 * ttA + ttB) - (ttB + 73 * ttA)) < 5e-10


def test_difference_of_ttstacks(xe):
    """TT:difference_of_TTStacks (ttArithmetic.cxx:116-130)."""
    xe.seed(116)
    ttO = xe.TTOperator.random([10] * 10, [4] * 4)
    ttA = xe.TTTensor.random([10] * 5, [4] * 4)
    ttB = xe.TTTensor.random([10] * 5, [4] * 4)
    assert (apply(xe, ttO, ttA) - apply(xe, ttO, ttA)).frob_norm() < 1e-7
    assert (apply(xe, ttO, ttB) - apply(xe, ttO, ttB)).frob_norm() < 1e-7


def test_ttstacks_frob_norm(xe):
    """TT:ttStacks_frob_norm (ttArithmetic.cxx:132-141): <I, I> = 10^5 and ||I I||_F = sqrt(10^5)."""
    I1 = xe.TTOperator.identity([10] * 10)
    I2 = xe.TTOperator.identity([10] * 10)
    # <I1, I2> = ||I||_F^2 = 10^5 (I1 = I2)
    assert abs(I1.frob_norm() * I2.frob_norm() - 1e5) <= 1e-9 * 1e5
    assert abs(op_prod(xe, I1, I2).frob_norm() - np.sqrt(1e5)) <= 1e-12 * np.sqrt(1e5)


def test_product(xe):
    """TT:product (ttArithmetic.cxx:202-254): operator x tensor and operator x operator (with transposed
    factors) against the dense products, 10^4 * 1e-15; the product operator has d + 2 nodes (ranks r_A r_B)."""
    xe.seed(202)
    ttA = xe.TTOperator.random([10] * 4, 1)
    ttB = xe.TTOperator.random([10] * 4, 1)
    ttD = xe.TTTensor.random([10] * 2, 2)
    A, B, D = op_mat(full(xe, ttA), 2), op_mat(full(xe, ttB), 2), full(xe, ttD).reshape(-1)
    bar = 1e4 * 1e-15
    assert np.linalg.norm(full(xe, apply(xe, ttA, ttD)).reshape(-1) - A @ D) < bar
    C = op_prod(xe, ttA, ttB)
    assert C.degree() == 4 and len(C.ranks()) == 1
    assert np.linalg.norm(op_mat(full(xe, C), 2) - A @ B) < bar
    # C(i/2,k/2) = A(j/2,i/2) * B(j/2,k/2): A^T B
    assert np.linalg.norm(op_mat(full(xe, op_prod(xe, transposed(xe, ttA), ttB)), 2) - A.T @ B) < bar
    # C(i^2,k^2) = A(i^2,j^2) * B(k^2,j^2): A B^T
    assert np.linalg.norm(op_mat(full(xe, op_prod(xe, ttA, transposed(xe, ttB))), 2) - A @ B.T) < bar
    # C(i^2,k^2) = A(j^2,i^2) * B(k^2,j^2): A^T B^T
    assert np.linalg.norm(op_mat(full(xe, op_prod(xe, transposed(xe, ttA), transposed(xe, ttB))), 2) - A.T @ B.T) < bar


def test_identities(xe):
    """TT:identities (ttArithmetic.cxx:256-289): a perturbed 4 x 4 identity I, products I I, I I^T against
    the dense ones at 1e-15."""
    I = np.zeros((2, 2, 2, 2))
    for idx in np.ndindex(2, 2, 2, 2):
        if (idx[0] == idx[2] and idx[1] == idx[3]) or idx == (0, 1, 0, 0):
            I[idx] = 1.0
    ttI = xe.TTOperator(xe.Tensor.from_ndarray(I))
    M = op_mat(I, 2)
    for C, want in ((op_prod(xe, ttI, ttI), M @ M), (op_prod(xe, ttI, transposed(xe, ttI)), M @ M.T)):
        got = op_mat(full(xe, C), 2)
        assert approx(want, got, 1e-15)
        assert approx(want.T, op_mat(full(xe, transposed(xe, C)), 2), 1e-15)   # C(k^2, i^2) forms


def test_transpose(xe):
    """TT:transpose (ttArithmetic.cxx:291-301)."""
    xe.seed(291)
    A = xe.Tensor.random([10] * 4)
    ttA = xe.TTOperator(A)
    ttA.transpose()
    assert approx(op_mat(A.to_ndarray(), 2).T, op_mat(full(xe, ttA), 2), 1e-14)


def test_ax_b(xe):
    """TT:ax_b (ttArithmetic.cxx:303-362): the identity operator applied to TTs (and transposed) leaves them
    unchanged; residuals A x - b assembled two ways agree to 1e-7."""
    xe.seed(303)
    X = xe.TTTensor.random([10] * 3, [2, 2])
    B = xe.TTTensor.random([10] * 3, [2, 2])
    I = np.zeros((10,) * 6)
    for a in range(10):
        for b in range(10):
            for c in range(10):
                I[a, b, c, a, b, c] = 1.0
    A = xe.TTOperator(xe.Tensor.from_ndarray(I))
    T = apply(xe, A, X) - B
    S = apply(xe, A, X) - B
    assert (T - S).frob_norm() < 1e-7
    fA, fX = op_mat(full(xe, A), 3), full(xe, X).reshape(-1)
    assert np.linalg.norm(fA @ fX - fX) < 1e-7
    T = apply(xe, A, X)
    assert np.linalg.norm(full(xe, T).reshape(-1) - fA @ fX) < 1e-7
    assert (T - X).frob_norm() < 1e-7
    assert (apply(xe, A, X) - X).frob_norm() < 1e-7
    T = apply_t(xe, A, X)
    assert (T - X).frob_norm() < 1e-7
    T = apply_t(xe, A, B) - B
    assert T.frob_norm() < 1e-7


def test_operator_times_tensor(xe):
    """TT:operator_times_tensor (ttArithmetic.cxx:364-406): chains of rank-2 operators (rounded) applied
    to a TT and multiplied together against the dense products, 2e-13..3e-13 (2e-15 for A B B^T)."""
    xe.seed(364)
    ttA = xe.TTOperator(xe.Tensor.random([10] * 4))
    ttA.round(2)
    ttB = xe.TTOperator(xe.Tensor.random([10] * 4))
    ttB.round(2)
    C = xe.Tensor.random([10, 10])
    ttC = xe.TTTensor(C)
    A, B, c = op_mat(full(xe, ttA), 2), op_mat(full(xe, ttB), 2), C.to_ndarray().reshape(-1)
    D = apply(xe, ttA, apply(xe, ttB, ttC))
    assert approx(A @ B @ c, full(xe, D).reshape(-1), 3e-13)
    D = apply(xe, ttA, apply(xe, transposed(xe, ttB), ttC))
    assert approx(A @ B.T @ c, full(xe, D).reshape(-1), 2e-13)
    assert approx(A @ B, op_mat(full(xe, op_prod(xe, ttA, ttB)), 2), 2e-13)
    assert approx(A @ A, op_mat(full(xe, op_prod(xe, ttA, ttA)), 2), 2e-13)
    assert approx(A @ B @ A.T, op_mat(full(xe, op_prod(xe, op_prod(xe, ttA, ttB), transposed(xe, ttA))), 2), 2e-13)
    assert approx(A @ B @ B.T, op_mat(full(xe, op_prod(xe, op_prod(xe, ttA, ttB), transposed(xe, ttB))), 2), 2e-13)
    assert approx(A @ B @ B.T @ A, op_mat(full(xe, op_prod(xe, op_prod(xe, op_prod(xe, ttA, ttB), transposed(xe, ttB)), ttA)), 2),
                  2e-13)


def test_disjoint_product(xe):
    """TT:disjoint_product (ttArithmetic.cxx:435-466): dyadic_product of TT-SVDs of random tensors of
    orders 0..5 (dims from dimDist(1, 5)) equals the dense outer product to 1e-13."""
    rng = np.random.default_rng(435)
    xe.seed(435)
    dimsA, dimsB = [], []
    for d in range(6):
        A, B = xe.Tensor.random(dimsA), xe.Tensor.random(dimsB)
        ttC = xe.dyadic_product(xe.TTTensor(A), xe.TTTensor(B))
        C = np.multiply.outer(A.to_ndarray(), B.to_ndarray())
        assert approx(C, full(xe, ttC), 1e-13)
        dimsA.append(int(rng.integers(1, 6)))
        dimsB.append(int(rng.integers(1, 6)))
