"""The tests' TT difference norm (tests/ttutil.py) against dense tensors."""
import numpy as np

from ttutil import tt_diff_norm


def _full(cores):
    res = cores[0]
    for c in cores[1:]:
        res = np.tensordot(res, c, axes=([res.ndim - 1], [0]))
    return res.reshape([c.shape[1] for c in cores])


def test_tt_diff_norm_matches_dense():
    rng = np.random.default_rng(0)
    dims, ra, rb = [3, 4, 2, 5], [1, 3, 4, 2, 1], [1, 2, 5, 3, 1]
    A = [rng.standard_normal((ra[k], dims[k], ra[k + 1])) for k in range(4)]
    B = [rng.standard_normal((rb[k], dims[k], rb[k + 1])) for k in range(4)]
    diff, nb = tt_diff_norm(A, B)
    assert abs(diff - np.linalg.norm(_full(A) - _full(B))) <= 1e-12 * diff
    assert abs(nb - np.linalg.norm(_full(B))) <= 1e-12 * nb
    assert tt_diff_norm(B, B)[0] <= 1e-13 * nb
