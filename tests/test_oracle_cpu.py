"""CPU: the oracle is pinned against golden vectors before it is trusted (no GPU needed)."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_rng_stream_matches_libstdcxx(ref):
    g = json.load(open(os.path.join(GOLD, "rng_baadf00d.json")))
    r = ref.Rng(g["seed"])
    vals = r.normal(len(g["normal"]))
    assert np.array_equal(vals, np.array(g["normal"]))  # bit-exact


@pytest.mark.parametrize("dims,shuffle", [
    ((64, 64, 64), (0, 2, 1)), ((3, 4, 5), (2, 1, 0)), ((2, 3, 4, 5), (1, 0, 3, 2)),
    ((1, 1, 6, 5, 7), (0, 1, 3, 4, 2)), ((4, 5), (0, 1)), ((2, 1, 3), (2, 0, 1)), ((7,), (0,)),
    ((3, 4, 2, 5), (3, 2, 1, 0)), ((2, 3, 4), (1, 2, 0)),
])
def test_reshuffle_oracle_is_a_permutation(ref, dims, shuffle):
    a = np.random.default_rng(1).standard_normal(dims)
    out = ref.reshuffle(a, shuffle)
    inv = [0] * len(shuffle)
    for i, s in enumerate(shuffle):
        inv[s] = i
    assert np.array_equal(out, np.transpose(a, inv))


def test_contract_matches_einsum(ref):
    rng = np.random.default_rng(2)
    B = rng.standard_normal((4, 5, 6))
    Cc = rng.standard_normal((5, 7, 6))
    # A(i,j) = B(i,k,l) * C(k,j,l): C reshuffled {0,2,1} then contract 2 modes
    Cr = ref.reshuffle(Cc, (0, 2, 1))
    A = ref.contract(B, False, Cr, False, 2)
    assert np.allclose(A, np.einsum("ikl,kjl->ij", B, Cc), rtol=1e-13, atol=1e-13)
    # transposed operands: A2(k,l,m) = sum_i B(i,k,l) * D(m,i)
    D = rng.standard_normal((3, 4))
    A2 = ref.contract(B, True, D, True, 1)
    assert np.allclose(A2, np.einsum("ikl,mi->klm", B, D), rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("m,n", [(8, 5), (5, 8), (6, 6), (1, 4), (4, 1)])
def test_qc_cq_properties(ref, m, n):
    A = np.random.default_rng(3).standard_normal((m, n))
    Q, Cm, r = ref.qc(A)
    assert r == min(m, n)
    assert np.allclose(Q @ Cm, A, atol=1e-13)
    assert np.allclose(Q.T @ Q, np.eye(r), atol=1e-13)
    Cc, Q2, r2 = ref.cq(A)
    assert r2 == min(m, n)
    assert np.allclose(Cc @ Q2, A, atol=1e-13)
    assert np.allclose(Q2 @ Q2.T, np.eye(r2), atol=1e-13)


def test_qc_rank_rule_signed_r00(ref):
    """blasLapackWrapper.cpp:268-272 compares against 16*eps*R_00 without abs: rank is only reduced
    when dgeqp3's R_00 > 0, i.e. when the pivot column's first entry is negative (dlarfg sign)."""
    rng = np.random.default_rng(4)
    a = rng.standard_normal((10, 1))
    b = rng.standard_normal((1, 3))
    A = a @ b                                   # rank 1, 10 x 3
    p = int(np.argmax(np.linalg.norm(A, axis=0)))
    _, _, r = ref.qc(A)
    if A[0, p] < 0:
        assert r == 1
    else:
        assert r == 3
    _, _, r2 = ref.qc(-A)
    assert {r, r2} == {1, 3}


def test_tt_round_oracle_properties(ref):
    rng = ref.Rng()
    x = ref.TT.random([4, 5, 3, 4, 2], [3, 6, 5, 2], rng)
    full = x.full()
    # random() ends with move_core(0): cores 1.. right-orthogonal
    for c in x.cores[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.allclose(M @ M.T, np.eye(M.shape[0]), atol=1e-12)
    y = x.copy()
    y.round(100)
    assert y.ranks == x.ranks
    assert np.linalg.norm(y.full() - full) <= 1e-13 * np.linalg.norm(full)
    z = x.copy()
    z.round(2)
    assert max(z.ranks) <= 2
    # x + x has doubled internal ranks; rounding recovers the ranks of x (SVD eps cut)
    s2 = ref.tt_add(x, x)
    assert s2.ranks == [2 * r for r in x.ranks]
    s2.round(100)
    assert s2.ranks == x.ranks
    assert np.linalg.norm(s2.full() - 2 * full) <= 1e-12 * np.linalg.norm(full)


def test_tt_dot_oracle(ref):
    rng = ref.Rng(7)
    x = ref.TT.random([3, 4, 3, 2], [2, 5, 3], rng)
    y = ref.TT.random([3, 4, 3, 2], [3, 2, 2], rng)
    assert np.isclose(ref.dot(x, y), float(np.sum(x.full() * y.full())), rtol=1e-12, atol=1e-12)
    assert np.isclose(x.frob_norm(), np.linalg.norm(x.full()), rtol=1e-12)
