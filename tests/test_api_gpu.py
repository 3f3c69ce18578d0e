"""The xerus C++ API (through the pybind module) on the GPU: indexed expressions, Tensor operations,
factorisations and TTTensor, checked against the reference's known answers (tests/golden) and the
CPU oracles (oracle/indexed.py, oracle/xerus_ref.py)."""
import json
import os

import numpy as np
import pytest

from oracle import indexed

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_products.json")))


def _idx(xe, names, tok):
    if isinstance(tok, int):
        return xe.Index(tok)
    p = indexed.parse(tok)
    if p[0] not in names:
        names[p[0]] = xe.Index()
    base = names[p[0]]
    op, n = p[1], p[2]
    if op == "&":
        return base & n
    if op == "/":
        return base / n
    return base ^ n if n != 1 else base


def _tensor(xe, arr):
    return xe.Tensor.from_ndarray(np.require(np.asarray(arr, dtype=np.float64), requirements="C"))


def _run(xe, lhs_tokens, terms, out=None, scale=1.0):
    """terms: [(xe.Tensor, tokens)]; returns the LHS tensor."""
    names = {}
    idx_terms = [T(*[_idx(xe, names, t) for t in toks]) for T, toks in terms]
    prod = idx_terms[0] if len(idx_terms) == 1 else idx_terms[0] * idx_terms[1]
    for it in idx_terms[2:]:
        prod = prod * it
    if scale != 1.0:
        prod = scale * prod
    out = xe.Tensor() if out is None else out
    out(*[_idx(xe, names, t) for t in lhs_tokens]) << prod
    return out


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_known_answers(xe, case):
    arrs = {k: np.array(v["values"], dtype=np.float64).reshape(v["dims"]) for k, v in case["inputs"].items()}
    tens = {k: _tensor(xe, a) for k, a in arrs.items()}
    out = _run(xe, case["lhs"], [(tens[n], toks) for n, toks in case["rhs"]], scale=case["scale"])
    np.testing.assert_array_equal(out.to_ndarray().reshape(-1), np.array(case["expected"], dtype=np.float64))


@pytest.mark.parametrize("case", GOLDEN["errors"], ids=[c["name"] for c in GOLDEN["errors"]])
def test_rejected_expressions(xe, case):
    A = xe.Tensor.random(case["dims"])
    B = xe.Tensor.random(case.get("dims_b", [1]))
    tens = {"A": A, "B": B}
    with pytest.raises(xe.generic_error):
        _run(xe, case["lhs"], [(tens[n], toks) for n, toks in case["rhs"]], out=xe.Tensor())


RANDOM_EXPRS = [
    # (lhs, [(dims, tokens), ...])
    (["i", "j"], [([64, 64, 64], ["i", "k", "l"]), ([64, 64, 64], ["k", "j", "l"])]),          # cfg1 shape
    (["j", "i"], [([17, 33, 9], ["i", "k", "l"]), ([9, 33, 21], ["l", "k", "j"])]),
    (["a", "d"], [([7, 8], ["a", "b"]), ([8, 9], ["b", "c"]), ([9, 10], ["c", "d"])]),        # 3-node closed form
    (["a", "e"], [([5, 6], ["a", "b"]), ([6, 7], ["b", "c"]), ([7, 8], ["c", "d"]), ([8, 9], ["d", "e"])]),   # heuristics
    (["a", "b", "c"], [([4, 5, 6], ["a", "x", "y"]), ([5, 7], ["x", "z"]), ([6, 7, 3], ["y", "z", "b"]), ([3, 4, 8], ["w", "v", "c"]),
                       ([3, 4], ["w", "v"])]),
    ([], [([6, 7, 8], ["i", "j", "k"]), ([8, 7, 6], ["k", "j", "i"])]),
    (["i", "j"], [([6, 6], ["i", "k"]), ([6, 6], ["k", "l"]), ([6, 6], ["l", "m"]), ([6, 6], ["m", "n"]), ([6, 6], ["n", "o"]),
                  ([6, 6], ["o", "j"])]),
    (["i^2", "j"], [([3, 4, 5, 6], ["i^2", "k^2"]), ([5, 6, 7], ["k^2", "j"])]),
    (["j", "i"], [([4, 4, 5], ["k", "k", "i"]), ([5, 3], ["i2", "j"]), ([5], ["i2"])]),
    (["i", "j"], [([5, 6], ["i", "j"]), ([4], ["k"]), ([4], ["k"])]),                            # unconnected scalar component
    (["i", "j"], [([3, 5, 4], ["i", 2, "j"])]),                                                  # slice
    (["m", "i"], [([4, 3, 4, 5], ["a", "i", "a", "k"]), ([5, 6], ["k", "m"])]),                  # trace + contraction
]


@pytest.mark.parametrize("k", range(len(RANDOM_EXPRS)))
def test_random_expressions_vs_oracle(xe, k):
    lhs, spec = RANDOM_EXPRS[k]
    rng = np.random.default_rng(100 + k)
    arrs = [rng.standard_normal(d) for d, _ in spec]
    out = _run(xe, lhs, [(_tensor(xe, a), toks) for a, (_, toks) in zip(arrs, spec)], scale=-0.5)
    ref = indexed.evaluate(lhs, [(a, toks) for a, (_, toks) in zip(arrs, spec)], scale=-0.5)
    got = out.to_ndarray()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(ref).max()))


def test_permutation_bit_exact(xe):
    rng = np.random.default_rng(3)
    a = rng.standard_normal((3, 4, 5, 6, 7))
    A = _tensor(xe, a)
    B = xe.Tensor()
    i, j, k, l, m = xe.indices(5)
    B(m, k, i, l, j) << A(i, j, k, l, m)
    np.testing.assert_array_equal(B.to_ndarray(), np.einsum("ijklm->mkilj", a))
    C = xe.reshuffle(A, [4, 2, 0, 3, 1])   # old mode i -> new position shuffle[i]
    np.testing.assert_array_equal(C.to_ndarray(), np.einsum("ijklm->kmjli", a))


def test_sums_and_updates(xe):
    rng = np.random.default_rng(4)
    a, b, d = rng.standard_normal((5, 6)), rng.standard_normal((6, 5)), rng.standard_normal((6, 6))
    A, B, D = _tensor(xe, a), _tensor(xe, b), _tensor(xe, d)
    i, j, k = xe.indices(3)
    R = xe.Tensor()
    R(i, j) << A(i, j) + B(j, i) - 2.0 * A(i, j)
    np.testing.assert_allclose(R.to_ndarray(), b.T - a, rtol=1e-14, atol=1e-14)
    R(i, j) << A(i, j)
    R(i, j).__iadd__(B(j, i))
    np.testing.assert_allclose(R.to_ndarray(), a + b.T, rtol=1e-14)
    R(i, j).__isub__(A(i, k) * D(k, j))
    np.testing.assert_allclose(R.to_ndarray(), a + b.T - a @ d, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(A.to_ndarray(), a)   # operands untouched


def test_aliasing_assignment(xe):
    rng = np.random.default_rng(5)
    a = rng.standard_normal((6, 6))
    A = _tensor(xe, a)
    i, j, k = xe.indices(3)
    A(i, j) << A(j, i)
    np.testing.assert_array_equal(A.to_ndarray(), a.T)
    A(i, k) << A(i, j) * A(j, k)
    np.testing.assert_allclose(A.to_ndarray(), a.T @ a.T, rtol=1e-13)


def test_scalar_results(xe):
    rng = np.random.default_rng(6)
    a, b = rng.standard_normal((4, 5)), rng.standard_normal((4, 5))
    A, B = _tensor(xe, a), _tensor(xe, b)
    i, j = xe.indices(2)
    assert float(A(i, j) * B(i, j)) == pytest.approx(float((a * b).sum()), rel=1e-13)
    assert float(A(i & 0) * B(i & 0)) == pytest.approx(float((a * b).sum()), rel=1e-13)
    assert xe.frob_norm(A(i, j)) == pytest.approx(np.linalg.norm(a), rel=1e-14)


def test_lazy_factor_and_cow(xe):
    rng = np.random.default_rng(7)
    a = rng.standard_normal((8, 9))
    A = _tensor(xe, a)
    B = 3.0 * A                       # shares storage, factor 3
    assert B.factor == 3.0 and A.factor == 1.0
    B[0] = 1.0                        # applies the factor and copies on write
    assert A[0] == a.reshape(-1)[0]
    np.testing.assert_allclose(B.to_ndarray().reshape(-1)[1:], 3.0 * a.reshape(-1)[1:], rtol=1e-15)
    i, j, k = xe.indices(3)
    C = xe.Tensor()
    C(i, k) << (2.0 * A)(i, j) * (A / 4.0)(k, j)
    np.testing.assert_allclose(C.to_ndarray(), 0.5 * a @ a.T, rtol=1e-13)
    assert A.frob_norm() == pytest.approx(np.linalg.norm(a), rel=1e-14)
    assert (-2.0 * A).frob_norm() == pytest.approx(2 * np.linalg.norm(a), rel=1e-14)


def test_contract_flags(xe):
    rng = np.random.default_rng(8)
    a, b = rng.standard_normal((6, 7, 8)), rng.standard_normal((7, 8, 5))
    A, B = _tensor(xe, a), _tensor(xe, b)
    R = xe.contract(A, False, B, False, 2)
    np.testing.assert_allclose(R.to_ndarray(), np.einsum("ijk,jkl->il", a, b), rtol=1e-13)
    bt = np.ascontiguousarray(np.moveaxis(b, 2, 0))   # (5,7,8)
    R2 = xe.contract(A, False, _tensor(xe, bt), True, 2)
    np.testing.assert_allclose(R2.to_ndarray(), np.einsum("ijk,ljk->il", a, bt), rtol=1e-13)
    at = np.ascontiguousarray(np.moveaxis(a, 0, 2))   # (7,8,6)
    R3 = xe.contract(_tensor(xe, at), True, B, False, 2)
    np.testing.assert_allclose(R3.to_ndarray(), np.einsum("jki,jkl->il", at, b), rtol=1e-13)


def test_mode_operations(xe):
    rng = np.random.default_rng(9)
    a = rng.standard_normal((3, 5, 4))
    A = _tensor(xe, a)
    A.resize_mode(1, 7)
    ref = np.zeros((3, 7, 4))
    ref[:, :5] = a
    np.testing.assert_array_equal(A.to_ndarray(), ref)
    A = _tensor(xe, a)
    A.resize_mode(1, 3)
    np.testing.assert_array_equal(A.to_ndarray(), a[:, :3])
    A = _tensor(xe, a)
    A.resize_mode(1, 7, 2)   # insert two zero slates at position 2
    ref = np.zeros((3, 7, 4))
    ref[:, :2] = a[:, :2]
    ref[:, 4:] = a[:, 2:]
    np.testing.assert_array_equal(A.to_ndarray(), ref)
    A = _tensor(xe, a)
    A.resize_mode(1, 3, 3)   # remove slates 1 and 2 (the two before the cut)
    np.testing.assert_array_equal(A.to_ndarray(), a[:, [0, 3, 4]])
    A = _tensor(xe, a)
    A.remove_slate(1, 2)
    np.testing.assert_array_equal(A.to_ndarray(), a[:, [0, 1, 3, 4]])
    A = _tensor(xe, a)
    A.fix_mode(1, 3)
    np.testing.assert_array_equal(A.to_ndarray(), a[:, 3])
    c = rng.standard_normal((4, 3, 4, 2))
    C = _tensor(xe, c)
    C.perform_trace(0, 2)
    np.testing.assert_allclose(C.to_ndarray(), np.einsum("aiaj->ij", c), rtol=1e-14)
    big = xe.Tensor([5, 6, 7])
    small = _tensor(xe, a)
    big.offset_add(small, [1, 0, 2])
    ref = np.zeros((5, 6, 7))
    ref[1:4, 0:5, 2:6] = a
    np.testing.assert_array_equal(big.to_ndarray(), ref)


def test_constructors(xe):
    np.testing.assert_array_equal(xe.Tensor.ones([2, 3]).to_ndarray(), np.ones((2, 3)))
    np.testing.assert_array_equal(xe.Tensor.identity([3, 2, 3, 2]).to_ndarray().reshape(6, 6), np.eye(6))
    k = np.zeros((3, 3, 3))
    for t in range(3):
        k[t, t, t] = 1
    np.testing.assert_array_equal(xe.Tensor.kronecker([3, 3, 3]).to_ndarray(), k)
    d = xe.Tensor.dirac([2, 3], [1, 2]).to_ndarray()
    assert d[1, 2] == 1 and d.sum() == 1
    assert xe.Tensor([4, 4]).frob_norm() == 0.0


def test_random_stream_matches_reference_rng(xe, ref):
    xe.seed(0xBAADF00D)
    T = xe.Tensor.random([7, 11])
    rng = ref.Rng(0xBAADF00D)
    np.testing.assert_array_equal(T.to_ndarray(), ref.tensor_random(rng, [7, 11]))


def test_save_load_roundtrip(xe, tmp_path):
    rng = np.random.default_rng(10)
    a = rng.standard_normal((3, 4, 2))
    A = _tensor(xe, a) * 2.5
    for tsv in (False, True):
        f = str(tmp_path / f"t{int(tsv)}.xrs")
        xe.save_to_file(A, f, tsv)
        B = xe.load_from_file(f)
        if tsv:   # the reference writes digits10 + 1 = 16 significant digits (tensor.cpp:1783)
            np.testing.assert_allclose(B.to_ndarray(), 2.5 * a, rtol=1e-15, atol=0)
        else:
            np.testing.assert_array_equal(B.to_ndarray(), 2.5 * a)
    # byte layout of the binary stream (misc/fileIO.h:103-118, tensor.cpp:1781-1804)
    from ttutil import read_xerus_file

    kind, payload = read_xerus_file(str(tmp_path / "t0.xrs"))
    assert kind == "xerus::Tensor"
    assert payload["dims"] == [3, 4, 2]
    np.testing.assert_array_equal(payload["data"].reshape(3, 4, 2), 2.5 * a)


def test_tt_file_roundtrip_and_layout(xe, tmp_path):
    """TTTensor files (ttNetwork.cpp:1455-1487 + tensorNetwork.cpp:1429-1466): the reference's node layout
    (ghost ones({1}) nodes around the components), canonical flag and core position, both formats."""
    from ttutil import read_xerus_file

    xe.seed(7)
    x = xe.TTTensor.random([4, 5, 3, 6], [3, 4, 5])
    dense = xe.Tensor(x).to_ndarray()
    for tsv in (False, True):
        f = str(tmp_path / f"tt{int(tsv)}.xrs")
        xe.save_to_file(x, f, tsv)
        assert xe.file_type(f) == "xerus::TTNetwork<false>"
        y = xe.load_from_file(f)
        assert y.ranks() == x.ranks() and y.canonicalized == x.canonicalized and y.corePosition == x.corePosition
        np.testing.assert_allclose(xe.Tensor(y).to_ndarray(), dense, rtol=0, atol=1e-14 * np.abs(dense).max())
    kind, p = read_xerus_file(str(tmp_path / "tt0.xrs"))
    assert kind == "xerus::TTNetwork<false>"
    assert p["canonicalized"] is True and p["corePosition"] == 0
    net = p["network"]
    d = 4
    assert net["dims"] == [4, 5, 3, 6]
    assert net["external"] == [(k + 1, 1, n) for k, n in enumerate([4, 5, 3, 6])]
    assert len(net["nodes"]) == d + 2
    assert net["nodes"][0]["links"] == [(False, 1, 0, 1)]
    assert net["nodes"][d + 1]["links"] == [(False, d, 2, 1)]
    ranks = [1] + x.ranks() + [1]
    for k in range(d):
        links = net["nodes"][k + 1]["links"]
        assert links[0] == (False, k, 0 if k == 0 else 2, ranks[k])
        assert links[1] == (True, 2 ** 64 - 1, k, [4, 5, 3, 6][k])
        assert links[2] == (False, k + 2, 0, ranks[k + 1])
        np.testing.assert_array_equal(net["nodes"][k + 1]["tensor"]["data"],
                                      x.get_component(k).to_ndarray().ravel())
    assert net["nodes"][0]["tensor"]["dims"] == [1] and net["nodes"][0]["tensor"]["data"][0] == 1.0


def test_factorisations(xe):
    rng = np.random.default_rng(11)
    a = rng.standard_normal((4, 5, 6, 3))
    A = _tensor(xe, a) * -2.0
    mat = -2.0 * a.reshape(20, 18)
    U, S, Vt = xe.calculate_svd(A, 2, 0, xe.EPSILON)
    u, s, vt = U.to_ndarray().reshape(20, -1), S.to_ndarray(), Vt.to_ndarray().reshape(-1, 18)
    np.testing.assert_allclose(u @ s @ vt, mat, rtol=0, atol=1e-12 * np.abs(mat).max())
    np.testing.assert_allclose(np.diag(s), np.linalg.svd(mat, compute_uv=False), rtol=1e-12)
    U, S, Vt = xe.calculate_svd(A, 2, 5, 0.0)
    assert S.dimensions == [5, 5] and U.dimensions == [4, 5, 5] and Vt.dimensions == [5, 6, 3]
    for name in ("qr", "qc"):
        Q, R = getattr(xe, "calculate_" + name)(A, 2)
        q = Q.to_ndarray().reshape(20, -1)
        np.testing.assert_allclose(q.T @ q, np.eye(q.shape[1]), atol=1e-13)
        np.testing.assert_allclose(q @ R.to_ndarray().reshape(q.shape[1], 18), mat, atol=1e-12 * np.abs(mat).max())
    for name in ("rq", "cq"):
        R, Q = getattr(xe, "calculate_" + name)(A, 2)
        q = Q.to_ndarray().reshape(-1, 18)
        np.testing.assert_allclose(q @ q.T, np.eye(q.shape[0]), atol=1e-13)
        np.testing.assert_allclose(R.to_ndarray().reshape(20, q.shape[0]) @ q, mat, atol=1e-12 * np.abs(mat).max())
    P = xe.pseudo_inverse(_tensor(xe, a.reshape(20, 18)), 1)
    np.testing.assert_allclose(P.to_ndarray(), np.linalg.pinv(a.reshape(20, 18)), atol=1e-12)


def test_qc_rank_reveals(xe):
    rng = np.random.default_rng(12)
    a = rng.standard_normal((30, 4)) @ rng.standard_normal((4, 25))
    Q, C = xe.calculate_qc(_tensor(xe, a), 1)
    assert Q.dimensions == [30, 4] and C.dimensions == [4, 25]


# ---------------------------------------------------------------------------------------------- TT
def test_tt_svd_roundtrip(xe):
    rng = np.random.default_rng(13)
    a = rng.standard_normal((4, 5, 3, 4))
    A = _tensor(xe, a)
    tt = xe.TTTensor(A)
    assert tt.ranks() == [4, 12, 4]
    np.testing.assert_allclose(xe.Tensor(tt).to_ndarray(), a, atol=1e-12)
    tt2 = xe.TTTensor(A, 0.0, 3)
    assert max(tt2.ranks()) <= 3
    assert tt.canonicalized and tt.corePosition == 0


def test_tt_random_matches_oracle(xe, ref):
    dims, ranks = [4, 5, 6, 5], [3, 7, 4]
    xe.seed(0xBAADF00D)
    x = xe.TTTensor.random_raw(dims, ranks)
    ox = ref.TT.random_raw(dims, ranks, ref.Rng(0xBAADF00D))
    for k in range(4):
        np.testing.assert_array_equal(x.get_component(k).to_ndarray(), ox.cores[k])
    full = xe.Tensor(x).to_ndarray()
    np.testing.assert_allclose(full, ox.full(), rtol=1e-12, atol=1e-12)


def test_tt_move_round_dot(xe):
    dims = [5, 6, 4, 7, 5]
    x = xe.TTTensor.random(dims, [4, 9, 9, 4])
    full = xe.Tensor(x).to_ndarray()
    nrm = np.linalg.norm(full)
    assert x.frob_norm() == pytest.approx(nrm, rel=1e-12)
    x.move_core(3)
    assert x.corePosition == 3
    np.testing.assert_allclose(xe.Tensor(x).to_ndarray(), full, atol=1e-12 * nrm)
    y = xe.TTTensor.random(dims, [3, 3, 3, 3])
    fy = xe.Tensor(y).to_ndarray()
    assert xe.dot(x, y) == pytest.approx(float((full * fy).sum()), abs=1e-10 * nrm * np.linalg.norm(fy))
    i = xe.Index()
    assert float(x(i & 0) * y(i & 0)) == pytest.approx(xe.dot(x, y), rel=1e-12)
    s = x + y
    np.testing.assert_allclose(xe.Tensor(s).to_ndarray(), full + fy, atol=1e-11 * nrm)
    assert max(s.ranks()) <= 12 and s.ranks()[0] <= 5
    s.round(12)                       # the sum has rank <= 12: rounding to 12 is exact
    np.testing.assert_allclose(xe.Tensor(s).to_ndarray(), full + fy, atol=1e-10 * nrm)
    s.round(1e-12)
    np.testing.assert_allclose(xe.Tensor(s).to_ndarray(), full + fy, atol=1e-10 * nrm)
    d = x - x
    d.move_core(0)
    assert d.frob_norm() <= 1e-12 * nrm
    assert xe.approx_equal(x, x * 1.0)


def test_tt_round_truncates_like_oracle(xe, ref):
    dims, ranks = [4, 5, 6, 5, 4], [4, 12, 12, 4]
    xe.seed(0xBAADF00D)
    x = xe.TTTensor.random_raw(dims, ranks)
    ox = ref.TT.random_raw(dims, ranks, ref.Rng(0xBAADF00D))
    x.round(3)
    ox.round([3, 3, 3, 3])
    assert x.ranks() == ox.ranks
    err_gpu = np.linalg.norm(xe.Tensor(x).to_ndarray() - ox.full())
    assert err_gpu <= 1e-8 * np.linalg.norm(ox.full())


@pytest.mark.parametrize("eps,max_rank", [(0.0, 0), (1e-3, 0), (0.05, 0), (0.0, 5), (1e-2, 7), (0.3, 0)])
def test_tt_svd_ranks_match_oracle(xe, ref, eps, max_rank):
    """TT-SVD constructor (ttNetwork.cpp:112-160): eps / maxRank cuts give the oracle's ranks, and the
    same tensor (the cut keeps the leading singular triplets; graded spectra keep gaps at the cuts)."""
    rng = np.random.default_rng(41)
    dims = [4, 5, 6, 5, 4]
    # a TT with geometrically decaying core scales: distinct, well separated singular values per edge
    ranks = [1, 4, 9, 9, 4, 1]
    cores = [rng.standard_normal((ranks[k], dims[k], ranks[k + 1])) for k in range(5)]
    for k in range(1, 5):
        cores[k] = cores[k] * (0.5 ** np.arange(ranks[k]))[:, None, None]
    full = ref.TT(cores).full()
    full = full + 1e-9 * rng.standard_normal(full.shape)
    mr = [max_rank] * 4   # oracle: 0 = no cap; the reference's default maxRank is size_t(-1)
    tt = xe.TTTensor(_tensor(xe, full), eps, max_rank if max_rank else 2**63)
    o = ref.tt_svd(full, eps, mr)
    assert tt.ranks() == o.ranks
    got = xe.Tensor(tt).to_ndarray()
    assert np.linalg.norm(got - o.full()) <= 1e-10 * np.linalg.norm(full)
