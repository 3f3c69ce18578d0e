"""ADF (algorithms/adf.cpp) and the measurement operators on the GPU vs the oracle's restatement
(oracle/xerus_ref.py: adf, tt_measure_sp / tt_measure_r1) and the reference's own ADF tests
(src/unitTests/ttCompletion.cxx:107-145, adf_random_low_rank).

ADF is gauge-covariant: both sides start from the same cores and run the same sweeps, so the represented
tensors and the residual norms are compared (the cores' orthogonal gauge after move_core differs, as for
every factorisation). Rank increases draw TTTensor::random from the seeded stream on both sides.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tt_from(xe, cores):
    dims = [c.shape[1] for c in cores]
    x = xe.TTTensor(dims)
    for k, c in enumerate(cores):
        x.set_component(k, xe.Tensor.from_ndarray(np.ascontiguousarray(c)))
    return x


def _full(xe, x):
    return xe.Tensor(x).to_ndarray()


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _sp_set(xe, pos, vals):
    s = xe.SinglePointMeasurementSet()
    for p, v in zip(pos.tolist(), vals.tolist()):
        s.add(p, v)
    return s


def test_measure_tt_single_point(xe, ref):
    rng = ref.Rng(21)
    dims, ranks = [5, 4, 6, 3, 5], [3, 4, 4, 2]
    t = ref.TT.random_raw(dims, ranks, rng)
    pos = ref.sp_random_positions(rng, 200, dims)
    x = _tt_from(xe, t.cores)
    s = _sp_set(xe, pos, np.zeros(len(pos)))
    s.measure(x)
    want = ref.tt_measure_sp(t, pos)
    assert np.abs(np.asarray(s.measuredValues) - want).max() <= 1e-13 * np.abs(want).max()
    assert s.test(x) <= 1e-14
    full = t.full()
    assert np.allclose(want, full[tuple(pos.T)], rtol=1e-13, atol=1e-13 * np.abs(full).max())


def test_measure_tt_rank_one(xe, ref):
    rng = np.random.default_rng(22)
    dims, ranks = [4, 3, 5, 4], [2, 3, 2]
    t = ref.TT.random_raw(dims, ranks, ref.Rng(22))
    M = 60
    vecs = [rng.standard_normal((M, n)) for n in dims]
    r1 = xe.RankOneMeasurementSet()
    for m in range(M):
        r1.add([xe.Tensor.from_ndarray(vecs[k][m].copy()) for k in range(len(dims))], 0.0)
    x = _tt_from(xe, t.cores)
    r1.measure(x)
    want = ref.tt_measure_r1(t, vecs)
    assert np.abs(np.asarray(r1.measuredValues) - want).max() <= 1e-12 * np.abs(want).max()
    dense = xe.Tensor(x)
    r2 = xe.RankOneMeasurementSet(r1)
    r2.measure(dense)   # host path (measurments.cpp:369-391)
    assert np.abs(np.asarray(r2.measuredValues) - want).max() <= 1e-12 * np.abs(want).max()


@pytest.mark.parametrize("kind", ["sp", "r1"])
def test_adf_matches_oracle_fixed_rank(xe, ref, kind):
    """A fixed number of sweeps at fixed ranks (minimalResidualDecrease 1.0 never stops early): the same
    iterate and residual as the restatement."""
    rng = ref.Rng(31)
    D, N, R = 5, 4, 2
    true = ref.TT.random([N] * D, [R] * (D - 1), rng)
    pos = ref.sp_random_positions(rng, 300, [N] * D)
    vals = ref.tt_measure_sp(true, pos)
    x0 = ref.TT.random_raw([N] * D, [R] * (D - 1), rng)
    ox = x0.copy()
    x = _tt_from(xe, x0.cores)
    meas = _sp_set(xe, pos, vals)
    var = xe.ADFVariant(6, 1e-14, 1.0)
    if kind == "sp":
        res = var(x, meas)
        ores = ref.adf(ox, vals, [R] * (D - 1), positions=pos, max_iterations=6, target=1e-14, min_decrease=1.0)
    else:
        res = var(x, xe.RankOneMeasurementSet(meas, [N] * D))
        vecs = [np.eye(N)[pos[:, k]] for k in range(D)]
        ores = ref.adf(ox, vals, [R] * (D - 1), vectors=vecs, max_iterations=6, target=1e-14, min_decrease=1.0)
    assert x.ranks() == ox.ranks
    assert res == pytest.approx(ores, rel=1e-9)
    assert _rel(_full(xe, x), ox.full()) <= 1e-9


def test_adf_rank_increase_matches_oracle(xe, ref):
    """From TTTensor::ones with maxRanks 3: the rank-increase branch (x + 1e-6 ||x|| r / ||r||, round) with
    r drawn from the seeded stream on both sides; 12 sweeps in total."""
    rng = ref.Rng(41)
    D, N, R = 5, 4, 3
    true = ref.TT.random([N] * D, [R] * (D - 1), rng)
    pos = ref.sp_random_positions(rng, 400, [N] * D)
    vals = ref.tt_measure_sp(true, pos)
    meas = _sp_set(xe, pos, vals)
    x = xe.TTTensor.ones([N] * D)
    ox = ref.tt_ones([N] * D)
    seed = 4242
    xe.seed(seed)
    res = xe.ADFVariant(12, 1e-14, 0.999)(x, meas, [R] * (D - 1))
    ores = ref.adf(ox, vals, [R] * (D - 1), positions=pos, max_iterations=12, target=1e-14, min_decrease=0.999, rng=ref.Rng(seed))
    assert x.ranks() == ox.ranks
    assert res == pytest.approx(ores, rel=1e-7)
    assert _rel(_full(xe, x), ox.full()) <= 1e-7


@pytest.mark.parametrize("rank_one", [False, True])
def test_adf_random_low_rank(xe, rank_one):
    """Port of Algorithm:adf_random_low_rank (ttCompletion.cxx:107-145): D = 6, N = 5, R = 3, CS = 10
    random point measurements of a random rank-3 TT; ADF(500, 1e-6, 0.999) from TTTensor::ones with
    maxRanks 3 must recover it to 1e-3 (relative Frobenius error)."""
    D, N, R, CS = 6, 5, 3, 10
    xe.seed(0xBAADF00D)
    true = xe.TTTensor.random([N] * D, [R] * (D - 1))
    meas = xe.SinglePointMeasurementSet.random(D * N * CS * R * R, [N] * D)
    meas.measure(true)
    ft = _full(xe, true)
    vals = np.asarray(meas.measuredValues)
    assert np.abs(vals - ft[tuple(np.asarray(meas.positions).T)]).max() <= 1e-12 * np.abs(ft).max()
    x = xe.TTTensor.ones([N] * D)
    m = xe.RankOneMeasurementSet(meas, [N] * D) if rank_one else meas
    xe.ADFVariant(500, 1e-6, 0.999)(x, m, [R] * (D - 1))
    assert _rel(_full(xe, x), ft) < 1e-3
