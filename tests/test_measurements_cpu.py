"""CPU: measurement-set bookkeeping of the C++ host API (measurments.cpp) -- host-only code, no GPU call.

SinglePointMeasurementSet::random draws its positions from misc::randomEngine with one
std::uniform_int_distribution per mode (measurments.cpp:211-236); the oracle restates libstdc++'s
uniform_int_distribution on the bit-exact mt19937_64 stream (oracle/xerus_ref.py:uniform_index), so the
seeded positions must be identical, in the reference's sorted order.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def xe_host():
    import xerus_amd.xerus as module

    return module


@pytest.mark.parametrize("num,dims,seed", [(50, [4, 5, 3], 0xBAADF00D), (300, [10] * 4, 7), (64, [2] * 6, 11)])
def test_random_positions_match_reference_stream(xe_host, ref, num, dims, seed):
    xe_host.seed(seed)
    s = xe_host.SinglePointMeasurementSet.random(num, dims)
    got = np.asarray(s.positions)
    want = ref.sp_random_positions(ref.Rng(seed), num, dims)
    assert got.shape == (num, len(dims))
    assert np.array_equal(got, want)
    assert s.size() == num and s.degree() == len(dims)
    assert s.measuredValues == [0.0] * num


def test_add_sort_norm(xe_host):
    s = xe_host.SinglePointMeasurementSet()
    pts = [([2, 1], 3.0), ([0, 4], -1.0), ([2, 0], 2.0), ([1, 1], 0.5)]
    for p, v in pts:
        s.add(p, v)
    s.sort()
    assert s.positions == [[0, 4], [1, 1], [2, 0], [2, 1]]
    assert s.measuredValues == [-1.0, 0.5, 2.0, 3.0]
    assert s.frob_norm() == pytest.approx(np.sqrt(1 + 0.25 + 4 + 9), rel=1e-15)
    with pytest.raises(RuntimeError):
        s.add([1, 2, 3], 1.0)   # wrong degree


def test_impossible_request(xe_host):
    with pytest.raises(RuntimeError):
        xe_host.SinglePointMeasurementSet.random(10, [3, 3])
