"""<x,y> on fp32 MFMA tiles (xrs_tt_dot_f32, dot32.hip) against the oracle's fp64 zipper (oracle/xerus_ref.py
dot, ttNetwork.cpp:782-789).

Tolerance: |d_f32 - d_ref| <= 1e-6 ||x|| ||y|| (the north star's fp32 bound); the fp32
roundings of the cores and of every product give ~1e-7. The environments are renormalised by powers of two
each step, so TTs whose norms leave the fp32 range (1e60 here) keep the same relative accuracy.
"""
import numpy as np
import pytest

from xerus_amd import capi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dims,ranks,scale", [
    ([5, 6], [4], 1.0),                              # d = 2: one core per end
    ([7, 3, 5], [6, 4], 1.0),                        # odd order, ragged ranks (partial 64-tiles)
    ([4, 5, 3, 4, 2], [3, 6, 5, 2], 1.0),
    ([20] * 6, [70, 90, 33, 129, 65], 1.0),           # ranks straddling the 64-wide tiles
    ([20] * 10, [20] + [256] * 7 + [20], 1.0),       # the bench's headline TT shape (cfg3 ranks)
    ([20] * 12, [256] * 11, 1.0),                    # cfg4 shape
    ([20] * 10, [64] * 9, 1e6),                      # ||x|| ~ 1e66: beyond fp32 without the renormalisation
    ([20] * 10, [64] * 9, 1e-6),                     # ||x|| ~ 1e-54
])
def test_dot_f32(handle, ref, dims, ranks, scale):
    rng = ref.Rng(11)
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    x.cores = [c * scale for c in x.cores]
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    d32 = gx.dot_f32(gy)
    assert np.isfinite(d32)
    assert abs(d32 - d_ref) <= 1e-6 * nx * ny, (d32, d_ref, nx * ny)
    # deterministic: fixed split-K slice order, fixed closing-sum order
    assert gx.dot_f32(gy) == d32
    # <x,x> (a positive quantity) to fp32 relative accuracy
    assert abs(gx.dot_f32(gx) - nx * nx) <= 1e-6 * nx * nx


def test_dot_f32_zero_and_errors(handle, ref):
    rng = ref.Rng(5)
    x = ref.TT.random_raw([6, 7, 5, 4], [5, 6, 3], rng)
    z = [np.zeros_like(c) for c in x.cores]
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gz = capi.TTDevice.from_cores(handle, z)
    assert gx.dot_f32(gz) == 0.0
    g1 = capi.TTDevice.from_cores(handle, [np.ones((1, 6, 1))])
    with pytest.raises(RuntimeError):
        g1.dot_f32(g1)   # one component: the two-ended zipper needs d >= 2
