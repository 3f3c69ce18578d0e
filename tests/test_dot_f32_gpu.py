"""<x,y> on fp32 MFMA tiles (xrs_tt_dot_f32, dot32.hip) against the oracle's fp64 zipper (oracle/xerus_ref.py
dot, ttNetwork.cpp:782-789).

Tolerance: |d_f32 - d_ref| <= 1e-6 ||x|| ||y|| (the north star's fp32 bound); the fp32
roundings of the cores and of every product give ~1e-7. The environments are renormalised by powers of two
each step, so TTs whose norms leave the fp32 range (1e60 here) keep the same relative accuracy.
For independent random TTs |<x,y>| is itself ~1e-7 ||x|| ||y||, so that bar alone is weak: correlated pairs
y = x + 0.1 z (|<x,y>| ~ ||x|| ||y||) are checked relative to |<x,y>|, and cores
outside the fp32 zipper's range (every core x 1e-25 or 1e25) must still give the fp64 value
(the fp64 zipper takes over, dot32.hip).
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


@pytest.mark.parametrize("dims,ranks", [
    ([20] * 6, [20, 64, 64, 64, 20]),
    ([20] * 10, [20] + [128] * 7 + [20]),
    ([7, 3, 5, 4], [6, 9, 4]),
])
def test_dot_f32_correlated(handle, ref, dims, ranks):
    rng = ref.Rng(23)
    x = ref.TT.random_raw(dims, ranks, rng)
    z = ref.TT.random_raw(dims, ranks, rng)
    z.cores = [c * (0.1 if k == 0 else 1.0) for k, c in enumerate(z.cores)]
    y = ref.tt_add(x, z)                 # y = x + 0.1 z: <x, y> ~ ||x|| ||y||
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    assert abs(d_ref) > 0.5 * nx * ny
    d32 = gx.dot_f32(gy)
    assert abs(d32 - d_ref) <= 1e-6 * abs(d_ref), (d32, d_ref, abs(d32 - d_ref) / abs(d_ref))


@pytest.mark.parametrize("scale,d", [(1e-40, 3), (1e40, 3), (1e-25, 4), (1e25, 4), (1e9, 4), (1e-15, 4)])
def test_dot_f32_core_range(handle, ref, scale, d):
    """Both TTs' cores scaled: 1e+-40 lies outside the fp32 zipper's core range [2^-100, 2^100) and
    must come back as the fp64 result (the fp64 zipper takes over); 1e+-25, 1e9, 1e-15 lie inside and run in
    fp32 at fp32 accuracy (every product has one raw core and one power-of-two normalised operand)."""
    rng = ref.Rng(31)
    dims, ranks = [20] * d, [20] * (d - 1)
    x = ref.TT.random_raw(dims, ranks, rng)
    z = ref.TT.random_raw(dims, ranks, rng)
    y = ref.tt_add(x, z)
    x.cores = [c * scale for c in x.cores]
    y.cores = [c * scale for c in y.cores]
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    assert np.isfinite(d_ref) and d_ref != 0.0
    d32 = gx.dot_f32(gy)
    assert np.isfinite(d32) and d32 != 0.0
    tol = 1e-12 if scale in (1e-40, 1e40) else 1e-6
    assert abs(d32 - d_ref) <= tol * abs(d_ref), (d32, d_ref, abs(d32 - d_ref) / abs(d_ref))
