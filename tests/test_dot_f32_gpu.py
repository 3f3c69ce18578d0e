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
    # the fused zipper (zip32.hip): heads only (d = 4), one end without a step (d = 5), uneven step counts
    # (d = 7), the headline shape at other scales (per-unit T exponents, exponent words)
    ([20] * 4, [20, 128, 20], 1.0),
    ([8] * 5, [8, 64, 64, 8], 1.0),
    ([10] * 7, [10, 96, 96, 96, 96, 10], 1.0),
    ([20] * 10, [20] + [256] * 7 + [20], 1e5),
    ([20] * 10, [20] + [256] * 7 + [20], 1e-5),
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


@pytest.mark.parametrize("scale,d", [(1e-40, 3), (1e40, 3), (1e-25, 4), (1e25, 4), (1e9, 4), (1e-15, 4),
                                     (1e-12, 6), (1e12, 6), (1e9, 6), (1e-15, 6)])
def test_dot_f32_core_range(handle, ref, scale, d):
    """Both TTs' cores scaled (d = 6 through the fused zipper's fp32 steps, where 1e+-40 would leave
    the fp64 range of the reference value itself): 1e+-40 lies outside the fp32 zipper's core range [2^-100, 2^100) and
    must come back as the fp64 result (the fp64 zipper takes over); 1e+-25, 1e9, 1e-15 lie inside and run in
    fp32 at fp32 accuracy (every product has one raw core and one power-of-two normalised operand)."""
    rng = ref.Rng(31)
    # d = 6: ranks 20 / 64 (x + z: 40 / 128), the fused zipper's heads and fp32 steps (zip32.hip)
    dims, ranks = [20] * d, ([20] * (d - 1) if d < 6 else [20] + [64] * (d - 3) + [20])
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


def test_dot_f32_fused_matches_per_product_form(ref):
    """The three forms of the fp32 zipper, each in its own process (the switch is read once): the default
    (dot32.hip's per-product launches), XRS_ZIP32=1 (zip32.hip's fused front end, then per-product steps) and
    XRS_ZIP32=2 (fused steps throughout). Cases: the headline shape, heads only (d = 4), one end without a step
    (d = 5), uneven step counts (d = 7), correlated pairs scaled by 1e+-12 (d = 6: fp32 steps, exponent words) and
    cores outside [2^-100, 2^100) (fp64 fallback, exact). All within the fp32 bar, bitwise repeatable."""
    import json
    import os
    import subprocess
    import sys

    code = r"""
import json, sys
sys.path.insert(0, %r)
import numpy as np
from oracle import xerus_ref as ref
from xerus_amd import capi
h = capi.Handle(0)
out = []
cases = [([20] * 10, [20] + [256] * 7 + [20], 1.0, 0), ([10] * 7, [10, 96, 96, 96, 96, 10], 1.0, 0),
         ([20] * 4, [20, 128, 20], 1.0, 0), ([8] * 5, [8, 64, 64, 8], 1.0, 0),
         ([20] * 6, [20, 64, 64, 64, 20], 1e12, 1), ([20] * 6, [20, 64, 64, 64, 20], 1e-12, 1),
         ([20] * 6, [20, 64, 64, 64, 20], 1.0, 2)]
for dims, ranks, scale, kind in cases:
    rng = ref.Rng(77)
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    if kind == 1:                      # correlated pair, every core scaled
        y = ref.tt_add(x, y)
        x.cores = [c * scale for c in x.cores]
        y.cores = [c * scale for c in y.cores]
    if kind == 2:                      # one core above, one below the fp32 zipper's range
        x.cores[2] = x.cores[2] * 2.0 ** 110
        x.cores[3] = x.cores[3] * 2.0 ** -110
    gx, gy = capi.TTDevice.from_cores(h, x.cores), capi.TTDevice.from_cores(h, y.cores)
    a, b = gx.dot_f32(gy), gx.dot_f32(gy)
    d_ref = ref.dot(x, y)
    nn = float(np.sqrt(ref.dot(x, x) * ref.dot(y, y)))
    out.append([a, b, d_ref, nn, kind, gx.dot(gy)])
print(json.dumps(out))
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for flag in ("0", "1", "2"):
        env = dict(os.environ, XRS_ZIP32=flag)
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        for a, b, d_ref, nn, kind, d64 in json.loads(p.stdout.strip().splitlines()[-1]):
            assert a == b, (flag, kind)
            if kind == 2:
                assert a == d64, (flag, a, d64)
            elif kind == 1:
                assert abs(a - d_ref) <= 1e-6 * abs(d_ref), (flag, a, d_ref)
            else:
                assert abs(a - d_ref) <= 1e-6 * nn, (flag, a, d_ref, nn)


def test_dot_f32_fused_core_out_of_range(handle, ref):
    """One core of x scaled by 2^110 and another by 2^-110 (the TT unchanged up to rounding): the fused zipper
    (d = 6, fp32 steps) sees a core outside [2^-100, 2^100) and returns the fp64 zipper's value."""
    rng = ref.Rng(37)
    dims, ranks = [20] * 6, [20, 64, 64, 64, 20]
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    x.cores[2] = x.cores[2] * 2.0 ** 110
    x.cores[3] = x.cores[3] * 2.0 ** -110
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d64, d32 = gx.dot(gy), gx.dot_f32(gy)
    assert d32 == d64
