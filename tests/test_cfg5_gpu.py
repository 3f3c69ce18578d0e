"""BASELINE configs[4] on one GPU: TTTensor order 16, n = 20, rank 512 (ranks [20, 400, 512 x 11, 400, 20],
487.5 MB of cores) -- round(512), truncating round(256) and <x,y> against the oracle.

Bars: non-truncating round: identical ranks and ||T(gpu) - T(ref)|| <= 1e-10 ||T|| (the
survey's bar is 1e-6); truncating round: identical ranks and truncation errors equal to 1e-6 ||x||;
<x,y> within 1e-12 ||x|| ||y||. Norms of TT differences are computed without cancellation: the
difference TT is left-orthogonalised with Householder QR (numpy, backward stable) and the norm read off
the last core; the oracle's own pivoted QR is too slow for rank-1024 differences.
"""
import time

import numpy as np
import pytest

import bench
from ttutil import tt_diff_norm
from xerus_amd import capi

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

D, N, R = 16, 20, 512


@pytest.fixture(scope="module")
def cfg5(ref):
    ranks = bench.tt_ranks(D, N, R)[1:-1]
    x = ref.TT.random_raw([N] * D, ranks, ref.Rng(5))
    return x


def test_cfg5_round_512_matches_oracle(handle, ref, cfg5):
    x = cfg5
    g = capi.TTDevice.from_cores(handle, x.cores)
    t0 = time.time()
    g.round(R)
    handle.synchronize()
    t_gpu = time.time() - t0
    y = x.copy()
    y.round(R)
    assert g.ranks == y.ranks == x.ranks
    gc = g.cores()
    diff, nrm = tt_diff_norm(gc, x.cores)
    assert diff <= 1e-10 * nrm, diff / nrm
    diff_ref, _ = tt_diff_norm(gc, y.cores)
    assert diff_ref <= 1e-10 * nrm, diff_ref / nrm
    for c in gc[1:]:   # right-canonical result (core at 0)
        M = c.reshape(c.shape[0], -1)
        assert np.abs(M @ M.T - np.eye(M.shape[0])).max() <= 1e-12
    print(f"cfg5 round(512): gpu {t_gpu * 1e3:.1f} ms (first call), rel diff {diff / nrm:.2e}")


def test_cfg5_truncating_round_256(handle, ref, cfg5):
    x = cfg5
    g = capi.TTDevice.from_cores(handle, x.cores)
    g.round(256)
    y = x.copy()
    y.round(256)
    assert g.ranks == y.ranks
    e_gpu, nrm = tt_diff_norm(g.cores(), x.cores)
    e_ref, _ = tt_diff_norm(y.cores, x.cores)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm, (e_gpu / nrm, e_ref / nrm)


def test_cfg5_dot(handle, ref, cfg5):
    x = cfg5
    y = ref.TT.random_raw([N] * D, x.ranks, ref.Rng(6))
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    assert abs(gx.dot(gy) - d_ref) <= 1e-12 * nx * ny
    assert abs(gx.dot(gx) - nx * nx) <= 1e-12 * nx * nx
