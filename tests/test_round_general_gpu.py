"""The truncating TT round on inputs the certified paths refuse, at BASELINE cfg3 size (order 10, n = 20,
r = 128), against the oracle (the reference's two-sweep algorithm on LAPACK, oracle/xerus_ref.py:
TTNetwork::round ttNetwork.cpp:644-684 -> round_edge tensorNetwork.cpp:678-818).

Inputs (seeded):
  graded  -- raw N(0,1) cores whose right rank index is scaled by 0.8^j: every edge unfolding has a
             decaying spectrum (kappa ~ 1e12 at the rank-128 edges), so no Gram-based certificate holds;
  sum     -- x + 1e-6 y with x, y random rank-128 TTs (rank 256, a 1e-6 tail).
Bars (BASELINE.md §3 / SURVEY §8(d)): identical ranks; truncation errors agree to 1e-6 ||x||. The
round's path is asserted so that these tests pin the general (non-certified) algorithm.
"""
import numpy as np
import pytest

from xerus_amd import capi

pytestmark = pytest.mark.gpu

EPSILON = 8 * np.finfo(float).eps


def graded_tt(ref, dims, ranks, decay, seed):
    x = ref.TT.random_raw(dims, ranks, ref.Rng(seed))
    for k in range(len(dims) - 1):
        b = x.cores[k].shape[2]
        x.cores[k] = x.cores[k] * (decay ** np.arange(b))[None, None, :]
    return x


def sum_tt(ref, dims, ranks, scale, seed):
    rng = ref.Rng(seed)
    x = ref.TT.random(dims, ranks, rng)
    y = ref.TT.random(dims, ranks, rng)
    y.cores[0] = y.cores[0] * scale
    return ref.tt_add(x, y)


def _check(handle, ref, x, max_ranks, eps, allowed_paths):
    from ttutil import tt_diff_norm

    g = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g.round(max_ranks, eps)
    path = handle.last_round_path()
    o = x.copy()
    o.round(max_ranks, eps)
    assert g.ranks == o.ranks, (g.ranks, o.ranks, path)
    e_gpu, nrm = tt_diff_norm(g.cores(), x.cores)
    e_ref, _ = tt_diff_norm(o.cores, x.cores)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm, (e_gpu / nrm, e_ref / nrm, path)
    assert path in allowed_paths, path
    for c in g.cores()[1:]:   # right-canonical result (core at 0)
        M = c.reshape(c.shape[0], -1)
        assert np.abs(M @ M.T - np.eye(M.shape[0])).max() <= 1e-10
    return g, o, path


CFG3 = ([20] * 10, [128] * 9)


def test_graded_round64(handle, ref):
    """round(64) of a graded-spectrum TT at cfg3 size: the maxRank cut on a decaying spectrum."""
    x = graded_tt(ref, *CFG3, decay=0.8, seed=101)
    _check(handle, ref, x, [64] * 9, EPSILON, ("general",))


def test_graded_round_eps(handle, ref):
    """round(1e-8) (eps only, maxRank = inf) of the graded TT: the eps rule sigma_j <= 1e-8 sigma_0 decides
    every rank; the singular values near the cut must be accurate to far better than sqrt(u)."""
    x = graded_tt(ref, *CFG3, decay=0.8, seed=102)
    g, o, _ = _check(handle, ref, x, [2 ** 62] * 9, 1e-8, ("general",))
    assert max(o.ranks) < 128   # the eps rule did cut


def test_sum_round64(handle, ref):
    """round(64) of x + 1e-6 y (ranks 256 with a 1e-6 tail at cfg3 size)."""
    x = sum_tt(ref, *CFG3, scale=1e-6, seed=103)
    _check(handle, ref, x, [64] * 9, EPSILON, ("general", "truncate"))


def test_sum_round_eps(handle, ref):
    """round(1e-7) of x + 1e-6 y: the eps rule removes y's contribution edge by edge."""
    x = sum_tt(ref, *CFG3, scale=1e-9, seed=104)
    g, o, _ = _check(handle, ref, x, [2 ** 62] * 9, 1e-7, ("general", "truncate"))
    assert o.ranks == [20] + [128] * 7 + [20]


@pytest.mark.parametrize("dims,ranks,max_rank,eps", [
    ([4, 5, 3, 4, 2], [3, 6, 5, 2], 3, 1e-3),
    ([6] * 6, [20] * 5, 9, 1e-10),
    ([20] * 6, [40] * 5, 100, 1e-6),
    ([3] * 8, [9] * 7, 4, EPSILON),
])
def test_graded_small(handle, ref, dims, ranks, max_rank, eps):
    """Small graded TTs (boundary ranks, tall and wide edges, maxRank and eps cuts together)."""
    x = graded_tt(ref, dims, ranks, decay=0.7, seed=105 + len(dims))
    _check(handle, ref, x, [max_rank] * (len(dims) - 1), eps, ("general", "reference", "truncate", "chain"))


def test_reference_path_ranks_above_512(handle, ref):
    """A graded TT with ranks 600 (both sides of the middle edges above 512): the general path covers ranks
    up to 512, so the reference's sequential sweep runs (tall / wide edge factors up to 1024 through the
    block Jacobi); same ranks and truncation error as the oracle."""
    x = graded_tt(ref, [30, 30, 30, 30], [600, 600, 600], decay=0.97, seed=121)
    _check(handle, ref, x, [400] * 3, EPSILON, ("reference", "truncate"))


def direct_sum_tt(ref, x, xp):
    """z = x (+) x' as a TT: every mode index doubled, z = x on the first halves, x' on the second halves,
    0 elsewhere; block-diagonal cores, so every edge unfolding is blockdiag(X_k, X'_k) and its singular
    values are the union of x's and x''s (each one twice for x' = x)."""
    d = x.order if hasattr(x, "order") else len(x.cores)
    cores = []
    for k in range(d):
        A, B = x.cores[k], xp.cores[k]
        a, n, b = A.shape
        a2, n2, b2 = B.shape
        ra = 1 if k == 0 else a + a2
        rb = 1 if k == d - 1 else b + b2
        Z = np.zeros((ra, n + n2, rb))
        Z[:a, :n, :b] = A
        Z[ra - a2:, n:, rb - b2:] = B
        cores.append(Z)
    return ref.TT(cores)


@pytest.mark.parametrize("scale,target", [(1.0, 8), (1.0, 10), (1.0 + 1e-9, 7), (1.0 + 1e-9, 10)])
def test_clustered_edge_spectra(handle, ref, scale, target):
    """Every edge Gram with eigenvalues in exact (scale 1) or close (1e-9 apart) pairs: z = x (+) s x. The
    exact pairs are kept or cut whole (even targets: the kept subspace is unique); the close pairs are also
    cut between their members. Inverse iteration inside a cluster must keep its vectors orthogonal. Same
    ranks and truncation error as the oracle, right-orthonormal cores to 1e-10, whichever path runs."""
    x = ref.TT.random([6] * 6, [6] * 5, ref.Rng(131))
    xs = x.copy()
    xs.cores[0] = xs.cores[0] * scale
    z = direct_sum_tt(ref, x, xs)
    assert z.ranks == [12] * 5
    _, _, path = _check(handle, ref, z, [target] * 5, EPSILON, ("truncate", "general", "reference"))
    print(f"clustered spectra scale {scale} target {target}: path {path}")


@pytest.mark.parametrize("max_rank,eps", [(2, 1e-6), (4, 1e-6), (2, EPSILON)])
def test_tall_right_end_after_cut(handle, ref, max_rank, eps):
    """x + y with graded spectra at mode size 3 (ranks [3,5,5,5,3] each, so the sum's right end is tall:
    r_5 = 6 > 3, r_4 = 10 > 3 * 3). Cutting edge 5 below its working rank leaves zero columns in the tall
    unfolding of core 4; the general round factors its Gram with those columns masked (k_pad_diag) instead
    of failing its Cholesky certificate and falling back to the reference's sweep. Same ranks and error as
    the oracle; with the eps cut (which the certified truncation refuses) the general path is the one that
    ran, with the maxRank cut alone the certified truncation may take it."""
    rng = ref.Rng(141)
    x = ref.TT.random_raw([3] * 6, [3, 5, 5, 5, 3], rng)
    y = ref.TT.random_raw([3] * 6, [3, 5, 5, 5, 3], rng)
    for t in (x, y):
        for k in range(5):
            b = t.cores[k].shape[2]
            t.cores[k] = t.cores[k] * (0.5 ** np.arange(b))[None, None, :]
    z = ref.tt_add(x, y)
    assert z.ranks == [6, 10, 10, 10, 6]
    _check(handle, ref, z, [max_rank] * 5, eps, ("general",) if eps > EPSILON else ("general", "truncate"))
