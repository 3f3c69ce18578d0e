"""GPU parity of the TT hot path (move_core, round, <x,y>, frob_norm) against the oracle.

Tolerances (BASELINE.md §3 / SURVEY §8(d)): inner products |d_gpu - d_ref| <= 1e-6 ||x|| ||y||;
non-truncating round: identical ranks and ||T(gpu) - T(ref)|| <= 1e-6 ||T(x)||; truncating round:
identical ranks and truncation errors equal to 1e-6 ||x||. The path is fp64 throughout, so the tests
also assert the much tighter rounding-level bounds the implementation actually reaches.
"""
import numpy as np
import pytest

from xerus_amd import capi

pytestmark = pytest.mark.gpu


def _tt_diff_norm(ref, a_cores, b_cores):
    """(||A - B||, ||B||) for two TTs without cancellation: the difference TT (block-diagonal sum
    with -B) is orthogonalised by the oracle (move_core(0), backward stable) and its norm read off the
    core, so the result is accurate to ~u*||B|| instead of the sqrt(u) floor of <A,A>-2<A,B>+<B,B>."""
    A = ref.TT([c.copy() for c in a_cores])
    B = ref.TT([c.copy() for c in b_cores])
    nb = [c.copy() for c in B.cores]
    nb[0] = -nb[0]
    D = ref.tt_add(A, ref.TT(nb))
    D.move_core(0)
    B.move_core(0)
    return D.frob_norm(), B.frob_norm()


@pytest.mark.parametrize("dims,ranks", [
    ([4, 5, 3, 4, 2], [3, 6, 5, 2]),
    ([3, 4, 5, 4, 3, 4, 5], [4, 6, 8, 6, 4, 3]),   # odd order: the two-ended zipper's left end idles once
    ([6, 5, 7, 4], [5, 9, 4]),                      # smallest two-ended order
    ([7, 3, 5], [6, 4]),                            # one-ended (d < 4)
    ([20] * 6, [16] * 5),
    ([20] * 10, [128] * 9),   # cfg3 shape
    ([20] * 12, [256] * 11),  # cfg4 shape
])
def test_dot(handle, ref, dims, ranks):
    rng = ref.Rng(3)
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    d_gpu = gx.dot(gy)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    assert abs(d_gpu - d_ref) <= 1e-12 * nx * ny
    assert abs(gx.dot(gx) - nx * nx) <= 1e-12 * nx * nx
    # <x, x> on the same cores takes the symmetric environments (gemm_sym); a copy of x (other pointers)
    # takes the general products: both the same value to rounding, the async form bitwise the sync one
    gx2 = capi.TTDevice.from_cores(handle, x.cores)
    assert abs(gx.dot(gx) - gx.dot(gx2)) <= 1e-13 * nx * nx
    if len(dims) >= 4:
        assert gx.dot_async(gx).result() == gx.dot(gx)
    # the asynchronous form runs the same two-ended zipper on the side streams: bitwise the same value
    # from order 4 on (below, the synchronous form is one-ended)
    d_async = gx.dot_async(gy).result()
    assert d_async == d_gpu if len(dims) >= 4 else abs(d_async - d_ref) <= 1e-12 * nx * ny


@pytest.mark.parametrize("dims,ranks", [
    ([4, 5, 3, 4, 2], [3, 6, 5, 2]),
    ([7, 3, 5], [6, 4]),
    ([5, 6], [4]),
    ([20] * 10, [128] * 9),
])
def test_dot_async_beside_round(handle, ref, dims, ranks):
    """x.dot_async(y) overlapped with x.round (which replaces x's cores): the inner product is the one of
    the pre-round x (the round's releases wait for it), the round is unaffected, and the handle accepts
    the next async call only after the wait."""
    rng = ref.Rng(11)
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_seq = gx.dot(gy)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    assert abs(d_seq - ref.dot(x, y)) <= 1e-12 * nx * ny
    target = max(1, max(ranks) // 2)
    for _ in range(3):
        fut = gx.dot_async(gy)
        with pytest.raises(capi.XrsError):
            gx.dot_async(gy)   # one in flight per handle
        before = [c.copy() for c in gx.cores()] if _ == 0 else None
        gx.round(target)
        d = fut.result()
        if _ == 0:
            assert d == d_seq if len(dims) >= 4 else abs(d - d_seq) <= 1e-13 * nx * ny
            ox = ref.TT([c.copy() for c in before])
            ox.round(target)
            assert gx.r == [1] + list(ox.ranks) + [1]
            e_ref, nrm = _tt_diff_norm(ref, ox.cores, before)
            e_gpu, _ = _tt_diff_norm(ref, gx.cores(), before)
            assert abs(e_gpu - e_ref) <= 1e-6 * nrm
        # next iteration: <x_rounded, y> against the synchronous zipper on the same cores
        assert abs(gx.dot_async(gy).result() - gx.dot(gy)) <= 1e-13 * nx * ny
    with pytest.raises(capi.XrsError):
        capi._check("xrs_tt_dot_wait", handle.lib.xrs_tt_dot_wait(handle.h, capi.C.byref(capi.C.c_double())))


@pytest.mark.parametrize("write", ["scal", "axpy", "copy", "upload", "gemm"])
def test_dot_async_fences_in_place_writes(handle, ref, write):
    """x.dot_async(y), then an in-place write into one of x's live cores through the C-ABI: the write
    waits for the in-flight product (fence_readers), so result() is the pre-write <x,y>."""
    rng = ref.Rng(31)
    dims, ranks = [20] * 8, [64] * 7
    x = ref.TT.random_raw(dims, ranks, rng)
    y = ref.TT.random_raw(dims, ranks, rng)
    gx = capi.TTDevice.from_cores(handle, x.cores)
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_before = gx.dot(gy)
    k = 3
    size = gx.r[k] * gx.dims[k] * gx.r[k + 1]
    core = capi.DeviceArray(handle, (size,), ptr=gx.ptrs[k], owned=False)
    other = handle.array(np.full(size, 0.5))
    fut = gx.dot_async(gy)
    if write == "scal":
        handle.scal(core, -3.0)
    elif write == "axpy":
        handle.axpy(core, 2.0, other)
    elif write == "copy":
        capi._check("xrs_copy", handle.lib.xrs_copy(handle.h, capi._DP(core.ptr), capi._DP(other.ptr), size))
    elif write == "upload":
        z = np.zeros(size)
        capi._check("xrs_upload", handle.lib.xrs_upload(handle.h, capi._DP(core.ptr), z.ctypes.data_as(capi._DP), size))
    else:
        a = handle.array(np.eye(gx.r[k]))
        b = handle.array(np.ones((gx.r[k], gx.dims[k] * gx.r[k + 1])))
        handle.gemm(core, gx.r[k], gx.dims[k] * gx.r[k + 1], 1.0, a, gx.r[k], False, gx.r[k], b, gx.dims[k] * gx.r[k + 1], False)
    assert fut.result() == d_before
    assert gx.dot(gy) != d_before   # the write did happen


@pytest.mark.parametrize("dims,ranks", [([4, 5, 3, 4, 2], [3, 6, 5, 2]), ([3, 3, 3, 3], [9, 9, 9]),
                                        ([20] * 6, [40] * 5), ([20] * 8, [128] * 7)])
def test_random_move_core_left(handle, ref, dims, ranks):
    """TTTensor::random = raw N(0,1) cores + move_core(0) (ttNetwork.h:129-157)."""
    rng = ref.Rng()
    x = ref.TT.random_raw(dims, ranks, rng)
    g = capi.TTDevice.from_cores(handle, x.cores)
    y = x.copy()
    y.move_core(0)
    g.move_core(0)
    assert g.ranks == y.ranks
    gc = g.cores()
    for c in gc[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.linalg.norm(M @ M.T - np.eye(M.shape[0])) <= 1e-12 * M.shape[0]
    diff, nrm = _tt_diff_norm(ref, gc, y.cores)
    assert diff <= 1e-12 * nrm


def test_move_core_right_and_back(handle, ref):
    rng = ref.Rng(5)
    x = ref.TT.random([6, 5, 4, 7, 3], [4, 8, 8, 3], rng)
    g = capi.TTDevice.from_cores(handle, x.cores, canonicalized=True, core_position=0)
    g.move_core(3)
    y = x.copy()
    y.move_core(3)
    assert g.ranks == y.ranks
    gc = g.cores()
    for c in gc[:3]:
        M = c.reshape(-1, c.shape[2])
        assert np.linalg.norm(M.T @ M - np.eye(M.shape[1])) <= 1e-12 * M.shape[1]
    diff, nrm = _tt_diff_norm(ref, gc, y.cores)
    assert diff <= 1e-12 * nrm
    assert abs(g.frob_norm() - y.frob_norm()) <= 1e-12 * nrm


@pytest.mark.parametrize("dims,ranks", [([4, 5, 3, 4, 2], [3, 6, 5, 2]), ([20] * 6, [40] * 5),
                                        ([20] * 10, [128] * 9)])
def test_round_non_truncating(handle, ref, dims, ranks):
    rng = ref.Rng(11)
    x = ref.TT.random(dims, ranks, rng)
    g = capi.TTDevice.from_cores(handle, x.cores, canonicalized=True, core_position=0)
    y = x.copy()
    y.round(max(ranks))
    g.round(max(ranks))
    assert g.ranks == y.ranks == x.ranks
    gc = g.cores()
    diff, nrm = _tt_diff_norm(ref, gc, x.cores)
    assert diff <= 1e-10 * nrm          # bar: 1e-6
    for c in gc[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.linalg.norm(M @ M.T - np.eye(M.shape[0])) <= 1e-12 * M.shape[0]


@pytest.mark.parametrize("dims,ranks,target", [([4, 5, 3, 4, 2], [3, 6, 5, 2], 2), ([6] * 5, [20] * 4, 7),
                                               ([20] * 6, [40] * 5, 17), ([20] * 10, [128] * 9, 64)])
def test_round_truncating(handle, ref, dims, ranks, target):
    rng = ref.Rng(13)
    x = ref.TT.random(dims, ranks, rng)
    g = capi.TTDevice.from_cores(handle, x.cores, canonicalized=True, core_position=0)
    y = x.copy()
    y.round(target)
    g.round(target)
    assert g.ranks == y.ranks
    if min(dims) >= 6:   # generic inputs take the certified device-resident truncation
        assert handle.last_round_path() == "truncate"
    e_ref, nrm = _tt_diff_norm(ref, y.cores, x.cores)
    e_gpu, _ = _tt_diff_norm(ref, g.cores(), x.cores)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm
    gc = g.cores()
    for c in gc[1:]:   # right-canonical result
        M = c.reshape(c.shape[0], -1)
        assert np.abs(M @ M.T - np.eye(M.shape[0])).max() <= 1e-12


@pytest.mark.parametrize("dims,ranks,target", [([20] * 10, [128] * 9, 128), ([20] * 8, [64] * 7, 40),
                                               ([6, 5, 7, 4, 6], [6, 12, 12, 6], 10)])
def test_round_sum_truncating(handle, ref, dims, ranks, target):
    """(x + y).round(r): doubled ranks with structural excess at both ends (r_1 = 2 n_0 > n_0): the
    reference's QC drops the left end exactly, the right end goes through the tall-edge SVD; same ranks
    and truncation error as the oracle's round of the same sum."""
    from ttutil import tt_diff_norm

    rng = ref.Rng(61)
    x = ref.TT.random(dims, ranks, rng)
    y = ref.TT.random(dims, ranks, rng)
    s = ref.tt_add(x, y)
    g = capi.TTDevice.from_cores(handle, [c.copy() for c in s.cores])
    g.round(target)
    path = handle.last_round_path()
    o = s.copy()
    o.round(target)
    assert g.ranks == o.ranks
    e_gpu, nrm = tt_diff_norm(g.cores(), s.cores)
    e_ref, _ = tt_diff_norm(o.cores, s.cores)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm, (e_gpu / nrm, e_ref / nrm, path)
    assert path == "truncate"


def test_round_sum_recovers_ranks(handle, ref):
    """x + x has doubled ranks; round() must cut them back (SVD eps rule, tensor.cpp:1469-1474)."""
    rng = ref.Rng(17)
    x = ref.TT.random([5, 4, 6, 3, 5], [4, 7, 6, 3], rng)
    s = ref.tt_add(x, x)
    g = capi.TTDevice.from_cores(handle, s.cores)
    y = s.copy()
    y.round(100)
    g.round(100)
    assert g.ranks == y.ranks == x.ranks
    diff, nrm = _tt_diff_norm(ref, g.cores(), [2 * c if i == 0 else c for i, c in enumerate(x.cores)])
    assert diff <= 1e-10 * nrm


@pytest.mark.parametrize("edge", [1, 3])
def test_round_certificate_fails_mid_sweep(handle, ref, edge):
    """The right unfolding of one interior core is rank-deficient: the certified right-to-left sweep
    (ranks within maxRank, left Grams well conditioned) must hand over to the reference's two-sweep
    algorithm at that edge and reproduce the reference's rank drop."""
    rng = ref.Rng(19)
    dims, ranks = [5, 5, 5, 5, 5], [4, 6, 6, 4]
    x = ref.TT.random_raw(dims, ranks, rng)
    c = x.cores[edge]
    a = c.shape[0]
    M = c.reshape(a, -1)
    U, S, Vt = np.linalg.svd(M, full_matrices=False)
    S[2:] = 0.0
    x.cores[edge] = ((U * S) @ Vt).reshape(c.shape)
    g = capi.TTDevice.from_cores(handle, [cc.copy() for cc in x.cores])
    y = x.copy()
    y.round(6)
    g.round(6)
    assert g.ranks == y.ranks
    assert g.ranks[edge - 1] == 2   # internal ranks: bond (edge-1, edge)
    diff, nrm = _tt_diff_norm(ref, g.cores(), x.cores)
    assert diff <= 1e-10 * nrm


def test_round_bench_shape(handle, ref):
    """The benched configuration (order 10, n = 20, rank 256): certified path, exact ranks, same tensor."""
    rng = ref.Rng(23)
    x = ref.TT.random_raw([20] * 10, [256] * 9, rng)
    g = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g.move_core(0)
    r0 = g.ranks
    g.round(256)
    assert g.ranks == r0
    gc = g.cores()
    for c in gc[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.linalg.norm(M @ M.T - np.eye(M.shape[0])) <= 1e-12 * M.shape[0]
    diff, nrm = _tt_diff_norm(ref, gc, x.cores)
    assert diff <= 1e-10 * nrm


@pytest.mark.parametrize("ranks", [[20, 400, 400, 20], [20, 300, 300, 20]])
def test_round_ranks_above_256(handle, ref, ranks):
    """Edges with 256 < r <= 512 factor through the 2 x 2-block Cholesky (factor_big): certified path,
    exact ranks, right-orthonormal cores, same tensor as the input."""
    rng = ref.Rng(29)
    x = ref.TT.random_raw([20] * 5, ranks, rng)
    g = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g.round(512)
    assert g.ranks == ranks
    gc = g.cores()
    for c in gc[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.abs(M @ M.T - np.eye(M.shape[0])).max() <= 1e-13
    diff, nrm = _tt_diff_norm(ref, gc, x.cores)
    assert diff <= 1e-10 * nrm


def test_tt_errors(handle, ref):
    rng = ref.Rng(1)
    x = ref.TT.random([3, 3, 3], [2, 2], rng)
    g = capi.TTDevice.from_cores(handle, x.cores, canonicalized=True, core_position=0)
    with pytest.raises(capi.XrsError):
        g.round([0, 2])
    with pytest.raises(capi.XrsError):
        g.move_core(5)


def test_round_many_edges_above_256(handle, ref):
    """Order 25, rank 300: 22 edges with 256 < r <= 512 need 66 factor_big jobs in the certified pass,
    more than one argument table holds (kBigMax = 64): the jobs go out in chunks."""
    import bench
    from ttutil import tt_diff_norm

    d, n, r = 25, 20, 300
    ranks = bench.tt_ranks(d, n, r)[1:-1]
    assert sum(1 for q in ranks if q > 256) == 22
    x = ref.TT.random_raw([n] * d, ranks, ref.Rng(53))
    g = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g.round(r)
    y = x.copy()
    y.round(r)
    assert g.ranks == y.ranks == ranks
    diff, nrm = tt_diff_norm(g.cores(), x.cores)
    assert diff <= 1e-10 * nrm


@pytest.mark.parametrize("n,ranks", [(30, [30, 600, 600, 30]), (40, [40, 1024, 40])])
def test_round_ranks_above_512(handle, ref, n, ranks):
    """Ranks above 512: blocked Cholesky with explicit inverses (chol_full) in the certified chain round,
    the 8-row / 1024-column block Jacobi in the truncating round, blocked CholeskyQR2 in move_core.
    Same tensor and exact ranks without a cut; the oracle's ranks and truncation error with one."""
    d = len(ranks) + 1
    x = ref.TT.random_raw([n] * d, ranks, ref.Rng(61))
    g = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g.round(max(ranks))
    assert g.ranks == ranks
    assert handle.last_round_path() == "chain"
    gc = g.cores()
    for c in gc[1:]:
        M = c.reshape(c.shape[0], -1)
        assert np.abs(M @ M.T - np.eye(M.shape[0])).max() <= 1e-12
    diff, nrm = _tt_diff_norm(ref, gc, x.cores)
    assert diff <= 1e-10 * nrm
    # move the core to the end and back (QR sweeps through the > 512 unfoldings)
    g.move_core(d - 1)
    g.move_core(0)
    diff, _ = _tt_diff_norm(ref, g.cores(), x.cores)
    assert diff <= 1e-10 * nrm
    # truncating round to half the largest rank
    target = max(ranks) // 2
    g2 = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    g2.round(target)
    y = x.copy()
    y.round(target)
    assert g2.ranks == y.ranks
    assert handle.last_round_path() == "truncate"
    e_ref, _ = _tt_diff_norm(ref, y.cores, x.cores)
    e_gpu, _ = _tt_diff_norm(ref, g2.cores(), x.cores)
    assert abs(e_gpu - e_ref) <= 1e-6 * nrm


@pytest.mark.parametrize("edge", [None, 1])
def test_dot_async_beside_fallback_round(handle, ref, edge):
    """x.dot_async(y) before a round whose first certificate fails (x + x: doubled ranks; or a
    rank-deficient interior core): the round falls back (truncating / sequential paths), which open the
    product's gate at their own chain pass or at the first release; the product is still the one of the
    pre-round x and the round is the reference's."""
    rng = ref.Rng(23)
    if edge is None:
        x0 = ref.TT.random([5, 4, 6, 3, 5], [4, 7, 6, 3], rng)
        x = ref.tt_add(x0, x0)
        target = 100
    else:
        x = ref.TT.random_raw([5, 5, 5, 5, 5], [4, 6, 6, 4], rng)
        c = x.cores[edge]
        U, S, Vt = np.linalg.svd(c.reshape(c.shape[0], -1), full_matrices=False)
        S[2:] = 0.0
        x.cores[edge] = ((U * S) @ Vt).reshape(c.shape)
        target = 6
    y = ref.TT.random_raw(x.dims, x.ranks, rng)
    gx = capi.TTDevice.from_cores(handle, [c.copy() for c in x.cores])
    gy = capi.TTDevice.from_cores(handle, y.cores)
    d_ref = ref.dot(x, y)
    nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
    fut = gx.dot_async(gy)
    gx.round(target)
    assert abs(fut.result() - d_ref) <= 1e-12 * nx * ny
    ox = x.copy()
    ox.round(target)
    assert gx.ranks == ox.ranks
