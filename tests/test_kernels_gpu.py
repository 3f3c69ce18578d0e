"""GPU parity of the level-1/3 and permutation kernels against the oracle (through the C-ABI)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PERMS = [
    ((64, 64, 64), (0, 2, 1)),            # cfg1's C reshuffle
    ((64, 64, 64), (2, 1, 0)),
    ((256, 20, 256), (1, 0, 2)),          # contiguous block kept
    ((256, 20, 256), (2, 1, 0)),
    ((1, 1, 256, 20, 256), (0, 1, 3, 4, 2)),  # cfg4 zipper reshuffle
    ((1, 1, 256, 256), (0, 1, 3, 2)),
    ((1024, 1024), (1, 0)),
    ((20, 20, 20, 20, 20, 20), (5, 4, 3, 2, 1, 0)),
    ((3, 5, 7, 11), (2, 0, 3, 1)),
    ((2, 3, 4, 5, 6), (4, 2, 0, 1, 3)),
    ((33, 65), (1, 0)),                   # ragged tiles
    ((3, 128, 192), (0, 2, 1)),           # 64 x 64 16-B tiles, batched
    ((192, 5, 64), (2, 1, 0)),            # 64 x 64 tiles with an odd batch stride (16-B path off)
    ((1, 7, 1), (2, 1, 0)),
    ((5,), (0,)),
    ((0, 4), (1, 0)),                     # empty
    ((4, 1, 3, 1, 2), (3, 0, 4, 1, 2)),
]


@pytest.mark.parametrize("dims,shuffle", PERMS)
def test_permute_bit_exact(handle, ref, dims, shuffle):
    a = np.random.default_rng(11).standard_normal(dims)
    d = handle.array(a)
    out = handle.reshuffle(d, shuffle).numpy()
    expect = ref.reshuffle(a, shuffle)
    assert out.shape == expect.shape
    assert np.array_equal(out, expect)


def test_permute_all_orders_small_modes(handle, ref):
    """Every permutation of a 5-mode tensor with small, unequal modes (the grouped-mode transpose path:
    groups of innermost input / output modes, ragged flattened extents), bit-exact against the oracle."""
    import itertools

    dims = (3, 5, 2, 7, 4)
    a = np.random.default_rng(5).standard_normal(dims)
    d = handle.array(a)
    for shuffle in itertools.permutations(range(5)):
        out = handle.reshuffle(d, shuffle).numpy()
        assert np.array_equal(out, ref.reshuffle(a, shuffle)), shuffle


@pytest.mark.parametrize("dims,shuffle", [((20, 20, 20, 20), (3, 2, 1, 0)), ((6, 40, 6, 40), (1, 3, 0, 2)),
                                          ((9, 9, 9, 9, 9), (4, 0, 3, 1, 2)), ((2, 300, 3, 17), (3, 1, 0, 2))])
def test_permute_grouped_shapes(handle, ref, dims, shuffle):
    a = np.random.default_rng(6).standard_normal(dims)
    out = handle.reshuffle(handle.array(a), shuffle).numpy()
    assert np.array_equal(out, ref.reshuffle(a, shuffle))


def test_permute_rejects_bad_shuffle(handle):
    from xerus_amd.capi import XrsError

    d = handle.array(np.zeros((2, 3)))
    o = handle.empty((3, 2))
    with pytest.raises(XrsError):
        handle.permute(o, d, (2, 3), (0, 0))


GEMMS = [
    (64, 64, 4096, False, False),    # cfg1 GEMM
    (1024, 1024, 1024, False, False),  # cfg2
    (256, 5120, 256, True, False),   # TT zipper step 1
    (256, 256, 5120, True, False),   # TT zipper step 2 (split-K)
    (5120, 256, 256, False, False),  # R * core
    (256, 256, 5120, False, True),   # Gram of a wide core
    (128, 2560, 128, True, True),
    # whole-tile shapes of the LDS-DMA pipeline (k_gemm_glds): 64x80 / 80x64 / 64x64 / 32x32 tiles, every
    # transpose combination
    (256, 5120, 256, False, False), (256, 5120, 256, False, True), (5120, 256, 256, True, True),
    (5120, 256, 256, True, False), (512, 10240, 512, False, False), (320, 640, 96, True, False),
    (64, 160, 64, False, True), (96, 96, 64, True, True),
    (1, 37, 19, False, False), (37, 1, 19, True, False), (13, 17, 1, False, True),
    (100, 3, 7, True, True), (129, 131, 67, False, False), (65, 63, 2000, True, True),
]


@pytest.mark.parametrize("M,N,K,ta,tb", GEMMS)
def test_gemm_fp64(handle, ref, M, N, K, ta, tb):
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    A = rng.standard_normal((K, M) if ta else (M, K))
    B = rng.standard_normal((N, K) if tb else (K, N))
    alpha = -1.75
    dA, dB = handle.array(A), handle.array(B)
    Cd = handle.matmul(dA, ta, dB, tb, alpha).numpy()
    expect = ref.gemm(A, ta, B, tb, alpha)
    err = np.linalg.norm(Cd - expect) / max(np.linalg.norm(expect), 1e-300)
    assert err <= 1e-13, err  # fp64 MFMA: relative Frobenius error at rounding level


BATCHED = [
    (9, 256, 256, 5120, False, True),    # chain-round check Grams (split-K, in-launch combine)
    (7, 5120, 256, 256, False, False),   # right-factor transforms
    (7, 256, 5120, 256, False, False),   # left-factor transforms
    (3, 256, 256, 5120, True, False),
    (5, 33, 65, 700, True, True),        # ragged tiles
    (40, 64, 64, 64, False, False),      # more entries than one launch holds (32)
    (4, 64, 128, 256, False, False),     # 2 tiles x 4 entries x 2 split-K slices, small slabs: the in-launch combine
    (4, 64, 128, 256, True, True),       # under the XCD-grouped (entry, slice) order, a non-identity remap (r05: the
                                         # combine's own slice is the remapped one, not blockIdx.z)
    (1, 17, 19, 23, False, False),
]


@pytest.mark.parametrize("cnt,M,N,K,ta,tb", BATCHED)
def test_gemm_batched_fp64(handle, ref, cnt, M, N, K, ta, tb):
    """xrs_gemm_batched: every entry matches the GEMM oracle and the single-GEMM path (tile choice may differ)."""
    rng = np.random.default_rng(cnt * 1000 + M + N + K)
    As = [rng.standard_normal((K, M) if ta else (M, K)) for _ in range(cnt)]
    Bs = [rng.standard_normal((N, K) if tb else (K, N)) for _ in range(cnt)]
    dA = [handle.array(a) for a in As]
    dB = [handle.array(b) for b in Bs]
    dC = [handle.empty((M, N)) for _ in range(cnt)]
    lda = M if ta else K
    ldb = K if tb else N
    handle.gemm_batched(dC, M, N, 0.5, dA, lda, ta, K, dB, ldb, tb)
    for i in range(cnt):
        got = dC[i].numpy()
        expect = ref.gemm(As[i], ta, Bs[i], tb, 0.5)
        err = np.linalg.norm(got - expect) / max(np.linalg.norm(expect), 1e-300)
        assert err <= 1e-13, (i, err)
    single = handle.matmul(dA[0], ta, dB[0], tb, 0.5).numpy()
    assert np.linalg.norm(single - dC[0].numpy()) <= 1e-13 * np.linalg.norm(single)


SYMS = [
    (256, 5120, True, False),   # chain Gram M^T T (split-K, two-kernel reduce)
    (256, 5120, False, True),   # right chain / check Gram M T^T
    (20, 400, True, False),     # edge core
    (100, 3000, False, True),   # ragged tiles across the diagonal
    (512, 10240, False, True),  # cfg5
    (33, 17, True, False),
    (48, 6000, True, False),    # 16 x 16 tiled reduce over 32 x 32 GEMM tiles (N not a tile multiple)
    (160, 8192, False, True),   # tiled reduce, 55 slices (two chunks)
]


@pytest.mark.parametrize("N,K,ta,tb", SYMS)
def test_gemm_sym_fp64(handle, ref, N, K, ta, tb):
    """xrs_gemm_sym on M^T G M / X X^T products: exactly symmetric, equal to the GEMM oracle."""
    rng = np.random.default_rng(N + K)
    X = rng.standard_normal((K, N) if ta else (N, K))
    G = rng.standard_normal((K, K)) if K <= 1000 else None
    if G is not None:   # B = G X (K x N) with G symmetric: op(A) op(B) = X^T (G_s X) is symmetric
        Gs = G + G.T
        A = X
        B = (Gs @ X) if ta else (X @ Gs)
    else:
        A = B = X
    dA, dB, dC = handle.array(A), handle.array(B), handle.empty((N, N))
    lda = A.shape[1]
    ldb = B.shape[1]
    handle.gemm_sym(dC, N, 0.5, dA, lda, ta, K, dB, ldb, tb)
    got = dC.numpy()
    expect = ref.gemm(A, ta, B, tb, 0.5)
    assert np.array_equal(got, got.T)
    err = np.linalg.norm(got - expect) / np.linalg.norm(expect)
    assert err <= 1e-13, err


def test_gemm_zero_k(handle):
    dA, dB = handle.array(np.zeros((3, 0))), handle.array(np.zeros((0, 4)))
    out = handle.empty((3, 4))
    handle.gemm(out, 3, 4, 1.0, dA, 1, False, 0, dB, 4, False)
    assert np.array_equal(out.numpy(), np.zeros((3, 4)))


def test_level1(handle):
    rng = np.random.default_rng(5)
    x, y = rng.standard_normal(100003), rng.standard_normal(100003)
    dx, dy = handle.array(x), handle.array(y)
    assert np.isclose(handle.nrm2(dx), np.linalg.norm(x), rtol=1e-14)
    assert np.isclose(handle.dot(dx, dy), x @ y, rtol=1e-12)
    assert np.isclose(handle.asum(dx), np.abs(x).sum(), rtol=1e-14)
    handle.scal(dx, 2.5)
    assert np.allclose(dx.numpy(), 2.5 * x, rtol=0, atol=0)
    handle.axpy(dy, -0.5, dx)
    assert np.allclose(dy.numpy(), y - 0.5 * (2.5 * x), rtol=1e-15, atol=1e-15)
    M = rng.standard_normal((37, 53))
    s = rng.standard_normal(37)
    dM = handle.array(M)
    handle.scale_rows(dM, handle.array(s))
    assert np.array_equal(dM.numpy(), M * s[:, None])
