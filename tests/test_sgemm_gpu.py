"""fp32-MFMA GEMM (xrs_gemm_f32, sgemm_impl.hpp) against the oracle's matrix product (oracle/xerus_ref.py gemm:
blasWrapper::matrix_matrix_product, blasLapackWrapper.cpp:149-195) evaluated in fp64 on the same fp32 inputs.

Tolerance: relative Frobenius error <= 1e-6 (the north star's bound; the fp32 products and sums give
~1e-7 at K <= 5120). Every tile configuration of the kernel family is reached by the shapes below (auto
selection: 128x128 for large grids, 64x80 / 80x64 for the TT zipper's wide / tall shapes, 64x64 with split-K
for r x r Grams, 32x32 for small outputs), with all four transposition pairs, the scalar staging path
(ragged extents, unaligned pointers) and the in-launch split-K combine.
"""
import numpy as np
import pytest

from xerus_amd import capi

pytestmark = pytest.mark.gpu


def _run(handle, ref, M, N, K, ta, tb, alpha=1.0, seed=0, offset=0):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    dA, dB = capi.Float32Array.from_host(handle, A, offset), capi.Float32Array.from_host(handle, B, offset)
    dC = capi.Float32Array(handle, (M, N))
    handle.gemm_f32(dC, M, N, alpha, dA, A.shape[1], ta, K, dB, B.shape[1], tb)
    got = dC.numpy()
    expect = ref.gemm(A.astype(np.float64), ta, B.astype(np.float64), tb, alpha)
    err = np.linalg.norm(got - expect) / max(np.linalg.norm(expect), 1e-300)
    # deterministic: a second call gives the same bits
    handle.gemm_f32(dC, M, N, alpha, dA, A.shape[1], ta, K, dB, B.shape[1], tb)
    same = np.array_equal(dC.numpy(), got)
    for d in (dA, dB, dC):
        d.free()
    return err, same


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [
    (1024, 1024, 1024),   # BASELINE configs[1]: 64x64 tiles, one per CU
    (2048, 2048, 96),     # 128x128 tiles
    (256, 5120, 256),     # zipper T = E^T X_k shape: 64x80 tiles
    (5120, 256, 256),     # right-end T = X_k F: 80x64 tiles
    (256, 256, 5120),     # environment product: 64x64 tiles, 16-way split-K, in-launch combine
    (20, 20, 400),        # rank-20 zipper step: 32x32 tile, split-K
])
def test_gemm_f32_shapes(handle, ref, M, N, K, ta, tb):
    err, same = _run(handle, ref, M, N, K, ta, tb, seed=M + N + K)
    assert err <= 1e-6, err
    assert same


@pytest.mark.parametrize("M,N,K", [(33, 70, 129), (1, 1, 1), (5, 7, 3), (97, 65, 1000), (130, 2, 77)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, True), (True, False)])
def test_gemm_f32_ragged(handle, ref, M, N, K, ta, tb):
    err, same = _run(handle, ref, M, N, K, ta, tb, alpha=-0.75, seed=7)
    assert err <= 1e-6, err
    assert same


def test_gemm_f32_unaligned_and_alpha(handle, ref):
    # an operand one float past a 16-B boundary takes the scalar staging path
    err, same = _run(handle, ref, 256, 320, 96, False, False, alpha=2.5, offset=1)
    assert err <= 1e-6, err
    assert same


def test_gemm_f32_k0_and_errors(handle):
    A = capi.Float32Array.from_host(handle, np.ones((4, 1), np.float32))
    B = capi.Float32Array.from_host(handle, np.ones((1, 3), np.float32))
    C = capi.Float32Array.from_host(handle, np.full((4, 3), 7.0, np.float32))
    handle.gemm_f32(C, 4, 3, 1.0, A, 1, False, 0, B, 3, False)   # K = 0: C = 0 (beta = 0)
    assert np.array_equal(C.numpy(), np.zeros((4, 3), np.float32))
    with pytest.raises(capi.XrsError):
        handle.gemm_f32(C, 4, 3, 1.0, A, 0, False, 1, B, 3, False)   # lda < K
    with pytest.raises(capi.XrsError):
        handle.gemm_f32(C, 4, 3, 1.0, C, 3, False, 3, B, 3, False)   # C aliases A
