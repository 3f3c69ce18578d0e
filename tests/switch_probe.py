"""Subprocess body of tests/test_switches_gpu.py: a fixed set of GPU computations run under the environment
switch being tested (the library reads its XRS_* switches once per process). Prints one JSON line of
results (errors against numpy / the oracle, round paths, <x,y> values); test infrastructure only."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle import xerus_ref as ref  # noqa: E402
from ttutil import tt_diff_norm  # noqa: E402
from xerus_amd import capi  # noqa: E402


def main():
    h = capi.Handle(0)
    out = {}
    rng = np.random.default_rng(7)
    # GEMMs: a TT-chain shape (LDS-DMA pipeline eligible) and an odd shape (general kernel)
    errs = []
    for (m, n, k) in ((256, 5120, 256), (300, 170, 1000)):
        A, B = rng.standard_normal((m, k)), rng.standard_normal((k, n))
        dA, dB, dC = h.array(A), h.array(B), h.empty((m, n))
        h.gemm(dC, m, n, 1.0, dA, k, False, k, dB, n, False)
        E = A @ B
        errs.append(float(np.abs(dC.numpy() - E).max() / np.abs(E).max()))
    out["gemm_err"] = max(errs)
    # fp32 split-K product (xrs_gemm_f32; XRS_SG_TARGET moves its slice count)
    A32 = rng.standard_normal((5120, 256)).astype(np.float32)
    B32 = rng.standard_normal((5120, 256)).astype(np.float32)
    dA, dB, dC = h.array_f32(A32), h.array_f32(B32), capi.Float32Array(h, (256, 256))
    h.gemm_f32(dC, 256, 256, 1.0, dA, 256, True, 5120, dB, 256, False)
    E = A32.astype(np.float64).T @ B32.astype(np.float64)
    out["sgemm_err"] = float(np.linalg.norm(dC.numpy() - E) / np.linalg.norm(E))
    for d in (dA, dB, dC):
        d.free()
    # <x,y> synchronous and asynchronous (the gate)
    dims, ranks = [10] * 6, [10, 40, 40, 40, 10]
    x = ref.TT.random_raw(dims, ranks, ref.Rng(3))
    y = ref.TT.random_raw(dims, ranks, ref.Rng(4))
    gx, gy = capi.TTDevice.from_cores(h, x.cores), capi.TTDevice.from_cores(h, y.cores)
    nxy = np.sqrt(ref.dot(x, x) * ref.dot(y, y))
    d_ref = ref.dot(x, y)
    out["dot_err"] = abs(gx.dot(gy) - d_ref) / nxy
    out["dot_async_err"] = abs(gx.dot_async(gy).result() - d_ref) / nxy
    # fp32 <x,y> (xrs_tt_dot_f32; ranks divisible by 4 so that XRS_ZIP32 can pick the fused zipper, whose
    # per-workgroup stamps XRS_ZIP_STAMPS prints)
    x4 = ref.TT.random_raw(dims, [8, 32, 32, 32, 8], ref.Rng(13))
    y4 = ref.TT.random_raw(dims, [8, 32, 32, 32, 8], ref.Rng(14))
    g4x, g4y = capi.TTDevice.from_cores(h, x4.cores), capi.TTDevice.from_cores(h, y4.cores)
    out["dot32_err"] = abs(g4x.dot_f32(g4y) - ref.dot(x4, y4)) / np.sqrt(ref.dot(x4, x4) * ref.dot(y4, y4))
    # non-truncating round (the certified chain)
    gc = capi.TTDevice.from_cores(h, x.cores)
    gc.round(40)
    out["chain_path"] = h.last_round_path()
    e, nrm = tt_diff_norm(gc.cores(), x.cores)
    out["chain_err"] = e / nrm
    # truncating round of a random TT (certified truncation) and of a graded one (general path)
    xt = ref.TT.random(dims, ranks, ref.Rng(5))
    g = capi.TTDevice.from_cores(h, xt.cores, canonicalized=True, core_position=0)
    g.round(17)
    out["trunc_path"] = h.last_round_path()
    o = xt.copy()
    o.round(17)
    e_gpu, nrm = tt_diff_norm(g.cores(), xt.cores)
    e_ref, _ = tt_diff_norm(o.cores, xt.cores)
    out["trunc_ranks_ok"] = g.ranks == o.ranks
    out["trunc_err_diff"] = abs(e_gpu - e_ref) / nrm
    xg = ref.TT.random_raw(dims, ranks, ref.Rng(6))
    for k in range(len(dims) - 1):
        xg.cores[k] = xg.cores[k] * (0.7 ** np.arange(xg.cores[k].shape[2]))[None, None, :]
    gg = capi.TTDevice.from_cores(h, [c.copy() for c in xg.cores])
    gg.round(12)
    out["graded_path"] = h.last_round_path()
    og = xg.copy()
    og.round(12)
    e_gpu, nrm = tt_diff_norm(gg.cores(), xg.cores)
    e_ref, _ = tt_diff_norm(og.cores, xg.cores)
    out["graded_ranks_ok"] = gg.ranks == og.ranks
    out["graded_err_diff"] = abs(e_gpu - e_ref) / nrm
    # flat spectra cut inside the cluster (repeated singular values): x has cores that are left- AND
    # right-orthonormal, so every edge's singular values are all 1; x + x has edge spectra {2 (r times), 0} and its
    # left end is structurally rank deficient (the exact QC steps; on the GPU it ends on the reference's sweep);
    # round(r / 2) cuts inside the cluster. The kept subspace of the first cut is arbitrary within the cluster and
    # the later edges' spectra depend on it, so only the ranks and the TT-SVD quasi-optimality (each error within
    # sqrt(d - 1) of the other's) are comparable with the oracle -- not the error itself
    fr, fn, fd = 10, 10, 6
    frng = np.random.default_rng(11)
    fc = [np.linalg.qr(frng.standard_normal((fn, fr)))[0].reshape(1, fn, fr)]
    for _ in range(fd - 2):
        fc.append(np.stack([np.linalg.qr(frng.standard_normal((fr, fr)))[0] for _ in range(fn)], axis=1) / np.sqrt(fn))
    fc.append(np.linalg.qr(frng.standard_normal((fn, fr)))[0].T.reshape(fr, fn, 1))
    xs = ref.tt_add(ref.TT(fc), ref.TT([c.copy() for c in fc]))
    gf = capi.TTDevice.from_cores(h, [c.copy() for c in xs.cores])
    gf.round(fr // 2)
    out["flat_path"] = h.last_round_path()
    of = xs.copy()
    of.round(fr // 2)
    e_gpu, nrm = tt_diff_norm(gf.cores(), xs.cores)
    e_ref, _ = tt_diff_norm(of.cores, xs.cores)
    out["flat_ranks_ok"] = gf.ranks == of.ranks
    out["flat_err_gpu"], out["flat_err_ref"] = e_gpu / nrm, e_ref / nrm
    q = np.sqrt(fd - 1.0) * (1.0 + 1e-8)
    out["flat_err_ok"] = bool(e_gpu <= q * e_ref and e_ref <= q * e_gpu)
    # the block Jacobi right singular vectors (xrs_svd_rows_vt) and the eigensolver entry (xrs_sym_eig_top)
    W = rng.standard_normal((64, 96))
    S, Vt, sweeps = h.svd_rows_vt(h.array(W))
    out["svd_err"] = float(np.abs(S.numpy() - np.linalg.svd(W, compute_uv=False)).max() / np.linalg.norm(W, 2))
    # the dense API SVD (square: the bidiagonal route unless XRS_SVD_BIDIAG=0)
    Ad = rng.standard_normal((96, 96))
    Ua, Sa, Va = (x.numpy() for x in h.svd(h.array(Ad)))
    out["api_svd_res"] = float(np.linalg.norm((Ua * Sa) @ Va - Ad) / np.linalg.norm(Ad))
    out["api_svd_orth"] = float(max(np.abs(Ua.T @ Ua - np.eye(96)).max(), np.abs(Va @ Va.T - np.eye(96)).max()))
    P = W @ W.T
    lam, Ut, st = h.sym_eig_top(h.array(P), 8)
    out["eig_err"] = float(np.abs(lam.numpy() - np.linalg.eigvalsh(P)[::-1][:8]).max() / np.linalg.norm(P, 2))
    h.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
