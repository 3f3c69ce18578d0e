"""Backward errors of the factorisations on the GPU vs LAPACK (numpy/scipy) at the reference tests' shapes.

Diagnostics only (run on the GPU box): python tools/accuracy_probe.py
"""
import os
import sys

import numpy as np
from scipy.linalg import lapack

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
rng = np.random.default_rng(0)


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


print("shape           svd_gpu    svd_lapack  orthU_gpu  orthV_gpu   qc_gpu    cq_gpu    qr_lapack")
for m, n in [(1000, 10), (10, 1000), (100, 100), (90, 64), (64, 90), (128, 128), (30, 64), (256, 256), (512, 512)]:
    A = rng.standard_normal((m, n))
    dA = h.array(A)
    U, S, Vt = h.svd(dA)
    U, S, Vt = U.numpy(), S.numpy(), Vt.numpy()
    e_svd = rel((U * S) @ Vt, A)
    u2, s2, vt2, _ = lapack.dgesdd(A)
    e_lap = rel((u2[:, :len(s2)] * s2) @ vt2[:len(s2)], A)
    k = min(m, n)
    oU = np.abs(U.T @ U - np.eye(k)).max()
    oV = np.abs(Vt @ Vt.T - np.eye(k)).max()
    Q, Cm, r = h.qc(dA)
    e_qc = rel(Q.numpy() @ Cm.numpy(), A)
    Cc, Qq, r2 = h.cq(dA)
    e_cq = rel(Cc.numpy() @ Qq.numpy(), A)
    q, rr = np.linalg.qr(A)
    e_qr = rel(q @ rr, A)
    print(f"{m:4d}x{n:<5d}  {e_svd:9.2e}  {e_lap:9.2e}  {oU:9.2e}  {oV:9.2e}  {e_qc:9.2e}  {e_cq:9.2e}  {e_qr:9.2e}")

import xerus_amd.xerus as xe  # noqa: E402

xe.seed(0xBAADF00D)
for dims in ([10, 10, 10, 10], [5, 6, 3, 1, 4, 2, 8, 1], [2] * 8):
    B = xe.Tensor.random(dims)
    b = B.to_ndarray()
    tt = xe.TTTensor(B, 1e-14) if dims[0] != 10 else xe.TTTensor(B)
    e0 = rel(xe.Tensor(tt).to_ndarray(), b)
    z = xe.TTTensor(xe.Tensor(dims))
    s = tt + z
    e1 = rel(xe.Tensor(s).to_ndarray(), b)
    tt2 = tt.__copy__()
    tt2.move_core(tt2.degree() - 1)
    e2 = rel(xe.Tensor(tt2).to_ndarray(), b)
    print(f"TT {dims}: ranks {tt.ranks()} tt-svd {e0:.2e}  +zero {e1:.2e} ranks {s.ranks()}  move_core(d-1) {e2:.2e}")
