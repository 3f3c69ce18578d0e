"""Phase stamps of the fp32 GEMM (diagnostic build tools/sgstamps/libxerus_amd.so, -DXRS_SG_STAMPS): per workgroup
s_memtime at start / prologue done / main loop done / ticket done / end; printed as percentiles over the
workgroups of the LAST launch, relative to the earliest start.
    XRS_LIB_PATH=tools/sgstamps/libxerus_amd.so python tools/sgemm_stamps.py M N K TA TB [cfg,splits]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xerus_amd import capi  # noqa: E402

M, N, K, ta, tb = (int(a) for a in sys.argv[1:6])
if len(sys.argv) > 6:
    os.environ["XRS_SGEMM"] = sys.argv[6]
h = capi.Handle(0)
lib = h.lib
lib.xrs_debug_sg_stamps.argtypes = [C.c_void_p]
rng = np.random.default_rng(0)
A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
B = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
dA, dB, dC = h.array_f32(A), h.array_f32(B), capi.Float32Array(h, (M, N))
nwg = 4096
buf = h.zeros((8 * nwg,))
for rep in range(12):
    h.synchronize()
    lib.xrs_debug_sg_stamps(C.c_void_p(buf.ptr))
    h.gemm_f32(dC, M, N, 1.0, dA, A.shape[1], bool(ta), K, dB, B.shape[1], bool(tb))
    h.synchronize()
    lib.xrs_debug_sg_stamps(C.c_void_p(0))
st = buf.numpy().view(np.uint64).reshape(nwg, 8)
st = st[st[:, 0] != 0]
t0 = st[:, 0].min()
rel = (st[:, :5].astype(np.int64) - np.int64(t0))
print(f"{M}x{N}x{K} ta={ta} tb={tb} cfg={os.environ.get('XRS_SGEMM', 'auto')}: {len(st)} workgroups (cycles from the first start)")
names = ["start", "prologue", "mainloop", "ticket", "end"]
for i, nm in enumerate(names):
    col = rel[:, i]
    col = col[st[:, i] != 0]
    if len(col):
        print(f"  {nm:9s} p0 {np.percentile(col, 0):8.0f} p50 {np.percentile(col, 50):8.0f} p90 {np.percentile(col, 90):8.0f} max {col.max():8.0f}  (n={len(col)})")
d = st[:, 2].astype(np.int64) - st[:, 1].astype(np.int64)
print(f"  main loop per wg: p50 {np.median(d):.0f}  min {d.min()}  max {d.max()}")
d = st[:, 1].astype(np.int64) - st[:, 0].astype(np.int64)
print(f"  prologue per wg:  p50 {np.median(d):.0f}")
m = st[:, 4] != 0
if m.any():
    d = st[m, 4].astype(np.int64) - st[m, 3].astype(np.int64)
    print(f"  combine (last slices): p50 {np.median(d):.0f} max {d.max()}")
