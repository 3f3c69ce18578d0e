"""Workgroup timeline of the TT-shaped GEMMs (diagnostic; needs tools/trace/libxerus_amd.so from
`make -C tools trace/libxerus_amd.so`, i.e. gemm.hip built with -DXRS_GEMM_TRACE).

python tools/gemm_trace.py  ->  per shape: kernel span, workgroup durations, workgroups per CU, how many
ran concurrently on one CU, and when the last workgroup started (s_memrealtime, 10 ns ticks)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("XRS_LIB_PATH", os.path.join(ROOT, "tools", "trace", "libxerus_amd.so"))
sys.path.insert(0, ROOT)
from xerus_amd import capi  # noqa: E402

SHAPES = [  # (M, N, K, ta, tb, sym, what)
    (256, 5120, 256, 0, 0, 0, "E X (NN wide)"),
    (5120, 256, 256, 0, 0, 0, "M H (NN tall)"),
    (256, 256, 5120, 1, 0, 1, "Gram M^T T (TN sym)"),
    (256, 256, 5120, 0, 1, 1, "Gram M T^T (NT sym)"),
]
MAXWG = 1 << 16
h = capi.Handle(0)
lib = h.lib
lib.xrs_debug_gemm_trace.restype = C.c_int
lib.xrs_debug_gemm_trace.argtypes = [C.c_void_p, C.c_void_p]
rng = np.random.default_rng(0)
tbuf = h.zeros((3 * MAXWG,))
sbuf = h.zeros((16 * MAXWG,))
for M, N, K, ta, tb, sym, what in SHAPES:
    A = h.array(rng.standard_normal((K, M) if ta else (M, K)))
    B = h.array(rng.standard_normal((N, K) if tb else (K, N)))
    Cm = h.empty((M, N))
    if sym:
        call = lambda: h.gemm_sym(Cm, M, 1.0, A, A.shape[1], bool(ta), K, B, B.shape[1], bool(tb))  # noqa: E731
    else:
        call = lambda: h.gemm(Cm, M, N, 1.0, A, A.shape[1], bool(ta), K, B, B.shape[1], bool(tb))  # noqa: E731
    for _ in range(20):
        call()
    h.synchronize()
    for rep in range(3):
        lib.xrs_memset_zero(h.h, capi._DP(tbuf.ptr), tbuf.size)
        lib.xrs_memset_zero(h.h, capi._DP(sbuf.ptr), sbuf.size)
        assert lib.xrs_debug_gemm_trace(C.c_void_p(tbuf.ptr), C.c_void_p(sbuf.ptr)) == 0
        call()
        h.synchronize()
        assert lib.xrs_debug_gemm_trace(None, None) == 0
        call()   # untraced neighbour, keeps the cache state of a chain
        h.synchronize()
        t = tbuf.numpy().view(np.uint64).reshape(-1, 3)
        t = t[t[:, 0] != 0]
        t0 = t[:, 0].astype(np.int64)
        t1 = t[:, 1].astype(np.int64)
        base = t0.min()
        s, e = (t0 - base) * 10, (t1 - base) * 10   # ns
        cu = (t[:, 2] >> np.uint64(32)).astype(np.int64) * 256 + ((t[:, 2] >> np.uint64(8)) & np.uint64(0xFF)).astype(np.int64)
        dur = e - s
        ucu, cnt = np.unique(cu, return_counts=True)
        # max concurrency per CU
        conc = 0
        for c in ucu:
            m = cu == c
            ev = sorted([(x, 1) for x in s[m]] + [(x, -1) for x in e[m]], key=lambda z: (z[0], z[1]))
            cur = 0
            for _, dlt in ev:
                cur += dlt
                conc = max(conc, cur)
        # per-CU last end (critical CU)
        cu_end = np.array([e[cu == c].max() for c in ucu])
        cu_busy = np.array([dur[cu == c].sum() for c in ucu])
        print(f"{what:22s} {M}x{N}x{K} rep{rep}: wgs {len(t)} span {e.max()/1e3:.2f} us | wg dur min/med/max "
              f"{dur.min()/1e3:.2f}/{np.median(dur)/1e3:.2f}/{dur.max()/1e3:.2f} us | last start {s.max()/1e3:.2f} us | "
              f"CUs {len(ucu)} wgs/CU min/max {cnt.min()}/{cnt.max()} conc max {conc} | CU end min/med "
              f"{cu_end.min()/1e3:.2f}/{np.median(cu_end)/1e3:.2f} us | CU busy(sum wg) med {np.median(cu_busy)/1e3:.2f} us",
              flush=True)
        st = sbuf.numpy().view(np.uint64).reshape(-1, 16).astype(np.int64)
        st = st[st[:, 15] != 0]
        if rep == 2 and len(st):
            # shader cycles (s_memtime) of the workgroup and at each K-step barrier: median over workgroups,
            # and the clock implied by cycles / wall duration
            cyc = np.median(st[:, 15])
            print(f"   cycles/wg med {cyc:.0f} -> clock {cyc / (np.median(dur) * 1e-9) / 1e9:.2f} GHz; step barriers (med cycles):",
                  [int(np.median(st[:, j])) for j in range(15) if np.count_nonzero(st[:, j]) > len(st) // 2])
        if rep == 2:
            # start-time histogram (1 us bins) and end-time histogram
            hs = np.bincount((s // 1000).astype(int))
            he = np.bincount((e // 1000).astype(int))
            print("   starts/us:", hs.tolist())
            print("   ends/us  :", he.tolist())
    A.free(); B.free(); Cm.free()
