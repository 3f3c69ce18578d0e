"""ctypes binding of the C-ABI in include/xerus_amd.h (libxerus_amd.so).

This is the Python side of the drop-in boundary: every call goes straight to the HIP kernels in
libxerus_amd.so. There is deliberately no CPU fallback — if the library (or a GPU) is missing,
loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("XRS_LIB_PATH") or os.path.join(_HERE, "libxerus_amd.so")   # (override: diagnostic builds)

_SZ = C.c_size_t
_DP = C.c_void_p

# (name, restype, argtypes) for every symbol declared in include/xerus_amd.h
SIGNATURES = {
    "xrs_create": (C.c_int, [C.POINTER(_DP), C.c_int]),
    "xrs_destroy": (C.c_int, [_DP]),
    "xrs_set_stream": (C.c_int, [_DP, _DP]),
    "xrs_get_stream": (_DP, [_DP]),
    "xrs_synchronize": (C.c_int, [_DP]),
    "xrs_last_error": (C.c_char_p, []),
    "xrs_version": (C.c_char_p, []),
    "xrs_malloc": (C.c_int, [_DP, C.POINTER(_DP), _SZ]),
    "xrs_free": (C.c_int, [_DP, _DP]),
    "xrs_pool_bytes": (_SZ, [_DP]),
    "xrs_upload": (C.c_int, [_DP, _DP, _DP, _SZ]),
    "xrs_download": (C.c_int, [_DP, _DP, _DP, _SZ]),
    "xrs_memset_zero": (C.c_int, [_DP, _DP, _SZ]),
    "xrs_copy": (C.c_int, [_DP, _DP, _DP, _SZ]),
    "xrs_nrm2": (C.c_int, [_DP, C.POINTER(C.c_double), _DP, _SZ]),
    "xrs_dot": (C.c_int, [_DP, C.POINTER(C.c_double), _DP, _DP, _SZ]),
    "xrs_asum": (C.c_int, [_DP, C.POINTER(C.c_double), _DP, _SZ]),
    "xrs_scal": (C.c_int, [_DP, _DP, C.c_double, _SZ]),
    "xrs_axpy": (C.c_int, [_DP, _DP, C.c_double, _DP, _SZ]),
    "xrs_scale_rows": (C.c_int, [_DP, _DP, _DP, _SZ, _SZ]),
    "xrs_gemm": (C.c_int, [_DP, _DP, _SZ, _SZ, C.c_double, _DP, _SZ, C.c_int, _SZ, _DP, _SZ, C.c_int]),
    "xrs_gemm_f32": (C.c_int, [_DP, _DP, _SZ, _SZ, C.c_float, _DP, _SZ, C.c_int, _SZ, _DP, _SZ, C.c_int]),
    "xrs_gemm_sym": (C.c_int,[_DP, _DP, _SZ, C.c_double, _DP, _SZ, C.c_int, _SZ, _DP, _SZ, C.c_int]),
    "xrs_gemm_batched": (C.c_int, [_DP, _SZ, C.POINTER(_DP), _SZ, _SZ, C.c_double, C.POINTER(_DP), _SZ, C.c_int, _SZ,
                                   C.POINTER(_DP), _SZ, C.c_int]),
    "xrs_permute": (C.c_int, [_DP, _DP, _DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "xrs_qc": (C.c_int, [_DP, _DP, _DP, C.POINTER(_SZ), _DP, _SZ, _SZ]),
    "xrs_cq": (C.c_int, [_DP, _DP, _DP, C.POINTER(_SZ), _DP, _SZ, _SZ]),
    "xrs_qr": (C.c_int, [_DP, _DP, _DP, _DP, _SZ, _SZ]),
    "xrs_rq": (C.c_int, [_DP, _DP, _DP, _DP, _SZ, _SZ]),
    "xrs_svd": (C.c_int, [_DP, _DP, _DP, _DP, _DP, _SZ, _SZ]),
    "xrs_solve": (C.c_int, [_DP, _DP, _DP, _SZ, _SZ, _DP, _SZ]),
    "xrs_solve_least_squares": (C.c_int, [_DP, _DP, _DP, _SZ, _SZ, _DP, _SZ]),
    "xrs_svd_rows_vt": (C.c_int, [_DP, _DP, _DP, C.POINTER(C.c_int), _DP, _SZ, _SZ, C.c_int]),
    "xrs_sym_eig_top": (C.c_int, [_DP, _DP, _DP, C.POINTER(C.c_int), _DP, _SZ, _SZ]),
    "xrs_sym_tridiag": (C.c_int, [_DP, _DP, _DP, _DP, _SZ]),
    "xrs_tt_entrywise_product": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.POINTER(_SZ), C.POINTER(_DP),
                                           C.c_double, C.POINTER(_DP)]),
    "xrs_tt_operator_apply": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP),
                                        C.POINTER(_SZ), C.POINTER(_DP), C.c_int, C.POINTER(_DP)]),
    "xrs_tt_move_core": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.c_int, _SZ, _SZ, C.c_int]),
    "xrs_tt_round": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.c_int, _SZ,
                               C.POINTER(_SZ), C.c_double]),
    "xrs_tt_dot": (C.c_int, [_DP, C.POINTER(C.c_double), _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP),
                             C.POINTER(_SZ), C.POINTER(_DP)]),
    "xrs_tt_dot_async": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.POINTER(_SZ),
                                   C.POINTER(_DP)]),
    "xrs_tt_dot_wait": (C.c_int, [_DP, C.POINTER(C.c_double)]),
    "xrs_tt_dot_f32": (C.c_int, [_DP, C.POINTER(C.c_double), _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP),
                                 C.POINTER(_SZ), C.POINTER(_DP)]),
    "xrs_tt_round_sharded": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.POINTER(_SZ),
                                       C.c_double, _DP, _DP, C.POINTER(C.c_int)]),
    "xrs_tt_round_sharded_ex": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.POINTER(_SZ),
                                          C.c_double, C.c_int, C.c_int, _DP, _DP, C.POINTER(C.c_int)]),
    "xrs_tt_dot_sharded": (C.c_int, [_DP, C.POINTER(C.c_double), _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP),
                                     C.POINTER(_SZ), C.POINTER(_DP), _DP, _DP]),
    "xrs_tt_last_round_path": (C.c_int, [_DP]),
    "xrs_tt_soft_threshold": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.POINTER(_SZ), C.POINTER(_DP), C.c_int, _SZ,
                                        C.POINTER(C.c_double)]),
    "xrs_comm_unique_id": (C.c_int, [_DP]),
    "xrs_comm_create": (C.c_int, [_DP, C.c_int, C.c_int, _DP, C.POINTER(_DP)]),
    "xrs_comm_emulate": (C.c_int, [_DP, C.c_int, C.POINTER(_DP)]),
    "xrs_comm_destroy": (C.c_int, [_DP]),
    "xrs_comm_calls": (_SZ, [_DP]),
    "xrs_comm_allreduce": (C.c_int, [_DP, _DP, _SZ]),
    "xrs_comm_allgather": (C.c_int, [_DP, _DP, _DP, _SZ]),
    "xrs_tt_gather_sharded": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.c_int, C.c_int, C.POINTER(_SZ), C.POINTER(_DP),
                                        C.POINTER(_DP), _DP, _DP]),
    "xrs_tt_shard": (C.c_int, [_DP, _SZ, C.POINTER(_SZ), C.c_int, C.c_int, C.POINTER(_SZ), C.POINTER(_DP), C.POINTER(_DP)]),
    "xrs_prof_begin": (C.c_int, [_DP, C.c_uint32]),
    "xrs_prof_end": (C.c_int, [_DP, C.POINTER(_SZ), C.POINTER(C.c_double), C.POINTER(C.c_double),
                               C.POINTER(C.c_double)]),
}

KFAM_GEMM, KFAM_PERMUTE, KFAM_QR, KFAM_SVD, KFAM_ELEMWISE, KFAM_SPLITK = 1, 2, 4, 8, 16, 32
ROUND_PATHS = {0: None, 1: "chain", 2: "truncate", 3: "reference", 4: "general"}

_lib = None


class XrsError(RuntimeError):
    """A non-zero status from the C-ABI (the reference raises xerus::misc::generic_error)."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed with status {code}: {msg}")
        self.code = code


def load(path: str | None = None) -> C.CDLL:
    """Load libxerus_amd.so and attach the signatures. Raises if the library is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"{p} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check(fn: str, status: int):
    if status != 0:
        raise XrsError(fn, status, load().xrs_last_error().decode())


def _arr(vals: Sequence[int]):
    return (_SZ * len(vals))(*[int(v) for v in vals])


class Handle:
    """One HIP stream + caching allocator (xrs_handle_t)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.h = _DP()
        _check("xrs_create", self.lib.xrs_create(C.byref(self.h), device))

    def close(self):
        if self.h:
            _check("xrs_destroy", self.lib.xrs_destroy(self.h))
            self.h = _DP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- memory
    def malloc(self, nbytes: int) -> int:
        p = _DP()
        _check("xrs_malloc", self.lib.xrs_malloc(self.h, C.byref(p), nbytes))
        return p.value or 0

    def free(self, ptr: int):
        _check("xrs_free", self.lib.xrs_free(self.h, _DP(ptr)))

    def synchronize(self):
        _check("xrs_synchronize", self.lib.xrs_synchronize(self.h))

    def set_stream(self, stream_ptr: int | None):
        _check("xrs_set_stream", self.lib.xrs_set_stream(self.h, _DP(stream_ptr or 0)))

    def stream(self) -> int:
        return self.lib.xrs_get_stream(self.h) or 0

    def array(self, a: np.ndarray) -> "DeviceArray":
        return DeviceArray.from_host(self, a)

    def empty(self, shape) -> "DeviceArray":
        return DeviceArray(self, tuple(int(s) for s in shape))

    def zeros(self, shape) -> "DeviceArray":
        d = DeviceArray(self, tuple(int(s) for s in shape))
        _check("xrs_memset_zero", self.lib.xrs_memset_zero(self.h, _DP(d.ptr), d.size))
        return d

    # ---- kernels
    def gemm(self, C_: "DeviceArray", M, N, alpha, A: "DeviceArray", lda, transA, K, B: "DeviceArray", ldb, transB):
        _check("xrs_gemm", self.lib.xrs_gemm(self.h, _DP(C_.ptr), M, N, alpha, _DP(A.ptr), lda, int(transA), K,
                                            _DP(B.ptr), ldb, int(transB)))

    def gemm_f32(self, C_: "Float32Array", M, N, alpha, A: "Float32Array", lda, transA, K, B: "Float32Array", ldb, transB):
        """xrs_gemm_f32: the fp32-MFMA GEMM on Float32Array operands."""
        _check("xrs_gemm_f32", self.lib.xrs_gemm_f32(self.h, _DP(C_.ptr), M, N, float(alpha), _DP(A.ptr), lda, int(transA),
                                                    K, _DP(B.ptr), ldb, int(transB)))

    def array_f32(self, a: np.ndarray) -> "Float32Array":
        return Float32Array.from_host(self, a)

    def gemm_sym(self, C_: "DeviceArray", N, alpha, A: "DeviceArray", lda, transA, K, B: "DeviceArray", ldb, transB):
        _check("xrs_gemm_sym", self.lib.xrs_gemm_sym(self.h, _DP(C_.ptr), N, alpha, _DP(A.ptr), lda, int(transA), K,
                                                    _DP(B.ptr), ldb, int(transB)))

    def gemm_batched(self, Cs, M, N, alpha, As, lda, transA, K, Bs, ldb, transB):
        """xrs_gemm_batched over lists of DeviceArrays (same shapes)."""
        cnt = len(Cs)
        tab = lambda xs: (_DP * max(1, cnt))(*[_DP(x.ptr) for x in xs])  # noqa: E731
        _check("xrs_gemm_batched", self.lib.xrs_gemm_batched(self.h, cnt, tab(Cs), M, N, alpha, tab(As), lda, int(transA),
                                                            K, tab(Bs), ldb, int(transB)))

    def matmul(self, A: "DeviceArray", transA: bool, B: "DeviceArray", transB: bool, alpha: float = 1.0):
        """Row-major C = alpha*op(A)*op(B) with the reference's inline-overload ld convention."""
        am, ak = (A.shape[1], A.shape[0]) if transA else (A.shape[0], A.shape[1])
        bk, bn = (B.shape[1], B.shape[0]) if transB else (B.shape[0], B.shape[1])
        assert ak == bk, (A.shape, B.shape)
        out = self.empty((am, bn))
        self.gemm(out, am, bn, alpha, A, A.shape[1], transA, ak, B, B.shape[1], transB)
        return out

    def permute(self, out: "DeviceArray", inp: "DeviceArray", dims, shuffle):
        _check("xrs_permute", self.lib.xrs_permute(self.h, _DP(out.ptr), _DP(inp.ptr), len(dims), _arr(dims),
                                                  _arr(shuffle)))

    def reshuffle(self, inp: "DeviceArray", shuffle):
        dims = inp.shape
        out_dims = [0] * len(dims)
        for i, s in enumerate(shuffle):
            out_dims[s] = dims[i]
        out = self.empty(tuple(out_dims))
        self.permute(out, inp, dims, shuffle)
        return out

    def nrm2(self, x: "DeviceArray") -> float:
        r = C.c_double()
        _check("xrs_nrm2", self.lib.xrs_nrm2(self.h, C.byref(r), _DP(x.ptr), x.size))
        return r.value

    def dot(self, x: "DeviceArray", y: "DeviceArray") -> float:
        r = C.c_double()
        _check("xrs_dot", self.lib.xrs_dot(self.h, C.byref(r), _DP(x.ptr), _DP(y.ptr), x.size))
        return r.value

    def asum(self, x: "DeviceArray") -> float:
        r = C.c_double()
        _check("xrs_asum", self.lib.xrs_asum(self.h, C.byref(r), _DP(x.ptr), x.size))
        return r.value

    def scal(self, x: "DeviceArray", alpha: float):
        _check("xrs_scal", self.lib.xrs_scal(self.h, _DP(x.ptr), alpha, x.size))

    def axpy(self, y: "DeviceArray", alpha: float, x: "DeviceArray"):
        _check("xrs_axpy", self.lib.xrs_axpy(self.h, _DP(y.ptr), alpha, _DP(x.ptr), x.size))

    def scale_rows(self, X: "DeviceArray", s: "DeviceArray"):
        _check("xrs_scale_rows", self.lib.xrs_scale_rows(self.h, _DP(X.ptr), _DP(s.ptr), X.shape[0], X.size // max(1, X.shape[0])))

    def qc(self, A: "DeviceArray"):
        m, n = A.shape
        k = min(m, n)
        Q, Cm = self.empty((m, k)), self.empty((k, n))
        r = _SZ()
        _check("xrs_qc", self.lib.xrs_qc(self.h, _DP(Q.ptr), _DP(Cm.ptr), C.byref(r), _DP(A.ptr), m, n))
        rank = r.value
        Q.shape, Cm.shape = (m, rank), (rank, n)
        return Q, Cm, rank

    def cq(self, A: "DeviceArray"):
        m, n = A.shape
        k = min(m, n)
        Cm, Q = self.empty((m, k)), self.empty((k, n))
        r = _SZ()
        _check("xrs_cq", self.lib.xrs_cq(self.h, _DP(Cm.ptr), _DP(Q.ptr), C.byref(r), _DP(A.ptr), m, n))
        rank = r.value
        Cm.shape, Q.shape = (m, rank), (rank, n)
        return Cm, Q, rank

    def qr(self, A: "DeviceArray"):
        m, n = A.shape
        k = min(m, n)
        Q, R = self.empty((m, k)), self.empty((k, n))
        _check("xrs_qr", self.lib.xrs_qr(self.h, _DP(Q.ptr), _DP(R.ptr), _DP(A.ptr), m, n))
        return Q, R

    def rq(self, A: "DeviceArray"):
        m, n = A.shape
        k = min(m, n)
        R, Q = self.empty((m, k)), self.empty((k, n))
        _check("xrs_rq", self.lib.xrs_rq(self.h, _DP(R.ptr), _DP(Q.ptr), _DP(A.ptr), m, n))
        return R, Q

    def svd(self, A: "DeviceArray"):
        m, n = A.shape
        k = min(m, n)
        U, S, Vt = self.empty((m, k)), self.empty((k,)), self.empty((k, n))
        _check("xrs_svd", self.lib.xrs_svd(self.h, _DP(U.ptr), _DP(S.ptr), _DP(Vt.ptr), _DP(A.ptr), m, n))
        return U, S, Vt

    def solve(self, A: "DeviceArray", B: "DeviceArray", least_squares: bool = False):
        """X with A X = B (xrs_solve; least_squares: xrs_solve_least_squares). B: m x p (or length m)."""
        m, n = A.shape
        p = B.shape[1] if len(B.shape) == 2 else 1
        X = self.empty((n, p) if len(B.shape) == 2 else (n,))
        fn = "xrs_solve_least_squares" if least_squares else "xrs_solve"
        _check(fn, getattr(self.lib, fn)(self.h, _DP(X.ptr), _DP(A.ptr), m, n, _DP(B.ptr), p))
        return X

    def sym_eig_top(self, A: "DeviceArray", kk: int):
        """(lam, Ut, status): the kk largest eigenpairs of the symmetric A (n <= 128), xrs_sym_eig_top."""
        n = A.shape[0]
        lam, Ut, st = self.empty((kk,)), self.empty((kk, n)), C.c_int()
        _check("xrs_sym_eig_top", self.lib.xrs_sym_eig_top(self.h, _DP(lam.ptr), _DP(Ut.ptr), C.byref(st), _DP(A.ptr), n, kk))
        return lam, Ut, st.value

    def sym_tridiag(self, A: "DeviceArray"):
        """(d, e) of the Householder tridiagonalisation of the symmetric A (xrs_sym_tridiag)."""
        n = A.shape[0]
        d, e = self.empty((n,)), self.empty((n,))
        _check("xrs_sym_tridiag", self.lib.xrs_sym_tridiag(self.h, _DP(d.ptr), _DP(e.ptr), _DP(A.ptr), n))
        return d.numpy(), e.numpy()[: n - 1]

    def svd_rows_vt(self, A: "DeviceArray", kernel: int = 0):
        """(S, Vt, sweeps) of the rows of A (p <= q <= 512) by one-sided Jacobi (xrs_svd_rows_vt)."""
        p, q = A.shape
        S, Vt, sw = self.empty((p,)), self.empty((p, q)), C.c_int()
        _check("xrs_svd_rows_vt", self.lib.xrs_svd_rows_vt(self.h, _DP(S.ptr), _DP(Vt.ptr), C.byref(sw), _DP(A.ptr), p, q, kernel))
        return S, Vt, sw.value

    def tt_operator_apply(self, n, m, ra, A, rb, B, p=None, transpose=False):
        """xrs_tt_operator_apply on device cores (DeviceArrays); returns the product cores as numpy arrays
        (the device results are freed)."""
        d = len(n)
        out = (_DP * d)()
        tab = lambda xs: (_DP * d)(*[_DP(x.ptr) for x in xs])  # noqa: E731
        _check("xrs_tt_operator_apply", self.lib.xrs_tt_operator_apply(
            self.h, d, _arr(n), _arr(m), _arr(p) if p is not None else None, _arr(ra), tab(A), _arr(rb), tab(B),
            int(transpose), out))
        res = []
        for k in range(d):
            nk = m[k] if transpose else n[k]
            shape = (ra[k] * rb[k], nk) + ((p[k],) if p is not None else ()) + (ra[k + 1] * rb[k + 1],)
            arr = DeviceArray(self, shape, ptr=out[k], owned=False)
            res.append(arr.numpy())
            self.free(out[k])
        return res

    def last_round_path(self) -> str | None:
        """"chain" / "truncate" / "general" / "reference": the algorithm of this handle's last TT round."""
        return ROUND_PATHS[self.lib.xrs_tt_last_round_path(self.h)]

    # ---- profiling
    def prof_begin(self, mask: int):
        _check("xrs_prof_begin", self.lib.xrs_prof_begin(self.h, mask))

    def prof_end(self):
        n, ms, fl, by = _SZ(), C.c_double(), C.c_double(), C.c_double()
        _check("xrs_prof_end", self.lib.xrs_prof_end(self.h, C.byref(n), C.byref(ms), C.byref(fl), C.byref(by)))
        return {"launches": n.value, "ms": ms.value, "flops": fl.value, "bytes": by.value}


class DeviceArray:
    """A row-major float64 array in the handle's device pool."""

    def __init__(self, handle: Handle, shape: tuple, ptr: int | None = None, owned: bool = True):
        self.handle = handle
        self.shape = tuple(shape)
        self.capacity = self.size
        self.owned = owned and ptr is None
        self.ptr = ptr if ptr is not None else (handle.malloc(max(8, self.capacity * 8)))

    @property
    def size(self) -> int:
        """Elements of the current shape (a factorisation may shrink the shape to the rank)."""
        return int(np.prod(self.shape)) if self.shape else 1

    @classmethod
    def from_host(cls, handle: Handle, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a, dtype=np.float64)
        d = cls(handle, a.shape)
        if a.size:
            _check("xrs_upload", handle.lib.xrs_upload(handle.h, _DP(d.ptr), a.ctypes.data_as(_DP), a.size))
        return d

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=np.float64)
        assert self.size <= self.capacity, "shape exceeds the allocation"
        if self.size:
            _check("xrs_download", self.handle.lib.xrs_download(self.handle.h, out.ctypes.data_as(_DP), _DP(self.ptr),
                                                               self.size))
        return out

    def free(self):
        if self.owned and self.ptr:
            self.handle.free(self.ptr)
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Float32Array:
    """A row-major float32 array in the handle's device pool (operands of xrs_gemm_f32). The C-ABI's
    upload / download move doubles, so the float32 payload travels as doubles' bytes (padded to 8 B);
    `offset` (floats) views the array at an unaligned start, to exercise the scalar staging path."""

    def __init__(self, handle: Handle, shape: tuple, offset: int = 0):
        self.handle = handle
        self.shape = tuple(int(s) for s in shape)
        self.offset = int(offset)
        self._words = max(1, (self.size + self.offset + 1) // 2)
        self.base = handle.malloc(8 * self._words)
        self.ptr = self.base + 4 * self.offset

    @property
    def size(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    @classmethod
    def from_host(cls, handle: Handle, a: np.ndarray, offset: int = 0) -> "Float32Array":
        a = np.ascontiguousarray(a, dtype=np.float32)
        d = cls(handle, a.shape, offset)
        buf = np.zeros(2 * d._words, dtype=np.float32)
        buf[d.offset:d.offset + a.size] = a.ravel()
        _check("xrs_upload", handle.lib.xrs_upload(handle.h, _DP(d.base), buf.view(np.float64).ctypes.data_as(_DP), d._words))
        return d

    def numpy(self) -> np.ndarray:
        buf = np.empty(self._words, dtype=np.float64)
        _check("xrs_download", self.handle.lib.xrs_download(self.handle.h, buf.ctypes.data_as(_DP), _DP(self.base), self._words))
        return buf.view(np.float32)[self.offset:self.offset + self.size].reshape(self.shape).copy()

    def free(self):
        if self.base:
            self.handle.free(self.base)
        self.base = self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DotFuture:
    """Result of TTDevice.dot_async."""

    def __init__(self, handle: Handle):
        self.handle = handle
        self._value = None

    def result(self) -> float:
        if self._value is None:
            out = C.c_double()
            _check("xrs_tt_dot_wait", self.handle.lib.xrs_tt_dot_wait(self.handle.h, C.byref(out)))
            self._value = out.value
        return self._value


class TTDevice:
    """A TT tensor whose cores live in the handle's device pool (core k: (r[k], n[k], r[k+1]) row-major).

    Thin wrapper over xrs_tt_* — the TT hot path runs entirely on the GPU."""

    def __init__(self, handle: Handle, dims, ranks, ptrs, canonicalized=False, core_position=0):
        self.handle = handle
        self.dims = [int(x) for x in dims]
        self.r = [int(x) for x in ranks]        # d+1 entries
        self.ptrs = list(ptrs)
        self.canonicalized = canonicalized
        self.core_position = core_position

    @classmethod
    def from_cores(cls, handle: Handle, cores, canonicalized=False, core_position=0) -> "TTDevice":
        dims = [c.shape[1] for c in cores]
        ranks = [cores[0].shape[0]] + [c.shape[2] for c in cores]
        ptrs = []
        for c in cores:
            c = np.ascontiguousarray(c, dtype=np.float64)
            p = handle.malloc(max(8, c.size * 8))
            _check("xrs_upload", handle.lib.xrs_upload(handle.h, _DP(p), c.ctypes.data_as(_DP), c.size))
            ptrs.append(p)
        return cls(handle, dims, ranks, ptrs, canonicalized, core_position)

    def clone(self) -> "TTDevice":
        """Device-side copy of every core (stream-ordered, no host round trip)."""
        ptrs = []
        for k, p in enumerate(self.ptrs):
            size = self.r[k] * self.dims[k] * self.r[k + 1]
            q = self.handle.malloc(max(8, size * 8))
            _check("xrs_copy", self.handle.lib.xrs_copy(self.handle.h, _DP(q), _DP(p), size))
            ptrs.append(q)
        return TTDevice(self.handle, self.dims, self.r, ptrs, self.canonicalized, self.core_position)

    @property
    def order(self):
        return len(self.dims)

    @property
    def ranks(self):
        return self.r[1:-1]

    def cores(self):
        out = []
        for k, p in enumerate(self.ptrs):
            shp = (self.r[k], self.dims[k], self.r[k + 1])
            a = np.empty(shp)
            _check("xrs_download", self.handle.lib.xrs_download(self.handle.h, a.ctypes.data_as(_DP), _DP(p), a.size))
            out.append(a)
        return out

    def _arrays(self):
        # ctypes views are cached and reused while r / ptrs are the lists the last call produced (the C
        # side updates them in place); ~16 us of Python per call otherwise
        c = getattr(self, "_cache", None)
        if c is not None and c[3] is self.r and c[4] is self.ptrs:
            return c[0], c[1], c[2]
        d = self.order
        n = _arr(self.dims)
        r = _arr(self.r)
        cores = (_DP * d)(*self.ptrs)
        self._cache = (n, r, cores, self.r, self.ptrs)
        return n, r, cores

    def _writeback(self, r, cores):
        self.r = r[:]
        self.ptrs = [p or 0 for p in cores[:]]
        c = getattr(self, "_cache", None)
        if c is not None and c[1] is r and c[2] is cores:
            self._cache = (c[0], r, cores, self.r, self.ptrs)

    def move_core(self, position: int, keep_rank: bool = False):
        n, r, cores = self._arrays()
        st = self.handle.lib.xrs_tt_move_core(self.handle.h, self.order, n, r, cores, int(self.canonicalized),
                                              self.core_position, position, int(keep_rank))
        self._writeback(r, cores)
        _check("xrs_tt_move_core", st)
        self.canonicalized, self.core_position = True, position

    def round(self, max_ranks, eps: float = 8 * np.finfo(float).eps):
        d = self.order
        if isinstance(max_ranks, (int, np.integer)):
            max_ranks = [int(max_ranks)] * (d - 1)
        n, r, cores = self._arrays()
        key = tuple(max_ranks)
        mc = getattr(self, "_mr_cache", None)
        if mc is None or mc[0] != key:
            mc = (key, _arr(list(max_ranks) + [1]))
            self._mr_cache = mc
        mr = mc[1]
        st = self.handle.lib.xrs_tt_round(self.handle.h, d, n, r, cores, int(self.canonicalized), self.core_position,
                                          mr, eps)
        self._writeback(r, cores)
        _check("xrs_tt_round", st)
        self.canonicalized, self.core_position = True, 0

    def soft_threshold(self, taus):
        """TTNetwork::soft_threshold (xrs_tt_soft_threshold): taus[0] applies to the LAST edge."""
        d = self.order
        if isinstance(taus, (int, float)):
            taus = [float(taus)] * (d - 1)
        n, r, cores = self._arrays()
        t = (C.c_double * max(1, d - 1))(*taus)
        st = self.handle.lib.xrs_tt_soft_threshold(self.handle.h, d, n, r, cores, int(self.canonicalized),
                                                   self.core_position, t)
        self._writeback(r, cores)
        _check("xrs_tt_soft_threshold", st)
        self.canonicalized, self.core_position = True, 0

    def dot(self, other: "TTDevice") -> float:
        if self.dims != other.dims:
            raise ValueError(f"dot of TTs with different dimensions: {self.dims} vs {other.dims}")
        out = C.c_double()
        n, rx, xc = self._arrays()
        _, ry, yc = other._arrays()
        _check("xrs_tt_dot", self.handle.lib.xrs_tt_dot(self.handle.h, C.byref(out), self.order, n, rx, xc, ry, yc))
        return out.value

    def dot_f32(self, other: "TTDevice") -> float:
        """<self, other> on fp32 MFMA tiles (xrs_tt_dot_f32): a reduced-precision side path, error ~1e-7
        ||self|| ||other||; dot() is the fp64 product the reference computes."""
        if self.dims != other.dims:
            raise ValueError(f"dot of TTs with different dimensions: {self.dims} vs {other.dims}")
        out = C.c_double()
        n, rx, xc = self._arrays()
        _, ry, yc = other._arrays()
        _check("xrs_tt_dot_f32", self.handle.lib.xrs_tt_dot_f32(self.handle.h, C.byref(out), self.order, n, rx, xc, ry, yc))
        return out.value

    def dot_async(self, other: "TTDevice") -> "DotFuture":
        """<self, other> enqueued on the handle's side streams (xrs_tt_dot_async): work enqueued next on the
        handle's main stream (e.g. self.round) runs beside it; DotFuture.result() waits."""
        if self.dims != other.dims:
            raise ValueError(f"dot of TTs with different dimensions: {self.dims} vs {other.dims}")
        if other.handle is not self.handle:
            raise ValueError("dot_async: both TTs must live on the same handle")
        n, rx, xc = self._arrays()
        _, ry, yc = other._arrays()
        _check("xrs_tt_dot_async", self.handle.lib.xrs_tt_dot_async(self.handle.h, self.order, n, rx, xc, ry, yc))
        return DotFuture(self.handle)

    def frob_norm(self) -> float:
        if self.canonicalized:
            k = self.core_position
            size = self.r[k] * self.dims[k] * self.r[k + 1]
            return self.handle.nrm2(DeviceArray(self.handle, (size,), ptr=self.ptrs[k], owned=False))
        return float(np.sqrt(max(0.0, self.dot(self))))

    def free(self):
        for p in self.ptrs:
            if p:
                self.handle.free(p)
        self.ptrs = [0] * len(self.ptrs)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
