"""CPU oracle: a restatement of the reference's algorithms on the hot path.

TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline — never as the product path.

Every function cites the reference file:line it follows (reference: xerus v3.0.1 at
/root/reference, which is NOT available at run time on the GPU box). The linear algebra calls the
same LAPACK routines the reference calls through LAPACKE (dgeqp3, dorgqr, dgeqrf, dgerqf, dorgrq,
dgesdd — via scipy.linalg.lapack, scipy-openblas 0.3.29) and BLAS dgemm (numpy). The byte-exact
pieces (reshuffle, Tensor::random's input stream) are restated in C (oracle/csrc/oracle.c).

Pinning: the reference itself is unbuildable in this image (it needs cblas.h/lapacke.h, SuiteSparse
CHOLMOD and Boost headers that are absent), so this oracle is pinned by the
reference's own known-answer tests re-expressed as data in tests/golden/ (products, assignments,
factorisation properties, TT rounding properties) and by the libstdc++ RNG stream.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
from scipy.linalg import lapack

DBL_EPSILON = float(np.finfo(np.float64).eps)
EPSILON = 8 * DBL_EPSILON  # include/xerus/basic.h:51

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = C.CDLL(path)
        lib.orc_reshuffle.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        lib.orc_rng_seed.argtypes = [C.c_void_p, C.c_uint64]
        lib.orc_rng_seed_engine.argtypes = [C.c_void_p, C.c_uint64]
        lib.orc_rng_next.argtypes = [C.c_void_p]
        lib.orc_rng_next.restype = C.c_uint64
        lib.orc_rng_normal.argtypes = [C.c_void_p]
        lib.orc_rng_normal.restype = C.c_double
        lib.orc_rng_fill_normal.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        lib.orc_rng_state_bytes.restype = C.c_size_t
        _LIB = lib
    return _LIB


# ------------------------------------------------------------------------------------------------
# Random input stream (include/xerus/tensor.h:212-220, misc/random.cpp:29-30, test.cpp:96-108)
class Rng:
    """std::mt19937_64 + std::normal_distribution<double> exactly as libstdc++ draws them."""

    SEED = 0xBAADF00D  # src/xerus/test/test.cpp:105

    def __init__(self, seed: int = SEED):
        lib = _lib()
        self._state = C.create_string_buffer(lib.orc_rng_state_bytes())
        lib.orc_rng_seed(self._state, seed)

    def normal(self, n: int) -> np.ndarray:
        out = np.empty(int(n), dtype=np.float64)
        if n:
            _lib().orc_rng_fill_normal(self._state, out.ctypes.data, out.size)
        return out


def tensor_random(rng: Rng, dims: Sequence[int]) -> np.ndarray:
    """Tensor::random: entries drawn in row-major order (tensor.h:212-220)."""
    dims = tuple(int(d) for d in dims)
    return rng.normal(int(np.prod(dims)) if dims else 1).reshape(dims)


# ------------------------------------------------------------------------------------------------
# Permutation (indexedTensor_tensor_evaluate.cpp:55-143) — bit-exact C restatement
def reshuffle(base: np.ndarray, shuffle: Sequence[int]) -> np.ndarray:
    base = np.ascontiguousarray(base, dtype=np.float64)
    dims = base.shape
    assert sorted(shuffle) == list(range(len(dims))), "shuffle must be a permutation"
    out_dims = [0] * len(dims)
    for i, s in enumerate(shuffle):
        out_dims[s] = dims[i]
    out = np.empty(out_dims, dtype=np.float64)
    if base.ndim == 0:
        out[()] = base[()]
        return out
    arr = lambda v: (C.c_size_t * len(v))(*v)
    _lib().orc_reshuffle(out.ctypes.data, base.ctypes.data, len(dims), arr(dims), arr(list(shuffle)))
    return out


# ------------------------------------------------------------------------------------------------
# Contraction (tensor.cpp:1252-1352 -> blasWrapper::matrix_matrix_product, blasLapackWrapper.cpp:149-195)
def contract(lhs: np.ndarray, lhs_trans: bool, rhs: np.ndarray, rhs_trans: bool, num_modes: int,
             alpha: float = 1.0) -> np.ndarray:
    lo = lhs.ndim - num_modes
    ro = rhs.ndim - num_modes
    l_rem = lhs.shape[num_modes:] if lhs_trans else lhs.shape[:lo]
    l_con = lhs.shape[:num_modes] if lhs_trans else lhs.shape[lo:]
    r_rem = rhs.shape[:ro] if rhs_trans else rhs.shape[num_modes:]
    r_con = rhs.shape[ro:] if rhs_trans else rhs.shape[:num_modes]
    assert tuple(l_con) == tuple(r_con), (lhs.shape, rhs.shape, num_modes)
    left, mid, right = int(np.prod(l_rem)), int(np.prod(l_con)), int(np.prod(r_rem))
    A = lhs.reshape((mid, left) if lhs_trans else (left, mid))
    B = rhs.reshape((right, mid) if rhs_trans else (mid, right))
    Cm = alpha * ((A.T if lhs_trans else A) @ (B.T if rhs_trans else B))
    return Cm.reshape(tuple(l_rem) + tuple(r_rem))


def gemm(A, transA, B, transB, alpha=1.0):
    return alpha * ((A.T if transA else A) @ (B.T if transB else B))


# ------------------------------------------------------------------------------------------------
# Factorisations (blasLapackWrapper.cpp:201-498)
def qc(A: np.ndarray):
    """Row-major QC with column pivoting (blasLapackWrapper.cpp:243-305)."""
    m, n = A.shape
    assert m > 0 and n > 0
    max_rank = min(m, n)
    qr_, jpvt, tau, _work, info = lapack.dgeqp3(np.asfortranarray(A, dtype=np.float64))
    assert info == 0, "dgeqp3 failed"
    # rank rule (:268-272): first k with |R_kk| < 16*eps*R_00 (R_00 NOT in abs)
    rank = 1
    while rank < max_rank and not (abs(qr_[rank, rank]) < 16 * DBL_EPSILON * qr_[0, 0]):
        rank += 1
    Cm = np.zeros((rank, n))
    for col in range(n):  # (:280-285) un-permute the upper triangle
        tgt = int(jpvt[col]) - 1
        rows = min(rank, col + 1)
        Cm[:rows, tgt] = qr_[:rows, col]
    q, _w, info = lapack.dorgqr(qr_[:, :max_rank].copy(order="F"), tau[:max_rank])
    assert info == 0
    return np.ascontiguousarray(q[:, :rank]), Cm, rank


def cq(A: np.ndarray):
    """Row-major CQ: col-major dgeqp3 on A^T (blasLapackWrapper.cpp:317-371)."""
    m, n = A.shape
    Qt, Ct, rank = qc(np.ascontiguousarray(A.T))  # A^T = Qt Ct  ->  A = Ct^T Qt^T
    return np.ascontiguousarray(Ct.T), np.ascontiguousarray(Qt.T), rank


def qr(A: np.ndarray):
    """Unpivoted QR, dgeqrf + dorgqr (blasLapackWrapper.cpp:388-431)."""
    m, n = A.shape
    k = min(m, n)
    qr_, tau, _w, info = lapack.dgeqrf(np.asfortranarray(A, dtype=np.float64))
    assert info == 0
    R = np.triu(qr_[:k, :])
    q, _w, info = lapack.dorgqr(qr_[:, :k].copy(order="F"), tau[:k])
    return np.ascontiguousarray(q), np.ascontiguousarray(R)


def rq(A: np.ndarray):
    """Unpivoted RQ (blasLapackWrapper.cpp:445-498): A = R Q, R m x k, Q k x n."""
    Qt, Rt = qr(np.ascontiguousarray(A.T))  # A^T = Qt Rt -> A = Rt^T Qt^T
    return np.ascontiguousarray(Rt.T), np.ascontiguousarray(Qt.T)


def svd(A: np.ndarray):
    """Thin SVD via dgesdd 'S' (blasLapackWrapper.cpp:210-232)."""
    u, s, vt, info = lapack.dgesdd(np.asfortranarray(A, dtype=np.float64), compute_uv=1, full_matrices=0)
    assert info == 0, "dgesdd failed"
    return np.ascontiguousarray(u), s.copy(), np.ascontiguousarray(vt)


def svd_rank(s: np.ndarray, max_rank: int, eps: float) -> int:
    """Rank cut of calculate_svd (tensor.cpp:1462-1474)."""
    rank = len(s)
    if max_rank != 0:
        rank = min(rank, max_rank)
    for j in range(1, rank):
        if s[j] <= eps * s[0]:
            return j
    return rank


# ------------------------------------------------------------------------------------------------
# TT format (ttNetwork.cpp / tensorNetwork.cpp). Core k has dims (r_k, n_k, r_{k+1}), r_0 = r_d = 1.
def reduce_to_maximal_ranks(ranks: Sequence[int], dims: Sequence[int]) -> List[int]:
    """ttNetwork.cpp:370-402 (TTTensor, N = 1)."""
    ranks = list(ranks)
    d = len(dims)
    cur = 1
    for i in range(d - 1):
        cur *= dims[i]
        if cur < ranks[i]:
            ranks[i] = cur
        else:
            cur = ranks[i]
    cur = 1
    for i in range(1, d):
        cur *= dims[d - i]
        if cur < ranks[d - i - 1]:
            ranks[d - i - 1] = cur
        else:
            cur = ranks[d - i - 1]
    return ranks


@dataclass
class TT:
    cores: List[np.ndarray]
    canonicalized: bool = False
    core_position: int = 0

    @property
    def order(self) -> int:
        return len(self.cores)

    @property
    def dims(self) -> List[int]:
        return [c.shape[1] for c in self.cores]

    @property
    def ranks(self) -> List[int]:
        return [c.shape[2] for c in self.cores[:-1]]

    def copy(self) -> "TT":
        return TT([c.copy() for c in self.cores], self.canonicalized, self.core_position)

    @staticmethod
    def random(dims: Sequence[int], ranks: Sequence[int], rng: Rng) -> "TT":
        """TTNetwork::random (include/xerus/ttNetwork.h:129-157): raw N(0,1) cores, then move_core(0)."""
        tt = TT.random_raw(dims, ranks, rng)
        tt.move_core(0)
        return tt

    @staticmethod
    def random_raw(dims: Sequence[int], ranks: Sequence[int], rng: Rng) -> "TT":
        target = reduce_to_maximal_ranks(ranks, dims)
        d = len(dims)
        cores = []
        for i in range(d):
            left = 1 if i == 0 else target[i - 1]
            right = 1 if i == d - 1 else target[i]
            cores.append(tensor_random(rng, (left, dims[i], right)))
        return TT(cores)

    # ---- transfer_core (tensorNetwork.cpp:821-909) restricted to TT neighbours
    def transfer_core(self, frm: int, to: int, allow_rank_reduction: bool = True):
        X = self.cores[frm]
        a, n, b = X.shape
        if to == frm + 1:  # posA = last mode -> QC / QR (:842-848), posB = 0 -> R * to (:873)
            M = X.reshape(a * n, b)
            if allow_rank_reduction:
                Q, R, rank = qc(M)
            else:
                Q, R = qr(M)
                rank = Q.shape[1]
            self.cores[frm] = Q.reshape(a, n, rank)
            nxt = self.cores[to]
            self.cores[to] = (R @ nxt.reshape(nxt.shape[0], -1)).reshape(rank, nxt.shape[1], nxt.shape[2])
        elif to == frm - 1:  # posA = 0 -> CQ / RQ (:834-841), posB = last -> to * R (:875-876)
            M = X.reshape(a, n * b)
            if allow_rank_reduction:
                R, Q, rank = cq(M)
            else:
                R, Q = rq(M)
                rank = Q.shape[0]
            self.cores[frm] = Q.reshape(rank, n, b)
            prv = self.cores[to]
            self.cores[to] = (prv.reshape(-1, prv.shape[2]) @ R).reshape(prv.shape[0], prv.shape[1], rank)
        else:
            raise ValueError("not neighbours")

    def exceeds_maximal_ranks(self) -> bool:
        return self.ranks != reduce_to_maximal_ranks(self.ranks, self.dims)

    def move_core(self, position: int, keep_rank: bool = False):
        """TTNetwork::move_core (ttNetwork.cpp:582-628)."""
        d = self.order
        assert 0 <= position < d
        if self.canonicalized:
            for k in range(self.core_position, position):
                self.transfer_core(k, k + 1, not keep_rank)
            for k in range(self.core_position, position, -1):
                self.transfer_core(k, k - 1, not keep_rank)
        else:
            for k in range(0, position):
                self.transfer_core(k, k + 1, not keep_rank)
            for k in range(d - 1, position, -1):
                self.transfer_core(k, k - 1, not keep_rank)
        while self.exceeds_maximal_ranks():
            for k in range(position, 0, -1):
                self.transfer_core(k, k - 1, not keep_rank)
            for k in range(0, d - 1):
                self.transfer_core(k, k + 1, not keep_rank)
            for k in range(d - 1, position, -1):
                self.transfer_core(k, k - 1, not keep_rank)
        self.canonicalized = True
        self.core_position = position

    # ---- round_edge (tensorNetwork.cpp:678-818) for TT: from = right core (fromPos = 0, transFrom),
    #      to = left core (toPos = last, transTo)
    def round_edge(self, frm: int, to: int, max_rank: int, eps: float, soft: float = 0.0):
        """soft > 0: the kept singular values become max(0, sigma - soft) (:766, :788)."""
        F = self.cores[frm]          # (b, n, c)
        T = self.cores[to]           # (a, n', b)
        b = F.shape[0]
        if 5 * F.size * T.size >= 6 * b ** 4:   # (:745)
            coreA, Qf, _ = cq(F.reshape(b, -1))           # F = coreA * Qf  (:749)
            Qt, coreB, _ = qc(T.reshape(-1, b))           # T = Qt * coreB  (:755)
            X = coreA.T @ coreB.T                         # contract(X, coreA, true, coreB, true, 1) (:761)
            U, S, Vt = svd(X)                             # (:764)
            k = svd_rank(S, max_rank, eps)
            U, S, Vt = U[:, :k], np.maximum(0.0, S[:k] - soft), Vt[:k, :]
            coreB = S[:, None] * Vt                       # (:769)
            self.cores[frm] = (U.T @ Qf).reshape(k, F.shape[1], F.shape[2])           # (:773)
            self.cores[to] = (Qt @ coreB.T).reshape(T.shape[0], T.shape[1], k)        # (:779)
        else:
            X = F.reshape(b, -1).T @ T.reshape(-1, b).T   # (n c) x (a n') (:783)
            U, S, Vt = svd(X)
            k = svd_rank(S, max_rank, eps)
            U, S, Vt = U[:, :k], np.maximum(0.0, S[:k] - soft), Vt[:k, :]
            self.cores[to] = (Vt.T * S[None, :]).reshape(T.shape[0], T.shape[1], k)   # (:790-791)
            self.cores[frm] = np.ascontiguousarray(U.T).reshape(k, F.shape[1], F.shape[2])  # (:797-802)

    def round(self, max_ranks, eps: float = EPSILON):
        """TTNetwork::round (ttNetwork.cpp:644-665); an int max_ranks means round(size_t) (:669-672)."""
        d = self.order
        if isinstance(max_ranks, (int, np.integer)):
            max_ranks = [int(max_ranks)] * (d - 1)
        init_canon, init_pos = self.canonicalized, self.core_position
        self.move_core(d - 1)
        for i in range(d - 1):
            self.round_edge(d - 1 - i, d - 2 - i, max_ranks[d - 2 - i], eps)
        self.core_position = 0
        self.canonicalized = True
        if init_canon:
            self.move_core(init_pos)

    def soft_threshold(self, taus):
        """TTNetwork::soft_threshold (ttNetwork.cpp:688-713): canonicalize_right, then
        round_edge(numComponents - i, numComponents - i - 1, max, 0.0, taus[i]) -- taus[0] at the LAST edge."""
        d = self.order
        if isinstance(taus, (int, float, np.floating)):
            taus = [float(taus)] * (d - 1)
        assert len(taus) == d - 1
        init_canon, init_pos = self.canonicalized, self.core_position
        self.move_core(d - 1)
        for i in range(d - 1):
            self.round_edge(d - 1 - i, d - 2 - i, 2 ** 62, 0.0, taus[i])
        self.core_position = 0
        self.canonicalized = True
        if init_canon:
            self.move_core(init_pos)

    # ---- evaluation
    def full(self) -> np.ndarray:
        res = self.cores[0]
        for c in self.cores[1:]:
            res = np.tensordot(res, c, axes=([res.ndim - 1], [0]))
        return res.reshape(self.dims)

    def frob_norm(self) -> float:
        """ttNetwork.cpp:782-789."""
        if self.canonicalized:
            return float(np.linalg.norm(self.cores[self.core_position]))
        return float(np.sqrt(max(0.0, dot(self, self))))


def tt_svd(full: np.ndarray, eps: float, max_ranks: Sequence[int]) -> TT:
    """TT-SVD constructor TTNetwork(const Tensor&, eps, maxRanks) (ttNetwork.cpp:112-160): right to left,
    calculate_svd(remains, S, node, remains, 1 + position, maxRanks[position - 1], eps) with the cut of
    tensor.cpp:1462-1474, node -> component `position`, remains <- U S; the rest is component 0, core at 0."""
    dims = tuple(full.shape)
    d = len(dims)
    assert len(max_ranks) == d - 1
    remains = np.asarray(full, dtype=np.float64).reshape((1,) + dims + (1,))
    cores: List[np.ndarray] = [None] * d  # type: ignore[list-item]
    for pos in range(d - 1, 0, -1):
        split = 1 + pos
        sh = remains.shape
        u, s, vt = svd(remains.reshape(int(np.prod(sh[:split])), -1))
        r = svd_rank(s, max_ranks[pos - 1], eps)
        cores[pos] = np.ascontiguousarray(vt[:r].reshape((r,) + sh[split:]))
        remains = (u[:, :r] * s[:r]).reshape(sh[:split] + (r,))
    cores[0] = np.ascontiguousarray(remains)
    return TT(cores, True, 0)


def dot(x: TT, y: TT) -> float:
    """<x,y> as a left-to-right zipper (the order the reference's heuristics pick)."""
    E = np.ones((1, 1))
    for X, Y in zip(x.cores, y.cores):
        rx, n, rx2 = X.shape
        ry, _, ry2 = Y.shape
        T = E.T @ X.reshape(rx, n * rx2)                     # ry x (n rx2)
        E = T.reshape(ry * n, rx2).T @ Y.reshape(ry * n, ry2)  # rx2 x ry2
    return float(E[0, 0])


def tt_flops_dot(x: TT, y: TT) -> float:
    f = 0.0
    for X, Y in zip(x.cores, y.cores):
        rx, n, rx2 = X.shape
        ry, _, ry2 = Y.shape
        f += 2.0 * rx * ry * n * rx2 + 2.0 * ry * n * rx2 * ry2
    return f


def tt_add(x: TT, y: TT) -> TT:
    """TTNetwork::operator+= (ttNetwork.cpp:797-847): block-diagonal core assembly, not canonical."""
    d = x.order
    assert x.dims == y.dims
    cores = []
    for k, (X, Y) in enumerate(zip(x.cores, y.cores)):
        if d == 1:
            cores.append(X + Y)
            continue
        a1, n, b1 = X.shape
        a2, _, b2 = Y.shape
        if k == 0:
            cores.append(np.concatenate([X, Y], axis=2))
        elif k == d - 1:
            cores.append(np.concatenate([X, Y], axis=0))
        else:
            Z = np.zeros((a1 + a2, n, b1 + b2))
            Z[:a1, :, :b1] = X
            Z[a1:, :, b1:] = Y
            cores.append(Z)
    return TT(cores)


# ------------------------------------------------------------------------------------------------
# TTOperator (TTNetwork<true>): core k has dims (r_k, n_k, m_k, r_{k+1}); dense form (n_0..n_{d-1}, m_0..m_{d-1}).
def op_full(cores: Sequence[np.ndarray]) -> np.ndarray:
    """Contract the operator cores and order the modes (i_0..i_{d-1}, j_0..j_{d-1}) (TTNetwork<true> layout,
    ttNetwork.cpp:70-100)."""
    d = len(cores)
    res = cores[0]
    for c in cores[1:]:
        res = np.tensordot(res, c, axes=([res.ndim - 1], [0]))
    res = res.reshape([s for c in cores for s in c.shape[1:3]])
    return np.ascontiguousarray(np.transpose(res, [2 * k for k in range(d)] + [2 * k + 1 for k in range(d)]))


def op_apply_cores(A: Sequence[np.ndarray], X: Sequence[np.ndarray], transpose: bool = False) -> List[np.ndarray]:
    """The contracted TTStack of A(i/2, j/2) * x(j&0) (ttStack.cpp:197-309): core k is
    C[(a,b), i, (a',b')] = sum_j A[a,i,j,a'] X[b,j,b'], fused ranks operator-major (the operator's node is
    contracted first, :216-228); transpose: x(i&0) * A(i/2, j/2), the row mode contracted."""
    out = []
    for Ak, Xk in zip(A, X):
        ra, n, m, ra2 = Ak.shape
        rb, _, rb2 = Xk.shape
        C = np.einsum('aijd,bic->abjdc', Ak, Xk) if transpose else np.einsum('aijd,bjc->abidc', Ak, Xk)
        out.append(np.ascontiguousarray(C.reshape(ra * rb, C.shape[2], ra2 * rb2)))
    return out


def op_op_cores(A: Sequence[np.ndarray], B: Sequence[np.ndarray]) -> List[np.ndarray]:
    """A(i/2, j/2) * B(j/2, k/2): C[(a,b), i, k, (a',b')] = sum_j A[a,i,j,a'] B[b,j,k,b'] (ttStack.cpp:197-309)."""
    out = []
    for Ak, Bk in zip(A, B):
        ra, n, m, ra2 = Ak.shape
        rb, _, p, rb2 = Bk.shape
        C = np.einsum('aijd,bjkc->abikdc', Ak, Bk)
        out.append(np.ascontiguousarray(C.reshape(ra * rb, n, p, ra2 * rb2)))
    return out


# ------------------------------------------------------------------------------------------------
# ALS (src/xerus/algorithms/als.cpp:35-565), single site, dense local solves (numpy).
def als(A: Sequence[np.ndarray] | None, x: TT, b: TT, spd: bool = True, num_half_sweeps: int = 0, eps: float = 1e-6,
        asd: bool = False, use_residual: bool = False, preserve_core: bool = True) -> float:
    """ALSVariant::solve restated for one site: x is modified in place, the last energy is returned.
    A: operator cores (r, n, m, r') or None (approximate b). Local operators: x A x (spd) or x A^T A x."""
    d = x.order
    canon_end, core_end = x.canonicalized, x.core_position
    plain = spd or A is None
    # prepare_x_for_als (:109-187)
    first, prod = 0, 1
    while first + 1 < d:
        n = x.dims[first]
        if x.ranks[first] < prod * n:
            break
        cur = x.cores[first].reshape(-1, x.cores[first].shape[2])
        x.cores[first + 1] = np.einsum('ac,cnb->anb', cur, x.cores[first + 1])
        I = np.zeros((prod, n, prod * n))
        for i0 in range(prod):
            for i1 in range(n):
                I[i0, i1, i0 * n + i1] = 1.0
        x.cores[first] = I
        x.canonicalized = False   # two set_component calls (ttNetwork.cpp:491): never both at the core
        first, prod = first + 1, prod * n
    first_not, prod = d, 1
    while first_not > first + 1:
        n = x.dims[first_not - 1]
        if x.ranks[first_not - 2] < prod * n:
            break
        cur = x.cores[first_not - 1].reshape(x.cores[first_not - 1].shape[0], -1)
        x.cores[first_not - 2] = np.einsum('anc,cb->anb', x.cores[first_not - 2], cur)
        I = np.zeros((prod * n, n, prod))
        for i1 in range(n):
            for i2 in range(prod):
                I[i1 * prod + i2, i1, i2] = 1.0
        x.cores[first_not - 1] = I
        x.canonicalized = False
        first_not, prod = first_not - 1, prod * n
    if canon_end and core_end < first:
        x.canonicalized, x.core_position = True, first
    else:
        if canon_end and core_end >= first_not:
            x.canonicalized, x.core_position = True, first_not - 1
        x.move_core(first, keep_rank=True)

    def op_left(E, k):
        X, Ak = x.cores[k], A[k]
        if spd:
            return np.einsum('pqr,pnc,qnmd,rme->cde', E, X, Ak, X)
        return np.einsum('pqrs,pnc,qmnd,rmle,slf->cdef', E, X, Ak, Ak, X)

    def op_right(E, k):
        X, Ak = x.cores[k], A[k]
        if spd:
            return np.einsum('pnc,qnmd,rme,cde->pqr', X, Ak, X, E)
        return np.einsum('pnc,qmnd,rmle,slf,cdef->pqrs', X, Ak, Ak, X, E)

    def rhs_left(E, k):
        X, B = x.cores[k], b.cores[k]
        if plain:
            return np.einsum('pq,pnc,qnd->cd', E, B, X)
        return np.einsum('pqr,pnc,qnmd,rme->cde', E, B, A[k], X)

    def rhs_right(E, k):
        X, B = x.cores[k], b.cores[k]
        if plain:
            return np.einsum('pnc,qnd,cd->pq', B, X, E)
        return np.einsum('pnc,qnmd,rme,cde->pqr', B, A[k], X, E)

    one_op = np.ones((1, 1, 1)) if plain else np.ones((1, 1, 1, 1))
    one_rhs = np.ones((1, 1)) if plain else np.ones((1, 1, 1))
    oL, oR, bL, bR = [one_op], [one_op], [one_rhs], [one_rhs]
    for i in range(d - 1, first, -1):
        if A is not None:
            oR.append(op_right(oR[-1], i))
        bR.append(rhs_right(bR[-1], i))
    for i in range(first):
        if A is not None:
            oL.append(op_left(oL[-1], i))
        bL.append(rhs_left(bL[-1], i))
    normB = b.frob_norm() if b.canonicalized else float(np.linalg.norm(b.full()))
    cur = first

    def residual():
        if A is None:
            return float(np.linalg.norm(x.full() - b.full()))
        if spd:
            Ax = TT(op_apply_cores(A, x.cores)).full()
            return float(np.linalg.norm(Ax - b.full())) / normB
        X, Ak, B = x.cores[cur], A[cur], b.cores[cur]
        xAtAx = np.einsum('pqrs,pnc,qmnd,rmle,slf,cdef->', oL[-1], X, Ak, Ak, X, oR[-1])
        bAx = np.einsum('pqr,pnc,qnmd,rme,cde->', bL[-1], B, Ak, X, bR[-1])
        return float(np.sqrt(xAtAx - 2 * bAx + normB ** 2) / normB)

    def energy():
        if use_residual or (A is not None and not spd):
            return residual()
        X, B = x.cores[cur], b.cores[cur]
        bx = np.einsum('pq,pnc,qnd,cd->', bL[-1], B, X, bR[-1])
        if A is None:
            return float(0.5 * np.sum(X * X) - bx)
        xAx = np.einsum('pqr,pnc,qnmd,rme,cde->', oL[-1], X, A[cur], X, oR[-1])
        return float(abs(0.5 * xAx - bx))

    last2, last, en = 1e102, 1e101, energy()
    half, increasing = 0, True
    while True:
        if A is not None:
            Ak = A[cur]
            if spd:
                Aloc = np.einsum('arp,rijs,bsc->aibpjc', oL[-1], Ak, oR[-1])
                rhs = np.einsum('ra,ric,cb->aib', bL[-1], b.cores[cur], bR[-1])
            else:
                Aloc = np.einsum('aqrp,qyis,ryjt,bstc->aibpjc', oL[-1], Ak, Ak, oR[-1])
                rhs = np.einsum('rqa,ric,qijd,cdb->ajb', bL[-1], b.cores[cur], Ak, bR[-1])
            shp = x.cores[cur].shape
            N = int(np.prod(shp))
            M = Aloc.reshape(N, N)
            if asd:
                xv = x.cores[cur].reshape(N)
                grad = rhs.reshape(N) - M @ xv
                if spd:
                    alpha = float(grad @ grad) / float(grad @ (M @ grad))
                else:
                    grad = M.T @ grad
                    alpha = float(np.linalg.norm(grad)) / float(np.linalg.norm(M @ grad))
                x.cores[cur] = (xv + alpha * grad).reshape(shp)
            else:
                x.cores[cur] = np.linalg.solve(M, rhs.reshape(N)).reshape(shp)
        else:
            x.cores[cur] = np.einsum('ra,ric,cb->aib', bL[-1], b.cores[cur], bR[-1])
        at_end = (not increasing and cur == first) or (increasing and cur == first_not - 1)
        if at_end:
            half += 1
            last2, last, en = last, en, energy()
            if half == num_half_sweeps or abs(last - en) < eps or abs(last2 - en) < eps or first_not - first <= 1:
                if canon_end and preserve_core:
                    x.move_core(core_end, keep_rank=True)
                return en
            increasing = not increasing
        if increasing:
            x.move_core(cur + 1, keep_rank=True)
            if A is not None:
                oR.pop()
                oL.append(op_left(oL[-1], cur))
            bR.pop()
            bL.append(rhs_left(bL[-1], cur))
            cur += 1
        else:
            x.move_core(cur - 1, keep_rank=True)
            if A is not None:
                oL.pop()
                oR.append(op_right(oR[-1], cur))
            bL.pop()
            bR.append(rhs_right(bR[-1], cur))
            cur -= 1


# ------------------------------------------------------------------------------------------------
# Two-site ALS = DMRG / DMRG_SPD (als.cpp:43-69 lapack_solver split, :383-423 local problems,
# :556-563 variants), dense local solves and numpy SVD splits truncated to the initial ranks.
# Decreasing sweeps extend the right stack by the site that leaves the window (currIndex + 1); the
# reference writes currIndex there (als.cpp:371-379), correct only for one site (see host/als.cpp).
def dmrg(A: Sequence[np.ndarray], x: TT, b: TT, spd: bool = True, num_half_sweeps: int = 0, eps: float = 1e-6,
         preserve_core: bool = True) -> float:
    d = x.order
    s = 2
    canon_end, core_end = x.canonicalized, x.core_position
    target = list(x.ranks)
    # prepare_x_for_als (:109-187), window of two sites at the right end
    first, prod = 0, 1
    while first + 1 < d:
        n = x.dims[first]
        if x.ranks[first] < prod * n:
            break
        cur0 = x.cores[first].reshape(-1, x.cores[first].shape[2])
        x.cores[first + 1] = np.einsum('ac,cnb->anb', cur0, x.cores[first + 1])
        I = np.zeros((prod, n, prod * n))
        for i0 in range(prod):
            for i1 in range(n):
                I[i0, i1, i0 * n + i1] = 1.0
        x.cores[first] = I
        x.canonicalized = False
        first, prod = first + 1, prod * n
    first_not, prod = d, 1
    while first_not > first + s:
        n = x.dims[first_not - 1]
        if x.ranks[first_not - 2] < prod * n:
            break
        cur0 = x.cores[first_not - 1].reshape(x.cores[first_not - 1].shape[0], -1)
        x.cores[first_not - 2] = np.einsum('anc,cb->anb', x.cores[first_not - 2], cur0)
        I = np.zeros((prod * n, n, prod))
        for i1 in range(n):
            for i2 in range(prod):
                I[i1 * prod + i2, i1, i2] = 1.0
        x.cores[first_not - 1] = I
        x.canonicalized = False
        first_not, prod = first_not - 1, prod * n
    if canon_end and core_end < first:
        x.canonicalized, x.core_position = True, first
    else:
        if canon_end and core_end >= first_not:
            x.canonicalized, x.core_position = True, first_not - 1
        x.move_core(first, keep_rank=True)

    def op_left(E, k):
        X, Ak = x.cores[k], A[k]
        if spd:
            return np.einsum('pqr,pnc,qnmd,rme->cde', E, X, Ak, X)
        return np.einsum('pqrs,pnc,qmnd,rmle,slf->cdef', E, X, Ak, Ak, X)

    def op_right(E, k):
        X, Ak = x.cores[k], A[k]
        if spd:
            return np.einsum('pnc,qnmd,rme,cde->pqr', X, Ak, X, E)
        return np.einsum('pnc,qmnd,rmle,slf,cdef->pqrs', X, Ak, Ak, X, E)

    def rhs_left(E, k):
        X, B = x.cores[k], b.cores[k]
        if spd:
            return np.einsum('pq,pnc,qnd->cd', E, B, X)
        return np.einsum('pqr,pnc,qnmd,rme->cde', E, B, A[k], X)

    def rhs_right(E, k):
        X, B = x.cores[k], b.cores[k]
        if spd:
            return np.einsum('pnc,qnd,cd->pq', B, X, E)
        return np.einsum('pnc,qnmd,rme,cde->pqr', B, A[k], X, E)

    one_op = np.ones((1, 1, 1)) if spd else np.ones((1, 1, 1, 1))
    one_rhs = np.ones((1, 1)) if spd else np.ones((1, 1, 1))
    oL, oR, bL, bR = [one_op], [one_op], [one_rhs], [one_rhs]
    for i in range(d - 1, first + s - 1, -1):
        oR.append(op_right(oR[-1], i))
        bR.append(rhs_right(bR[-1], i))
    for i in range(first):
        oL.append(op_left(oL[-1], i))
        bL.append(rhs_left(bL[-1], i))
    normB = b.frob_norm() if b.canonicalized else float(np.linalg.norm(b.full()))
    cur = first

    def window(E0, k, left_step):
        E = E0
        for q in range(s):
            E = left_step(E, k + q)
        return E

    def energy():
        if spd:
            xAx = float(np.sum(window(oL[-1], cur, op_left) * oR[-1]))
            bx = float(np.sum(window(bL[-1], cur, rhs_left) * bR[-1]))
            return float(abs(0.5 * xAx - bx))
        xAtAx = float(np.sum(window(oL[-1], cur, op_left) * oR[-1]))
        bAx = float(np.sum(window(bL[-1], cur, rhs_left) * bR[-1]))
        return float(np.sqrt(xAtAx - 2 * bAx + normB ** 2) / normB)

    last2, last, en = 1e102, 1e101, energy()
    half, increasing = 0, True
    while True:
        A0, A1 = A[cur], A[cur + 1]
        if spd:
            Aloc = np.einsum('arp,rijs,sklt,btc->aikbpjlc', oL[-1], A0, A1, oR[-1])
            rhs = np.einsum('ra,ric,ckd,db->aikb', bL[-1], b.cores[cur], b.cores[cur + 1], bR[-1])
        else:
            Aloc = np.einsum('aqrp,qyis,ryjt,sxku,txlv,buvc->aikbpjlc', oL[-1], A0, A0, A1, A1, oR[-1])
            rhs = np.einsum('rqa,ryc,qyid,czm,dzke,meb->aikb', bL[-1], b.cores[cur], A0, b.cores[cur + 1], A1, bR[-1])
        rl, n0, n1, rr = Aloc.shape[:4]
        N = rl * n0 * n1 * rr
        X = np.linalg.solve(Aloc.reshape(N, N), rhs.reshape(N)).reshape(rl, n0, n1, rr)
        M = X.reshape(rl * n0, n1 * rr)
        U, S, Vt = svd(M)
        k = svd_rank(S, target[cur], EPSILON)
        U, S, Vt = U[:, :k], S[:k], Vt[:k, :]
        if increasing:   # (U(i^2,j), S, x(k,l&1)) = SVD(x(i^2,l&2), targetRank[currIndex]); x = S x
            x.cores[cur] = U.reshape(rl, n0, k)
            x.cores[cur + 1] = (S[:, None] * Vt).reshape(k, n1, rr)
        else:            # (x(i&1,j), S, Vt(k,l&1)) = SVD(x(i&2,l^2), targetRank[currIndex]); x = x S
            x.cores[cur] = (U * S[None, :]).reshape(rl, n0, k)
            x.cores[cur + 1] = Vt.reshape(k, n1, rr)
        x.canonicalized = False
        at_end = (not increasing and cur == first) or (increasing and cur == first_not - s)
        if at_end:
            half += 1
            last2, last, en = last, en, energy()
            if half == num_half_sweeps or abs(last - en) < eps or abs(last2 - en) < eps or first_not - first <= s:
                if canon_end and preserve_core:
                    x.move_core(core_end, keep_rank=True)
                return en
            increasing = not increasing
        if increasing:
            oR.pop()
            oL.append(op_left(oL[-1], cur))
            bR.pop()
            bL.append(rhs_left(bL[-1], cur))
            cur += 1
        else:
            oL.pop()
            oR.append(op_right(oR[-1], cur + s - 1))
            bL.pop()
            bR.append(rhs_right(bR[-1], cur + s - 1))
            cur -= 1


# ------------------------------------------------------------------------------------------------
# Measurement sets and ADF (measurments.cpp, algorithms/adf.cpp). Test infrastructure: the reference's
# algorithm on numpy, with every stack entry computed per measurement (the reference's de-duplication of
# equal position prefixes, adf.cpp:102-191, shares identical products and changes no value).
def uniform_index(rng: Rng, n: int) -> int:
    """libstdc++ std::uniform_int_distribution<size_t>(0, n - 1)(mt19937_64): the 'downscaling' branch
    (urng range 2^64 - 1 > n - 1): scaling = (2^64 - 1) // n, reject draws >= n * scaling, then divide."""
    urngrange = (1 << 64) - 1
    scaling = urngrange // n
    past = n * scaling
    while True:
        v = int(_lib().orc_rng_next(rng._state))
        if v < past:
            return v // scaling


def sp_random_positions(rng: Rng, num: int, dims: Sequence[int]) -> np.ndarray:
    """SinglePointMeasurementSet::create_random_positions (measurments.cpp:211-236): distinct multi-indices
    drawn mode by mode, then sorted lexicographically."""
    seen, pos = set(), []
    while len(pos) < num:
        idx = [uniform_index(rng, int(n)) for n in dims]
        lin = 0
        for i, n in zip(idx, dims):
            lin = lin * int(n) + i
        if lin not in seen:
            seen.add(lin)
            pos.append(idx)
    pos.sort()
    return np.asarray(pos, dtype=np.int64).reshape(num, len(dims))


def tt_measure_sp(x: TT, pos: np.ndarray) -> np.ndarray:
    """x[positions] (SinglePointMeasurementSet::measure(TensorNetwork), measurments.cpp:120-148)."""
    F = np.ones((pos.shape[0], 1))
    for k, C in enumerate(x.cores):
        F = np.einsum("ma,amb->mb", F, C[:, pos[:, k], :])
    return F[:, 0]


def tt_measure_r1(x: TT, vecs: Sequence[np.ndarray]) -> np.ndarray:
    """<x, v_0 (x) ... (x) v_{d-1}> per measurement (RankOneMeasurementSet::measure, measurments.cpp:393-420)."""
    F = np.ones((vecs[0].shape[0], 1))
    for k, C in enumerate(x.cores):
        F = np.einsum("ma,mt,atb->mb", F, vecs[k], C)
    return F[:, 0]


def adf(x: TT, values: np.ndarray, max_ranks: Sequence[int], positions: np.ndarray | None = None,
        vectors: Sequence[np.ndarray] | None = None, max_iterations: int = 0, target: float = 1e-8,
        min_decrease: float = 0.999, rng: Rng | None = None) -> float:
    """ADFVariant::InternalSolver::solve (adf.cpp:566-604) with solve_with_current_ranks (:489-542) for a
    SinglePointMeasurementSet (positions, M x d) or a RankOneMeasurementSet (vectors[k]: M x n_k). x is
    updated in place; returns the final relative residual norm."""
    sp = positions is not None
    d = x.order
    dims = x.dims
    M = len(values)
    values = np.asarray(values, dtype=np.float64)
    max_ranks = reduce_to_maximal_ranks(list(max_ranks), dims)
    norm_meas = float(np.sqrt(np.sum(values ** 2)))   # :37-43 (sequential sum of squares)
    state = {"it": 0, "res": np.finfo(float).max, "last": np.finfo(float).max}

    def slices(C, k):   # (M, a, b): the component's matrix for each measurement
        if sp:
            return np.transpose(C[:, positions[:, k], :], (1, 0, 2))
        return np.einsum("mt,atb->mab", vectors[k], C)

    def value(Fm, C, Bm, k):   # Fm (M, a) . slice . Bm (M, b)
        return np.einsum("ma,mab,mb->m", Fm, slices(C, k), Bm)

    def solve_current():
        rd1 = rd2 = rd3 = 0.0
        Fs = {-1: np.ones((M, 1))}
        while max_iterations == 0 or state["it"] < max_iterations:
            x.move_core(0, keep_rank=True)
            Bs = {d: np.ones((M, 1))}
            for k in range(d - 1, 0, -1):   # :499-501
                Bs[k] = np.einsum("mab,mb->ma", slices(x.cores[k], k), Bs[k + 1])
            res = values - value(Fs[-1], x.cores[0], Bs[1], 0)
            state["last"] = state["res"]
            state["res"] = float(np.sqrt(np.sum(res ** 2))) / norm_meas
            rd4, rd3, rd2 = rd3, rd2, rd1
            rd1 = state["res"] / state["last"]
            if state["res"] < target or rd1 * rd2 * rd3 * rd4 > min_decrease ** 4:   # :520
                break
            for k in range(d):   # :524-540
                C = x.cores[k]
                a, n, b = C.shape
                if k > 0:
                    res = values - value(Fs[k - 1], C, Bs[k + 1], k)
                # projected gradient (:360-396): sum_m res_m F_m (x) e_pos / v_m (x) B_m
                w = res[:, None, None] * Fs[k - 1][:, :, None] * Bs[k + 1][:, None, :]   # (M, a, b)
                if sp:
                    G = np.zeros((n, a, b))
                    np.add.at(G, positions[:, k], w)
                else:
                    G = np.einsum("mt,mab->tab", vectors[k], w)
                D = np.ascontiguousarray(np.transpose(G, (1, 0, 2)))   # (a, n, b)
                # slicewise ||A(E(grad))||^2 (:413-465)
                vals2 = value(Fs[k - 1], D, Bs[k + 1], k) ** 2
                if sp:
                    nrm = np.zeros(n)
                    np.add.at(nrm, positions[:, k], vals2)
                else:
                    nrm = np.array([np.sum(vals2)])
                # update (:468-487)
                if sp:
                    for j in range(n):
                        pyr = float(np.sum(D[:, j, :] ** 2))
                        C[:, j, :] = C[:, j, :] + (pyr / nrm[j]) * D[:, j, :]
                else:
                    C[...] = C + (float(np.sum(D ** 2)) / float(np.sum(nrm))) * D
                x.cores[k] = C
                if k + 1 < d:
                    x.move_core(k + 1, keep_rank=True)
                    Fs[k] = np.einsum("ma,mab->mb", Fs[k - 1], slices(x.cores[k], k))
            state["it"] += 1

    x.move_core(0)   # canonicalize_left (:582)
    solve_current()
    while state["res"] > target and x.ranks != max_ranks and (max_iterations == 0 or state["it"] < max_iterations):
        x.move_core(0, keep_rank=True)   # :592-597: x + 1e-6 ||x|| rnd / ||rnd||, rnd a random rank-1 TT
        rnd = TT.random(dims, [1] * (d - 1), rng)
        nrnd = rnd.frob_norm()
        diff = rnd.copy()
        diff.cores[diff.core_position] = diff.cores[diff.core_position] * (1e-6 * x.frob_norm())
        diff.cores[diff.core_position] = diff.cores[diff.core_position] / nrnd
        x_new = tt_add(x, diff)
        x_new.move_core(0)                # the sum of canonical TTs is re-canonicalised (ttNetwork.cpp:841-843)
        x.cores, x.canonicalized, x.core_position = x_new.cores, x_new.canonicalized, x_new.core_position
        x.round(max_ranks)
        solve_current()
    return state["res"]


def tt_ones(dims: Sequence[int]) -> TT:
    """TTNetwork::ones (ttNetwork.cpp:170-191): all-ones rank-1 components, then canonicalize_left."""
    x = TT([np.ones((1, int(n), 1)) for n in dims])
    x.move_core(0)
    return x
