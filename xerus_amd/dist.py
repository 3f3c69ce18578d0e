"""Mode-sharded TT round and inner product across ranks.

xerus is single-process (no MPI/NCCL anywhere in the reference), so this layer is new design, not a
port. Layout: every rank holds, for every TT component k, a contiguous block of the mode index
(``mode_partition``) -- the row blocks of the tall unfolding (r_k n_k) x r_{k+1}. Every quantity the
round needs that sums over the mode index -- the left/right Gram chains, the orthogonality check, the
<x,y> zipper environments -- is a local GEMM followed by one all-reduce of an r x r matrix
(``xrs_allreduce_fn``, bound here to torch.distributed: RCCL over xGMI with the "nccl" backend, or
gloo with host staging); the per-core transforms are purely local. No data-path all-gather is needed.

The product path is the HIP library (xrs_tt_round_sharded / xrs_tt_dot_sharded); a round whose
certificate fails gathers the TT device to device (xrs_tt_gather_sharded: one all-gather), rounds it on
every rank and re-shards locally (ShardedTT.round_any). The helpers below only partition and move bytes.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Sequence

import numpy as np

from . import capi

ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)


def mode_partition(n: int, world: int, rank: int) -> tuple[int, int]:
    """Balanced contiguous block [start, start+count) of the mode index 0..n-1 owned by `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def shard_cores(cores: Sequence[np.ndarray], world: int, rank: int) -> list[np.ndarray]:
    """This rank's mode slices of full cores (r_k, n_k, r_{k+1})."""
    out = []
    for c in cores:
        s, m = mode_partition(c.shape[1], world, rank)
        out.append(np.ascontiguousarray(c[:, s:s + m, :]))
    return out


def unshard_cores(parts: Sequence[Sequence[np.ndarray]]) -> list[np.ndarray]:
    """Reassemble full cores from every rank's slices (parts[rank][k]), in rank order."""
    d = len(parts[0])
    return [np.concatenate([p[k] for p in parts], axis=1) for k in range(d)]


class _CudaArray:
    """__cuda_array_interface__ view of raw device memory (float64)."""

    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False), "version": 3}


class TorchAllReduce:
    """xrs_allreduce_fn backed by torch.distributed (sum, in place on the device buffer).

    nccl (= RCCL on ROCm) reduces the device buffer directly; gloo reduces a host copy. At world size 1
    no hook is handed to the C side (the local sums are the global ones) unless ``force_hook`` is set:
    then every reduction still goes through the collective (tests of the RCCL branch on one GPU)."""

    def __init__(self, group=None, force_hook: bool = False):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        initialized = dist.is_available() and dist.is_initialized()
        self.single = not initialized or (dist.get_world_size(group) == 1 and not force_hook)
        self.device_native = (not self.single) and dist.get_backend(group) == "nccl"
        self.calls = 0
        self.bytes = 0

        def _cb(_ctx, ptr, count):
            if self.single:   # one rank: the local sum is the global sum
                self.calls += 1
                return 0
            try:
                t = self.torch.as_tensor(_CudaArray(int(ptr), int(count)), device="cuda")
                if self.device_native:
                    self.dist.all_reduce(t, group=self.group)
                    self.torch.cuda.synchronize()
                else:
                    h = t.cpu()
                    self.dist.all_reduce(h, group=self.group)
                    t.copy_(h)
                    self.torch.cuda.synchronize()
                self.calls += 1
                self.bytes += 8 * int(count)
                return 0
            except Exception:   # reported to the C side as a failed collective
                return 1

        def _ag(_ctx, send, recv, count):
            try:
                world = self.dist.get_world_size(self.group)
                ts = self.torch.as_tensor(_CudaArray(int(send), int(count)), device="cuda")
                tr = self.torch.as_tensor(_CudaArray(int(recv), int(count) * world), device="cuda")
                if self.device_native:
                    self.dist.all_gather_into_tensor(tr, ts, group=self.group)
                else:
                    parts = [self.torch.empty(int(count), dtype=self.torch.float64) for _ in range(world)]
                    self.dist.all_gather(parts, ts.cpu(), group=self.group)
                    tr.copy_(self.torch.cat(parts).to(tr.device))
                self.torch.cuda.synchronize()
                self.calls += 1
                self.bytes += 8 * int(count) * world
                return 0
            except Exception:
                return 1

        self.fn = ALLREDUCE_FN(_cb)   # keep a reference: the C side only holds the pointer
        self.ag = ALLGATHER_FN(_ag)
        self.ctx = None

    @property
    def c_fn(self):
        # one rank: no hook at all (the C side then skips the stream synchronisation a hook needs)
        return None if self.single else C.cast(self.fn, C.c_void_p)

    @property
    def c_ag(self):
        return None if self.single else C.cast(self.ag, C.c_void_p)


class RcclComm:
    """The library's own RCCL communicator (xrs_comm_t) as the all-reduce hook: collectives are enqueued
    on the handle's stream by C++ (xrs_comm_allreduce), no Python callback and no host synchronisation per
    collective. The 128-byte unique id is broadcast over the existing torch.distributed group."""

    def __init__(self, handle: capi.Handle, group=None):
        import torch.distributed as dist

        self.handle, self.lib = handle, handle.lib
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        buf = C.create_string_buffer(128)
        if rank == 0:
            capi._check("xrs_comm_unique_id", self.lib.xrs_comm_unique_id(buf))
        if world > 1:
            obj = [bytes(buf.raw) if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            buf = C.create_string_buffer(obj[0], 128)
        self.comm = C.c_void_p()
        capi._check("xrs_comm_create", self.lib.xrs_comm_create(handle.h, world, rank, buf, C.byref(self.comm)))
        self.world, self.rank = world, rank
        self.device_native = True

    @property
    def c_fn(self):
        return C.cast(self.lib.xrs_comm_allreduce, C.c_void_p)

    @property
    def c_ag(self):
        return C.cast(self.lib.xrs_comm_allgather, C.c_void_p)

    @property
    def ctx(self):
        return self.comm

    @property
    def calls(self) -> int:
        return int(self.lib.xrs_comm_calls(self.comm))

    def close(self):
        if self.comm:
            capi._check("xrs_comm_destroy", self.lib.xrs_comm_destroy(self.comm))
            self.comm = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EmulatedComm(RcclComm):
    """xrs_comm_emulate: rank 0 of `world` ranks holding identical slices (the sum over ranks is `world` x the
    local value, enqueued on the stream). Per-rank timing of the sharded path on one GPU; not a collective.
    Rounds whose steps need a gathered core (tall right edges, left structural excess) report uncertified under
    it: a zero-padded core summed this way is not the TT's core."""

    def __init__(self, handle: capi.Handle, world: int):
        self.handle, self.lib = handle, handle.lib
        self.comm = C.c_void_p()
        capi._check("xrs_comm_emulate", self.lib.xrs_comm_emulate(handle.h, world, C.byref(self.comm)))
        self.world, self.rank = world, 0
        self.device_native = True


class ShardedTT:
    """This rank's mode slices of a TT (capi.TTDevice over the local slices) + the global mode sizes."""

    def __init__(self, handle: capi.Handle, local: capi.TTDevice, dims: Sequence[int], world: int, rank: int):
        self.handle, self.local, self.dims, self.world, self.rank = handle, local, list(dims), world, rank

    @classmethod
    def from_full_cores(cls, handle: capi.Handle, cores, world: int, rank: int) -> "ShardedTT":
        dims = [c.shape[1] for c in cores]
        return cls(handle, capi.TTDevice.from_cores(handle, shard_cores(cores, world, rank)), dims, world, rank)

    @property
    def ranks(self):
        return self.local.ranks

    def round(self, max_ranks, comm, eps: float = 8 * np.finfo(float).eps) -> bool:
        """Certified sharded round in place (TorchAllReduce or RcclComm); returns False (cores untouched) if
        the certificate fails -- gather and round on one device then."""
        t = self.local
        d = t.order
        if isinstance(max_ranks, (int, np.integer)):
            max_ranks = [int(max_ranks)] * (d - 1)
        n, r, cores = t._arrays()
        mr = capi._arr(list(max_ranks) + [1])
        cert = C.c_int(0)
        st = self.handle.lib.xrs_tt_round_sharded(self.handle.h, d, n, r, cores, mr, eps, comm.c_fn, comm.ctx,
                                                  C.byref(cert))
        t._writeback(r, cores)
        capi._check("xrs_tt_round_sharded", st)
        if cert.value:
            t.canonicalized, t.core_position = True, 0
        return bool(cert.value)

    def round_sharded(self, max_ranks, comm, eps: float = 8 * np.finfo(float).eps) -> str:
        """Sharded round for any spectrum (xrs_tt_round_sharded_ex: chain, certified truncation or the general
        round, all on the slices; tall right edges and left-end QC steps on cores gathered by one all-reduce).
        Returns "chain" / "truncate" / "general", or "" if every certificate failed (same tensor, left-end QC
        steps possibly applied -- gather and round on one device then)."""
        t = self.local
        d = t.order
        if isinstance(max_ranks, (int, np.integer)):
            max_ranks = [int(max_ranks)] * (d - 1)
        n, r, cores = t._arrays()
        mr = capi._arr(list(max_ranks) + [1])
        path = C.c_int(0)
        st = self.handle.lib.xrs_tt_round_sharded_ex(self.handle.h, d, n, r, cores, mr, eps, self.world, self.rank,
                                                     comm.c_fn, comm.ctx, C.byref(path))
        t._writeback(r, cores)
        capi._check("xrs_tt_round_sharded_ex", st)
        if path.value:
            t.canonicalized, t.core_position = True, 0
        return {1: "chain", 2: "truncate", 4: "general"}.get(path.value, "")

    def dot(self, other: "ShardedTT", comm) -> float:
        x, y = self.local, other.local
        if self.dims != other.dims or x.dims != y.dims:
            raise ValueError(f"dot of sharded TTs with different dimensions: {self.dims} vs {other.dims}")
        d = x.order
        out = C.c_double()
        xc = (capi._DP * d)(*[capi._DP(p) for p in x.ptrs])
        yc = (capi._DP * d)(*[capi._DP(p) for p in y.ptrs])
        capi._check("xrs_tt_dot_sharded",
                    self.handle.lib.xrs_tt_dot_sharded(self.handle.h, C.byref(out), d, capi._arr(x.dims),
                                                       capi._arr(x.r), xc, capi._arr(y.r), yc, comm.c_fn, comm.ctx))
        return out.value

    def gather_device(self, comm) -> capi.TTDevice:
        """Full cores on every rank, device to device (xrs_tt_gather_sharded: one all-gather of the padded
        slices of all components over the communicator's all-gather hook)."""
        t = self.local
        d = t.order
        out = (capi._DP * d)()
        world = self.world if comm.c_ag is not None or self.world > 1 else 1
        src = (capi._DP * d)(*[capi._DP(p) for p in t.ptrs])
        capi._check("xrs_tt_gather_sharded",
                    self.handle.lib.xrs_tt_gather_sharded(self.handle.h, d, capi._arr(self.dims), world, self.rank if world > 1 else 0,
                                                          capi._arr(t.r), src, out, comm.c_ag, comm.ctx))
        return capi.TTDevice(self.handle, self.dims, t.r, [p or 0 for p in out[:]], t.canonicalized, t.core_position)

    def round_any(self, max_ranks, comm, eps: float = 8 * np.finfo(float).eps) -> str:
        """The round for every input: the sharded round ("sharded": chain, certified truncation or general
        round, ShardedTT.round_sharded), else the TT is gathered on the
        device of every rank, rounded there by the single-GPU round (identical inputs and deterministic
        kernels: identical results on every rank) and re-sharded locally ("gathered")."""
        if self.round_sharded(max_ranks, comm, eps):
            return "sharded"
        full = self.gather_device(comm)
        full.round(max_ranks, eps)
        d = full.order
        src = (capi._DP * d)(*[capi._DP(p) for p in full.ptrs])
        out = (capi._DP * d)()
        capi._check("xrs_tt_shard", self.handle.lib.xrs_tt_shard(self.handle.h, d, capi._arr(self.dims), self.world, self.rank,
                                                                 capi._arr(full.r), src, out))
        local_dims = [mode_partition(n, self.world, self.rank)[1] for n in self.dims]
        new = capi.TTDevice(self.handle, local_dims, full.r, [p or 0 for p in out[:]], True, 0)
        full.free()
        self.local.free()
        self.local = new
        return "gathered"

    def gather(self, all_gather_object: Callable) -> list[np.ndarray]:
        """Full cores on every rank (all_gather_object: torch.distributed.all_gather_object-like)."""
        mine = self.local.cores()
        parts = [None] * self.world
        all_gather_object(parts, mine)
        return unshard_cores(parts)
