"""Mode-sharded TT round / <x,y> through the C-ABI (xrs_tt_round_sharded, xrs_tt_dot_sharded).

Two ranks share the box's single GPU (gloo all-reduce with host staging); one rank with the nccl
(= RCCL) backend and ``force_hook`` exercises the device-native all-reduce path (dist.all_reduce on the
device buffer through __cuda_array_interface__) and must give the null-hook results. Parity: same ranks
as the oracle's round, same represented tensor, <x,y> within 1e-12 ||x|| ||y||.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel_diff(ref, a_cores, b_cores):
    A = ref.TT([c.copy() for c in a_cores])
    nb = [c.copy() for c in b_cores]
    nb[0] = -nb[0]
    D = ref.tt_add(A, ref.TT(nb))
    D.move_core(0)
    B = ref.TT([c.copy() for c in b_cores])
    B.move_core(0)
    return D.frob_norm() / B.frob_norm()


def _worker(rank, world, port, backend, hook, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from oracle import xerus_ref as ref
        from xerus_amd import capi
        from xerus_amd import dist as xd

        torch.cuda.set_device(0)
        h = capi.Handle(0)
        comm = xd.RcclComm(h) if hook == "rccl" else xd.TorchAllReduce(force_hook=(hook == "force"))
        force = hook != "none"
        dims, ranks = [8, 6, 7, 5, 8, 6], [6, 12, 12, 10, 6]
        x = ref.TT.random_raw(dims, ranks, ref.Rng(31))
        y = ref.TT.random_raw(dims, ranks, ref.Rng(37))
        sx = xd.ShardedTT.from_full_cores(h, x.cores, world, rank)
        sy = xd.ShardedTT.from_full_cores(h, y.cores, world, rank)
        d_sh = sx.dot(sy, comm)
        d_ref = ref.dot(x, y)
        nx, ny = np.sqrt(ref.dot(x, x)), np.sqrt(ref.dot(y, y))
        # odd order: the two-ended zipper's left end idles in the last step
        dims7, ranks7 = [5, 6, 4, 7, 5, 6, 4], [5, 9, 11, 9, 8, 4]
        x7 = ref.TT.random_raw(dims7, ranks7, ref.Rng(41))
        y7 = ref.TT.random_raw(dims7, ranks7, ref.Rng(43))
        d7 = xd.ShardedTT.from_full_cores(h, x7.cores, world, rank).dot(
            xd.ShardedTT.from_full_cores(h, y7.cores, world, rank), comm)
        n7 = np.sqrt(ref.dot(x7, x7) * ref.dot(y7, y7))
        dot7_err = abs(d7 - ref.dot(x7, y7)) / n7
        cert = sx.round(12, comm)
        full = sx.gather(dist.all_gather_object)
        res = {"dot_err": abs(d_sh - d_ref) / (nx * ny), "dot7_err": dot7_err, "cert": cert, "ranks": sx.ranks}
        if rank == 0:
            xr = x.copy()
            xr.round(12)
            res["ref_ranks"] = xr.ranks
            res["diff"] = _rel_diff(ref, full, x.cores)
            # right-canonical: cores 1.. have orthonormal rows
            xs = ref.tt_add(x, x)
            xs.round(100)
            res["ref_ranks_sum"] = xs.ranks
            res["orth"] = max(np.abs(c.reshape(c.shape[0], -1) @ c.reshape(c.shape[0], -1).T - np.eye(c.shape[0])).max()
                              for c in full[1:])
        # doubled ranks (x + x): certificate must fail, cores untouched
        s2 = ref.tt_add(x, x)
        ss = xd.ShardedTT.from_full_cores(h, s2.cores, world, rank)
        before = ss.local.cores()
        res["cert_sum"] = ss.round(100, comm)
        after = ss.local.cores()
        res["untouched"] = all(np.array_equal(a, b) for a, b in zip(before, after))
        # ... and round_any completes it: device all-gather (xrs_tt_gather_sharded), the single-GPU round on
        # every rank, local re-shard (xrs_tt_shard); gather_device of the result on every rank
        res["any_path"] = ss.round_any(100, comm)
        res["any_ranks"] = ss.ranks
        g_full = ss.gather_device(comm)
        res["any_full"] = g_full.cores() if rank == 0 else None
        g_full.free()
        # device gather of an untouched sharded TT reproduces the full cores bit for bit
        gx = xd.ShardedTT.from_full_cores(h, y.cores, world, rank).gather_device(comm)
        res["gather_exact"] = all(np.array_equal(a, b) for a, b in zip(gx.cores(), y.cores))
        gx.free()
        # truncating sharded round (ranks 12 -> 8): the certified truncation with all-reduced Grams
        st = xd.ShardedTT.from_full_cores(h, x.cores, world, rank)
        res["cert_trunc"] = st.round(8, comm)
        full_t = st.gather(dist.all_gather_object)
        res["trunc_ranks"] = st.ranks
        if rank == 0:
            from ttutil import tt_diff_norm
            xo = x.copy()
            xo.round(8)
            res["trunc_ref_ranks"] = xo.ranks
            e_gpu, nrm = tt_diff_norm(full_t, x.cores)
            e_ref, _ = tt_diff_norm(xo.cores, x.cores)
            res["trunc_err_diff"] = abs(e_gpu - e_ref) / nrm
        res["calls"] = comm.calls
        res["device_native"] = comm.device_native
        if force:   # the same work with no hook (one rank): identical results
            null = xd.TorchAllReduce()
            assert null.c_fn is None
            sx0 = xd.ShardedTT.from_full_cores(h, x.cores, world, rank)
            sy0 = xd.ShardedTT.from_full_cores(h, y.cores, world, rank)
            res["dot_null_diff"] = abs(sx0.dot(sy0, null) - d_sh) / (nx * ny)
            sx0.round(12, null)
            res["round_null_diff"] = max(float(np.abs(a - b).max()) for a, b in zip(sx0.local.cores(), sx.local.cores()))
        out[rank] = res
        h.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,backend,hook", [(2, "gloo", "none"), (1, "nccl", "force"), (1, "nccl", "rccl")])
def test_sharded_round_and_dot(world, backend, hook):
    """hook: "none" (torch.distributed callback; a NULL hook at world 1), "force" (the callback even at world
    1: dist.all_reduce on the device buffer), "rccl" (xrs_comm_allreduce: C++ RCCL, stream-ordered)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), backend, hook, out), nprocs=world, join=True)
    force = hook != "none"
    r0 = out[0]
    for rank in range(world):
        r = out[rank]
        assert r["dot_err"] <= 1e-12
        assert r["dot7_err"] <= 1e-12
        assert r["cert"] is True
        assert r["ranks"] == r0["ref_ranks"]
        assert r["cert_sum"] is False and r["untouched"]
        assert r["any_path"] == "gathered"
        assert r["any_ranks"] == r0["ref_ranks_sum"]
        assert r["gather_exact"]
    assert r0["diff"] <= 1e-12
    from oracle import xerus_ref as ref
    from ttutil import tt_diff_norm
    x = ref.TT.random_raw([8, 6, 7, 5, 8, 6], [6, 12, 12, 10, 6], ref.Rng(31))
    e, nrm = tt_diff_norm(r0["any_full"], [2 * c if k == 0 else c for k, c in enumerate(x.cores)])
    assert e <= 1e-12 * nrm
    assert r0["orth"] <= 1e-13
    assert r0["calls"] > 0
    for rank in range(world):
        assert out[rank]["cert_trunc"] is True
        assert out[rank]["trunc_ranks"] == r0["trunc_ref_ranks"]
    assert r0["trunc_err_diff"] <= 1e-6
    if force:
        assert r0["device_native"] is True
        assert r0["dot_null_diff"] <= 1e-15
        assert r0["round_null_diff"] <= 1e-13
