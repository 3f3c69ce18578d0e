"""BASELINE configs[4] in its sharded form: TTTensor order 16, n = 20, rank 512, cores split by mode slices
over two ranks (gloo, both ranks on the box's one GPU) -- xrs_tt_round_sharded (round(512), the certified
chain round), xrs_tt_dot_sharded, and the truncating round(256) through ShardedTT.round_any.

Reference: TTNetwork::round (ttNetwork.cpp:644-665) and the TT inner product (ttNetwork.cpp:782-789); the
sharded form is new design. Bars: same ranks as the oracle; round(512) represents
the input and the single-GPU result to 1e-10 ||x||; <x,y> within 1e-12 ||x|| ||y|| of the oracle; truncation
errors of the sharded round(256) equal the oracle's to 1e-6 ||x||, and it stays sharded (no gather); the
certificate holds.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

D, N, R = 16, 20, 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import xerus_ref as ref
        from ttutil import tt_diff_norm
        from xerus_amd import capi
        from xerus_amd import dist as xd

        torch.cuda.set_device(0)
        h = capi.Handle(0)
        comm = xd.TorchAllReduce()
        ranks = bench.tt_ranks(D, N, R)[1:-1]
        x = ref.TT.random_raw([N] * D, ranks, ref.Rng(5))
        y = ref.TT.random_raw([N] * D, ranks, ref.Rng(6))
        res = {}
        sx = xd.ShardedTT.from_full_cores(h, x.cores, world, rank)
        sy = xd.ShardedTT.from_full_cores(h, y.cores, world, rank)
        res["dot"] = sx.dot(sy, comm)
        res["dot_xx"] = sx.dot(sx, comm)
        sy.local.free()
        res["cert"] = sx.round(R, comm)
        res["ranks"] = sx.ranks
        res["calls"] = comm.calls
        full = sx.gather_device(comm)
        if rank == 0:
            fc = full.cores()
            g = capi.TTDevice.from_cores(h, x.cores)
            g.round(R)
            diff, nrm = tt_diff_norm(fc, g.cores())
            res["diff_single"] = diff / nrm
            diff, nrm = tt_diff_norm(fc, x.cores)
            res["diff_input"] = diff / nrm
            res["orth"] = max(float(np.abs(c.reshape(c.shape[0], -1) @ c.reshape(c.shape[0], -1).T
                                           - np.eye(c.shape[0])).max()) for c in fc[1:])
            g.free()
            del fc
        full.free()
        sx.local.free()
        # truncating round(256): the certified sharded truncation, or the device gather + single-GPU round
        st = xd.ShardedTT.from_full_cores(h, x.cores, world, rank)
        res["trunc_path"] = st.round_any(256, comm)
        res["trunc_ranks"] = st.ranks
        full_t = st.gather_device(comm)
        if rank == 0:
            e, nrm = tt_diff_norm(full_t.cores(), x.cores)
            res["trunc_err"], res["nrm"] = e, nrm
        full_t.free()
        st.local.free()
        out[rank] = res
        h.close()
    finally:
        dist.destroy_process_group()


def test_cfg5_sharded_world2(ref):
    from ttutil import tt_diff_norm

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ranks = bench.tt_ranks(D, N, R)[1:-1]
    x = ref.TT.random_raw([N] * D, ranks, ref.Rng(5))
    y = ref.TT.random_raw([N] * D, ranks, ref.Rng(6))
    d_ref = ref.dot(x, y)
    nx2, ny2 = ref.dot(x, x), ref.dot(y, y)
    nx, ny = np.sqrt(nx2), np.sqrt(ny2)
    r0 = out[0]
    for rank in range(world):
        r = out[rank]
        assert r["cert"] is True
        assert r["ranks"] == ranks                    # round(512) keeps the oracle's (= the input) ranks
        assert abs(r["dot"] - d_ref) <= 1e-12 * nx * ny, abs(r["dot"] - d_ref) / (nx * ny)
        assert abs(r["dot_xx"] - nx2) <= 1e-12 * nx2
        assert r["calls"] > 0                         # the all-reduces went through the collective
        assert r["trunc_path"] == "sharded"            # xrs_tt_round_sharded_ex: no gather
        assert r["trunc_ranks"] == r0["trunc_ranks"]
    assert r0["diff_input"] <= 1e-10, r0["diff_input"]
    assert r0["diff_single"] <= 1e-10, r0["diff_single"]
    assert r0["orth"] <= 1e-12, r0["orth"]
    xo = x.copy()
    xo.round(256)
    assert r0["trunc_ranks"] == xo.ranks
    e_ref, nrm = tt_diff_norm(xo.cores, x.cores)
    assert abs(r0["trunc_err"] - e_ref) <= 1e-6 * nrm, (r0["trunc_err"] / nrm, e_ref / nrm)
    print(f"cfg5 sharded world 2: round(512) diff vs single GPU {r0['diff_single']:.2e}, truncating path "
          f"{r0['trunc_path']}, truncation error {r0['trunc_err'] / nrm:.6e} (oracle {e_ref / nrm:.6e})")
