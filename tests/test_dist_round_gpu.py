"""Sharded truncating rounds that used to gather onto one device: xrs_tt_round_sharded_ex over
world 2 / 3 gloo ranks, all on the box's one GPU.

  - (x + y).round(128) at the BASELINE configs[2] shape (order 10, n = 20, rank 128 each): the sum's left-end
    structural excess (QC steps on the gathered core) and its tall right edge (gathered, replicated);
  - a graded spectrum (raw cores, right rank index scaled by 0.8^j) round(64) and round(eps = 1e-8): the
    sharded general round (shifted CholeskyQR3 + Jacobi SVDs, device-side rank cuts);
  - a small x + y over 3 ranks with uneven mode blocks (n = 5: 2 / 2 / 1 slices).

Reference: TTNetwork::round (ttNetwork.cpp:644-665), TTNetwork::operator+= (ttNetwork.cpp:797-847); the
sharded form is new design. Bars: the round stays sharded (no gather); the oracle's ranks;
truncation error within 1e-6 ||s|| of the oracle's, and the result within 1e-6 ||s|| of the oracle's
result where the kept subspace is unique (the graded spectra); every rank holds the same result.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cases(ref):
    """name -> (full cores, max ranks, eps); deterministic (the oracle's Rng)."""
    out = {}
    d, n, r = 10, 20, 128
    ranks = bench.tt_ranks(d, n, r)[1:-1]
    x = ref.TT.random_raw([n] * d, ranks, ref.Rng(21))
    y = ref.TT.random_raw([n] * d, ranks, ref.Rng(22))
    out["sum128"] = (ref.tt_add(x, y).cores, [128] * (d - 1), 8 * np.finfo(float).eps)
    g = ref.TT.random_raw([n] * d, ranks, ref.Rng(23))
    gc = [c.copy() for c in g.cores]
    for k in range(d - 1):
        gc[k] = gc[k] * (0.8 ** np.arange(gc[k].shape[2]))[None, None, :]
    out["graded64"] = (gc, [64] * (d - 1), 8 * np.finfo(float).eps)
    out["graded_eps"] = (gc, [2 ** 62] * (d - 1), 1e-8)
    return out


def _small_cases(ref):
    d, n = 5, 5
    ranks = bench.tt_ranks(d, n, 6)[1:-1]
    x = ref.TT.random_raw([n] * d, ranks, ref.Rng(31))
    y = ref.TT.random_raw([n] * d, ranks, ref.Rng(32))
    return {"small_sum": (ref.tt_add(x, y).cores, [4] * (d - 1), 8 * np.finfo(float).eps)}


def _worker(rank, world, port, which, out):
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
        cases = _cases(ref) if which == "big" else _small_cases(ref)
        res = {}
        for name, (cores, mr, eps) in cases.items():
            st = xd.ShardedTT.from_full_cores(h, cores, world, rank)
            path = st.round_sharded(mr, comm, eps)
            full = st.gather_device(comm)
            fc = full.cores()
            rec = {"path": path, "ranks": list(full.r), "checksum": float(sum(np.abs(c).sum() for c in fc))}
            if rank == 0:
                e, nrm = tt_diff_norm(fc, cores)
                rec["err"], rec["nrm"] = e, nrm
                g = capi.TTDevice.from_cores(h, cores)
                g.round(mr, eps)
                rec["single_path"] = h.last_round_path()
                rec["diff_single"] = tt_diff_norm(fc, g.cores())[0] / nrm
                xo = ref.TT([c.copy() for c in cores])
                xo.round(mr, eps)
                rec["oracle_ranks"] = list(xo.ranks)
                rec["oracle_err"] = tt_diff_norm(xo.cores, cores)[0]
                rec["diff_oracle"] = tt_diff_norm(fc, xo.cores)[0] / nrm
                g.free()
            full.free()
            st.local.free()
            res[name] = rec
        out[rank] = res
        h.close()
    finally:
        dist.destroy_process_group()


def _run(world, which):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), which, out), nprocs=world, join=True)
    return dict(out)


def _check(out, world, unique):
    r0 = out[0]
    for name, rec in r0.items():
        assert rec["path"] in ("chain", "truncate", "general"), (name, rec["path"])
        for q in range(1, world):
            assert out[q][name]["path"] == rec["path"]
            assert out[q][name]["ranks"] == rec["ranks"]
            assert out[q][name]["checksum"] == rec["checksum"]   # the same gathered result on every rank
        assert rec["ranks"][1:-1] == rec["oracle_ranks"], (name, rec["ranks"], rec["oracle_ranks"])
        nrm = rec["nrm"]
        assert abs(rec["err"] - rec["oracle_err"]) <= 1e-6 * nrm, (name, rec["err"] / nrm, rec["oracle_err"] / nrm)
        assert rec["diff_single"] <= 1e-8, (name, rec["diff_single"])
        if name in unique:
            assert rec["diff_oracle"] <= 1e-6, (name, rec["diff_oracle"])
        print(f"{name} (world {world}): path {rec['path']}, ranks {rec['ranks'][1:-1]}, error {rec['err'] / nrm:.6e} "
              f"(oracle {rec['oracle_err'] / nrm:.6e}), vs single GPU {rec['diff_single']:.2e}, "
              f"vs oracle {rec['diff_oracle']:.2e}")


def test_sharded_sum_and_graded_rounds_world2():
    out = _run(2, "big")
    _check(out, 2, unique=("graded64", "graded_eps"))
    assert out[0]["graded64"]["path"] == "general"
    assert out[0]["graded_eps"]["path"] == "general"


def test_sharded_small_sum_world3_uneven():
    out = _run(3, "small")
    _check(out, 3, unique=())


def test_emulated_comm_rank0_of_replicated_tt(handle, ref):
    """xrs_comm_emulate (the per-rank timing probe's communicator, tools/cfg5_rank_probe.py): rank 0 of 3
    ranks holding identical slices equals the first m slices of the single-GPU round of the TT whose modes are
    the local block repeated 3 times (the chain round and the truncating round)."""
    from xerus_amd import capi
    from xerus_amd import dist as xd

    d, m, world = 6, 4, 3
    ranks = bench.tt_ranks(d, m, 12)[1:-1]
    x = ref.TT.random_raw([m] * d, ranks, ref.Rng(41))
    full = [np.concatenate([c] * world, axis=1) for c in x.cores]
    comm = xd.EmulatedComm(handle, world)
    try:
        for target in (12, 5):
            st = xd.ShardedTT(handle, capi.TTDevice.from_cores(handle, x.cores), [m * world] * d, world, 0)
            path = st.round_sharded(target, comm)
            assert path in ("chain", "truncate"), path
            g = capi.TTDevice.from_cores(handle, full)
            g.round(target)
            assert st.ranks == g.ranks
            # the represented tensors on rank 0's index block (the cores' gauge may differ by signs)
            a = ref.TT(st.local.cores()).full()
            b = ref.TT([c[:, :m, :] for c in g.cores()]).full()
            assert np.linalg.norm(a - b) <= 1e-10 * np.linalg.norm(b), (target, np.linalg.norm(a - b) / np.linalg.norm(b))
            st.local.free()
            g.free()
        assert comm.calls > 0
    finally:
        comm.close()


def test_emulated_comm_tall_right_edge_reports_uncertified(handle, ref):
    """under xrs_comm_emulate a core "gathered" by the all-reduce of a zero-padded block is nranks x
    rank 0's block, not the TT's core. A sum whose right edge is tall (r_{d-1} = 4 > n = 3) and whose first edge
    has structural excess needs such gathers: the round must report uncertified (path "") and leave the
    represented tensor as it was, not factorise a wrong matrix."""
    from xerus_amd import capi
    from xerus_amd import dist as xd

    d, world = 5, 3
    x = ref.TT.random_raw([1] * d, [2] * (d - 1), ref.Rng(51))
    y = ref.TT.random_raw([1] * d, [2] * (d - 1), ref.Rng(52))
    s = ref.tt_add(x, y)   # local mode size 1 (global 3), ranks 4: tall right edge, left excess
    before = ref.TT([c.copy() for c in s.cores]).full()
    comm = xd.EmulatedComm(handle, world)
    try:
        st = xd.ShardedTT(handle, capi.TTDevice.from_cores(handle, s.cores), [world] * d, world, 0)
        path = st.round_sharded(3, comm)
        assert path == "", path
        after = ref.TT(st.local.cores()).full()
        assert np.linalg.norm(after - before) <= 1e-12 * np.linalg.norm(before)
        st.local.free()
    finally:
        comm.close()
