"""Multi-rank (gloo, world_size 2, CPU) tests of the mode-sharded TT layer (xerus_amd.dist).

The C-ABI sharded kernels need a GPU (tests/test_dist_gpu.py); here the partitioning, gather and the
decomposition they rely on are checked: every mode-index sum of the round (left/right Gram chains) and
of <x,y> (zipper environments) equals the all-reduce of the per-rank partial sums.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xerus_amd import dist as xd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _random_tt(seed, dims, ranks):
    rng = np.random.default_rng(seed)
    r = [1] + list(ranks) + [1]
    return [rng.standard_normal((r[k], dims[k], r[k + 1])) for k in range(len(dims))]


def _left_grams(cores):
    G = [None, cores[0].reshape(-1, cores[0].shape[2]).T @ cores[0].reshape(-1, cores[0].shape[2])]
    for k in range(1, len(cores) - 1):
        a, n, b = cores[k].shape
        T = (G[k] @ cores[k].reshape(a, n * b)).reshape(a * n, b)
        G.append(cores[k].reshape(a * n, b).T @ T)
    return G


def _right_grams(cores):
    d = len(cores)
    H = [None] * d
    M = cores[-1].reshape(cores[-1].shape[0], -1)
    H[d - 1] = M @ M.T
    for k in range(d - 2, 0, -1):
        a, n, b = cores[k].shape
        T = cores[k].reshape(a * n, b) @ H[k + 1]
        H[k] = cores[k].reshape(a, n * b) @ T.reshape(a, n * b).T
    return H


def _sharded_left_grams(local, allreduce):
    """Same chain on this rank's slices, every Gram completed by an all-reduce (what xrs_tt_round_sharded does)."""
    G = [None, local[0].reshape(-1, local[0].shape[2]).T @ local[0].reshape(-1, local[0].shape[2])]
    allreduce(G[1])
    for k in range(1, len(local) - 1):
        a, n, b = local[k].shape
        T = (G[k] @ local[k].reshape(a, n * b)).reshape(a * n, b)
        g = local[k].reshape(a * n, b).T @ T
        allreduce(g)
        G.append(g)
    return G


def _sharded_right_grams(local, allreduce):
    d = len(local)
    H = [None] * d
    M = local[-1].reshape(local[-1].shape[0], -1)
    H[d - 1] = M @ M.T
    allreduce(H[d - 1])
    for k in range(d - 2, 0, -1):
        a, n, b = local[k].shape
        T = local[k].reshape(a * n, b) @ H[k + 1]
        H[k] = local[k].reshape(a, n * b) @ T.reshape(a, n * b).T
        allreduce(H[k])
    return H


def _sharded_dot(x, y, allreduce):
    E = np.ones((1, 1))
    for X, Y in zip(x, y):
        a, n, b = X.shape
        T = (E.T @ X.reshape(a, n * b)).reshape(-1, b)           # (b_y n) x a2
        E = T.T @ Y.reshape(-1, Y.shape[2])
        allreduce(E)
    return float(E[0, 0])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def allreduce(a):
            t = torch.from_numpy(a)
            dist.all_reduce(t)
            a[...] = t.numpy()

        dims, ranks = [5, 7, 3, 6, 4], [3, 6, 5, 4]
        x, y = _random_tt(1, dims, ranks), _random_tt(2, dims, ranks)
        lx, ly = xd.shard_cores(x, world, rank), xd.shard_cores(y, world, rank)
        # gather round trip
        parts = [None] * world
        dist.all_gather_object(parts, lx)
        back = xd.unshard_cores(parts)
        ok = all(np.array_equal(a, b) for a, b in zip(back, x))
        G, Gs = _left_grams(x), _sharded_left_grams(lx, allreduce)
        H, Hs = _right_grams(x), _sharded_right_grams(lx, allreduce)
        err = max(max(np.abs(G[k] - Gs[k]).max() / np.abs(G[k]).max() for k in range(1, len(dims))),
                  max(np.abs(H[k] - Hs[k]).max() / np.abs(H[k]).max() for k in range(1, len(dims))))
        full = np.einsum("aib,bjc,ckd,dle,emf->ijklm", *x)
        fully = np.einsum("aib,bjc,ckd,dle,emf->ijklm", *y)
        d_ref = float(np.sum(full * fully))
        d_sh = _sharded_dot(lx, ly, allreduce)
        out[rank] = (ok, err, abs(d_sh - d_ref) / (np.linalg.norm(full) * np.linalg.norm(fully)))
    finally:
        dist.destroy_process_group()


def test_mode_partition_covers():
    for n in (1, 2, 5, 20, 33):
        for world in (1, 2, 3, 8):
            spans = [xd.mode_partition(n, world, r) for r in range(world)]
            covered = [i for s, m in spans for i in range(s, s + m)]
            assert covered == list(range(n))
            assert max(m for _, m in spans) - min(m for _, m in spans) <= 1


def test_sharded_chains_world2_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for rank in range(2):
        ok, err, derr = out[rank]
        assert ok
        assert err <= 1e-13
        assert derr <= 1e-13
