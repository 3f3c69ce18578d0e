"""Benchmark of the MI355X TT hot path: "GFLOP/s on TT contraction + TT-round sweep time, order-10 rank-256".

One step = one TT inner product <x, y> (core-chain contraction) + one x.round(256) sweep on synthetic
random TTs of order 10, mode size 20, rank 256 (BASELINE.json north star; TTTensor::random semantics:
N(0,1) cores, then move_core(0)). Inputs are resident in HBM before the timed region; the round result
is canonical at core 0 with the same ranks, so every step repeats exactly the same work.

value = algorithmic GFLOP of the step / wall time (SURVEY §8(d) formulas, not hardware counters):
  <x,y>  : sum_k 2 a_x a_y n b_x + 2 a_y n b_x b_y           (zipper)
  round  : sum_edges 6 a n b^2 + 6 b^2 n' c + 22 b^3         (standard two-sweep TT rounding)
Multi-GPU: one process per GPU, every rank rounds/contracts its own TT pair (replicas, weak scaling,
no data-path collective); value = all ranks' flops / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # gfx950 dense fp64 matrix peak (MI355X spec)
HBM_PEAK_GBS = 8000.0


def tt_ranks(d, n, r):
    ranks = [r] * (d - 1)
    cur = 1
    for i in range(d - 1):
        cur *= n
        if cur < ranks[i]:
            ranks[i] = cur
        else:
            cur = ranks[i]
    cur = 1
    for i in range(1, d):
        cur *= n
        if cur < ranks[d - i - 1]:
            ranks[d - i - 1] = cur
        else:
            cur = ranks[d - i - 1]
    return [1] + ranks + [1]


def flops_dot(dims, rx, ry):
    return sum(2.0 * rx[k] * ry[k] * dims[k] * rx[k + 1] + 2.0 * ry[k] * dims[k] * rx[k + 1] * ry[k + 1]
               for k in range(len(dims)))


def flops_round(dims, r):
    f = 0.0
    for k in range(len(dims) - 1):   # edge between core k (a, n, b) and core k+1 (b, n', c)
        a, n, b, n2, c = r[k], dims[k], r[k + 1], dims[k + 1], r[k + 2]
        f += 6.0 * a * n * b * b + 6.0 * b * b * n2 * c + 22.0 * b ** 3
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--order", type=int, default=10)
    ap.add_argument("--mode", type=int, default=20)
    ap.add_argument("--rank", type=int, default=256)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-steps", type=int, default=2)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from oracle import xerus_ref as ref   # input generator (libstdc++ RNG restatement) + CPU baseline leg
    from xerus_amd import capi

    h = capi.Handle(local)
    d, n, r = args.order, args.mode, args.rank
    dims = [n] * d
    ranks = tt_ranks(d, n, r)
    rng = ref.Rng(ref.Rng.SEED + rank)
    # synthetic TTTensor::random inputs: raw N(0,1) cores uploaded, then move_core(0) ON THE GPU
    xr = ref.TT.random_raw(dims, ranks[1:-1], rng)
    yr = ref.TT.random_raw(dims, ranks[1:-1], rng)
    x = capi.TTDevice.from_cores(h, xr.cores)
    y = capi.TTDevice.from_cores(h, yr.cores)
    x.move_core(0)
    y.move_core(0)
    assert x.r == ranks and y.r == ranks, (x.r, ranks)

    f_dot = flops_dot(dims, ranks, ranks)
    f_round = flops_round(dims, ranks)
    f_step = f_dot + f_round

    def step(timing=None):
        t0 = time.perf_counter()
        x.dot(y)
        t1 = time.perf_counter()
        x.round(r)
        h.synchronize()
        t2 = time.perf_counter()
        if timing is not None:
            timing["dot"] += t1 - t0
            timing["round"] += t2 - t1

    for _ in range(args.warmup):
        step()

    def barrier():
        h.synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    h.prof_begin(capi.KFAM_GEMM)
    timing = {"dot": 0.0, "round": 0.0}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timing)
    barrier()
    elapsed = time.perf_counter() - t0
    prof = h.prof_end()

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = elapsed / args.steps * 1e3
    value = world * f_step * args.steps / elapsed / 1e9

    if rank == 0:
        gemm_tflops = prof["flops"] / (prof["ms"] * 1e-3) / 1e12 if prof["ms"] > 0 else 0.0
        roofline = {
            "bound": "mfma",
            "kernel": "k_gemm_f64 (all GEMM launches of the step, fp64 MFMA 16x16x4)",
            "achieved": round(gemm_tflops, 3),
            "peak": FP64_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(gemm_tflops / FP64_MFMA_PEAK_TFLOPS, 4),
            "traffic": None,
            "launches_per_step": prof["launches"] / args.steps,
            "avg_launch_us": prof["ms"] / max(1, prof["launches"]) * 1e3,
            "algorithmic_flops_per_launch": prof["flops"] / max(1, prof["launches"]),
        }
        cpu = None
        if not args.no_cpu:
            try:
                from threadpoolctl import threadpool_limits
            except ImportError:
                threadpool_limits = None
            xc, yc = xr.copy(), yr.copy()
            xc.move_core(0)
            yc.move_core(0)
            ctx = threadpool_limits(limits=1) if threadpool_limits else None
            if ctx:
                ctx.__enter__()
            t_c = time.perf_counter()
            for _ in range(args.cpu_steps):
                ref.dot(xc, yc)
                xc.round(r)
            t_c = time.perf_counter() - t_c
            if ctx:
                ctx.__exit__(None, None, None)
            cpu = {
                "value": round(f_step * args.cpu_steps / t_c / 1e9, 3),
                "unit": "GFLOP/s",
                "cores": 1,
                "kind": "port",
                "sample": f"{args.cpu_steps} full steps (<x,y> + round({r})) of the same order-{d} n={n} r={r} "
                          f"workload, numpy/scipy-LAPACK restatement of the reference (dgeqp3/dorgqr/dgesdd/dgemm), "
                          f"1 BLAS thread, {t_c:.2f} s",
                "ms_per_step": round(t_c / args.cpu_steps * 1e3, 2),
            }
        out = {
            "metric": "GFLOP/s on TT contraction + TT-round sweep time, order-10 rank-256",
            "value": round(value, 3),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (TTTensor::random semantics: N(0,1) cores via mt19937_64 seeded 0xBAADF00D + rank, "
                    "move_core(0) on the GPU)",
            "config": {
                "workload": f"TT order-{d} n={n} rank-{r}: <x,y> + x.round({r}) per step",
                "order": d, "mode_size": n, "rank": r, "ranks": ranks,
                "dot_ms": round(timing["dot"] / args.steps * 1e3, 4),
                "round_sweep_ms": round(timing["round"] / args.steps * 1e3, 4),
                "gflop_per_step": round(f_step / 1e9, 4),
                "parallelism": f"replicas x{world}",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
