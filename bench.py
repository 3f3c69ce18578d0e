"""Benchmark of the MI355X TT hot path: "GFLOP/s on TT contraction + TT-round sweep time, order-10 rank-256".

Headline step = one TT inner product <x, y> (core-chain contraction) + one x.round(256) on synthetic
random TTs of order 10, mode size 20, rank 256 (BASELINE.json north star). Inputs follow
TTTensor::random (ttNetwork.h:129-157): N(0,1) cores drawn by the product's own libstdc++ mt19937_64 +
normal_distribution (the reference's generator, xerus_amd.xerus.TTTensor.random_raw), then move_core(0)
on the GPU. They are resident in HBM before the timed region; round() keeps the tensor, the ranks and
the canonical form, so every step repeats the same work.

value = algorithmic GFLOP of the step / wall time (SURVEY 8(d) formulas, not hardware counters):
  <x,y>  : sum_k 2 a_x a_y n b_x + 2 a_y n b_x b_y           (zipper)
  round  : sum_edges 6 a n b^2 + 6 b^2 n' c + 22 b^3         (standard two-sweep TT rounding)
roofline: a second pass of the same K steps with a HIP event pair on every GEMM launch gives the average
GEMM launch duration (the events are recorded by the dispatch itself, hipExtLaunchKernelGGL; the pass
serialises the handle's fork lanes, so it is not the headline timing; its ms/step is reported as
roofline.events_pass_ms_per_step).
Multi-GPU: one process per GPU; the headline is replicas (every rank its own TT pair, weak scaling, no
data-path collective). The "cfg5" object adds BASELINE configs[4]: order-16 rank-512 round() sharded
over all ranks by mode slices (xerus_amd.dist; one r x r all-reduce per edge over RCCL), strong scaling.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-cfg5]
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
FP32_MFMA_PEAK_TFLOPS = 157.3  # gfx950 dense fp32 matrix peak (v_mfma_f32_*_f32, MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0           # HBM3E spec peak (MI355X_MICROARCH.md; 6.29 TB/s measured for a float4 copy)
SEED = 0xBAADF00D               # src/xerus/test/test.cpp:105


def tt_ranks(d, n, r):
    """reduce_to_maximal_ranks (ttNetwork.cpp:370-402) of a uniform rank r, with the boundary 1s."""
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


def random_cores(xe, dims, ranks, seed):
    """TTTensor::random_raw through the product's C++ API: the reference's RNG stream, cores (r, n, r')."""
    xe.seed(seed)
    tt = xe.TTTensor.random_raw(list(dims), list(ranks[1:-1]))
    return [np.ascontiguousarray(tt.get_component(k).to_ndarray()) for k in range(len(dims))]


def load_traffic():
    """HBM bytes per GEMM launch from the committed rocprofv3 PMC pass of this bench (or None)."""
    for tag in ("r06", "r05", "r04", "r03", "r02"):   # the newest committed pass
        p = os.path.join(ROOT, "profiles", tag, "pmc_traffic.json")
        if os.path.exists(p):
            break
    else:
        return None
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def bench_cfg5(h, xe, world, rank, dist, sync, steps, warmup):
    """BASELINE configs[4]: TTTensor order 16, n = 20, rank 512, round(512) sharded over all ranks."""
    from xerus_amd import dist as xd

    d, n, r = 16, 20, 512
    dims = [n] * d
    ranks = tt_ranks(d, n, r)
    cores = random_cores(xe, dims, ranks, SEED + 5)          # identical on every rank
    st = xd.ShardedTT.from_full_cores(h, cores, world, rank)
    del cores
    # several ranks over nccl: the library's RCCL communicator (all-reduces enqueued on the handle's stream,
    # no host round trip per collective); one rank: the null hook (no reduction points at all)
    comm, comm_kind = xd.TorchAllReduce(), "none" if world == 1 else "torch.distributed"
    if world > 1 and dist is not None and dist.get_backend() == "nccl":
        try:
            comm, comm_kind = xd.RcclComm(h), "rccl (xrs_comm_allreduce, stream-ordered)"
        except Exception as e:  # noqa: BLE001 -- keep the bench running on the torch.distributed hook
            print(f"[bench] RCCL communicator unavailable ({e}); using torch.distributed", file=sys.stderr)
    cert = st.round(r, comm)                                  # first call canonicalises (right-canonical)
    for _ in range(max(0, warmup - 1)):
        cert = st.round(r, comm) and cert
    calls0 = comm.calls
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        cert = st.round(r, comm) and cert
    h.synchronize()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    f = flops_round(dims, ranks)
    ms = elapsed / steps * 1e3
    # the truncating round(256) of the same TT (rank 512 -> 256; BASELINE.md §2 quotes the reference at 31.9 s /
    # 13.3 s for it): a fresh copy of the slices per call, host-timed, max over ranks
    trunc_ms, paths = [], set()
    for i in range(3):
        c = xd.ShardedTT(h, st.local.clone(), st.dims, world, rank)
        sync()
        t1 = time.perf_counter()
        paths.add(c.round_sharded(r // 2, comm) or "uncertified")
        h.synchronize()
        sync()
        t1 = time.perf_counter() - t1
        if dist is not None:
            import torch

            t = torch.tensor([t1], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t1 = float(t.item())
        if i:
            trunc_ms.append(t1 * 1e3)
        trunc_ranks = c.ranks
        c.local.free()
    out = {
        "workload": f"TT order-{d} n={n} rank-{r}: round({r}) sharded by mode slices over {world} rank(s)",
        "ms_per_round": round(ms, 3),
        "gflop_per_round": round(f / 1e9, 2),
        "tflops": round(f / (ms * 1e-3) / 1e12, 3),
        "scaling": "strong",
        "certified": bool(cert),
        "ranks_unchanged": st.ranks == ranks[1:-1],
        "allreduce_per_round": (comm.calls - calls0) / steps,
        "allreduce": comm_kind,
        "steps": steps,
        "round256_truncating": {
            "ms": round(float(np.mean(trunc_ms)), 3), "calls": len(trunc_ms), "path": sorted(paths),
            "ranks_out": trunc_ranks,
            "note": "x.round(256) from rank 512 (xrs_tt_round_sharded_ex on each rank's slices), host wall per call "
                    "after one untimed call, max over ranks",
        },
    }
    if hasattr(comm, "close"):
        comm.close()
    st.local.free()
    return out


def _timed(fn, reps, sync):
    """mean wall ms of fn() over reps calls (one warm-up call first), synchronised on both sides."""
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps * 1e3


def _events(h, mask, fn, reps, warm=1):
    """HIP-event timing of every kernel of family `mask` launched by fn() (reps calls after `warm` untimed ones):
    per-launch mean."""
    from xerus_amd import capi  # noqa: F401

    for _ in range(warm):
        fn()
    h.synchronize()
    h.prof_begin(mask)
    for _ in range(reps):
        fn()
    p = h.prof_end()
    n = max(1, p["launches"])
    return {"launches": p["launches"] / reps, "us_per_launch": p["ms"] / n * 1e3, "flops_per_launch": p["flops"] / n,
            "bytes_per_launch": p["bytes"] / n}


def bench_cfg2(h):
    """BASELINE configs[1]: one dense 1024^3 contraction -> one fp64 MFMA GEMM (inputs resident in HBM)."""
    from xerus_amd import capi

    n = 1024
    rng = np.random.default_rng(1)
    A, B = h.array(rng.standard_normal((n, n))), h.array(rng.standard_normal((n, n)))
    C = h.empty((n, n))
    ev = _events(h, capi.KFAM_GEMM, lambda: h.gemm(C, n, n, 1.0, A, n, False, n, B, n, False), 20, warm=150)
    tf = 2.0 * n ** 3 / (ev["us_per_launch"] * 1e-6) / 1e12
    return {"workload": "A(i,j) = B(i,k) * C(k,j), 1024^3, fp64 MFMA GEMM", "us": round(ev["us_per_launch"], 2),
            "tflops": round(tf, 2), "frac_fp64_peak": round(tf / FP64_MFMA_PEAK_TFLOPS, 3),
            "timing": "dispatch begin/end events (hipExtLaunchKernelGGL), mean of 20 after 150 untimed"}


def bench_cfg2_f32(h):
    """BASELINE configs[1] on the fp32 matrix cores (xrs_gemm_f32, "MFMA fp32"): 1024^3, fp32 operands resident in
    HBM; its error against the fp64 product of the same fp32 inputs."""
    from xerus_amd import capi

    n = 1024
    rng = np.random.default_rng(1)
    A32, B32 = rng.standard_normal((n, n)).astype(np.float32), rng.standard_normal((n, n)).astype(np.float32)
    A, B, C = h.array_f32(A32), h.array_f32(B32), capi.Float32Array(h, (n, n))
    # (300 untimed launches, ~7 ms: the GPU's clocks reach their steady state -- after 20 the mean was 23.8 us,
    # after 200-1000 21.4-22.7 us, tools/cfg2f32_warm.py, profiles/r05/cfg2f32_warm_r05w2.txt)
    ev = _events(h, capi.KFAM_GEMM, lambda: h.gemm_f32(C, n, n, 1.0, A, n, False, n, B, n, False), 50, warm=300)
    expect = A32.astype(np.float64) @ B32.astype(np.float64)
    err = float(np.linalg.norm(C.numpy() - expect) / np.linalg.norm(expect))
    for d in (A, B, C):
        d.free()
    tf = 2.0 * n ** 3 / (ev["us_per_launch"] * 1e-6) / 1e12
    return {"workload": "A(i,j) = B(i,k) * C(k,j), 1024^3, fp32 MFMA GEMM (xrs_gemm_f32)", "us": round(ev["us_per_launch"], 2),
            "tflops": round(tf, 2), "frac_fp32_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 3), "peak_tflops": FP32_MFMA_PEAK_TFLOPS,
            "rel_frob_err_vs_fp64": err, "timing": "dispatch begin/end events (hipExtLaunchKernelGGL), mean of 50 after 300 untimed"}


def bench_cfg1(xe):
    """BASELINE configs[0] through the C++ host API: A(i,j) = B(i,k,l) * C(k,j,l), 64^3 (permute + GEMM)."""
    rng = np.random.default_rng(2)
    B = xe.Tensor.from_ndarray(rng.standard_normal((64, 64, 64)))
    Cc = xe.Tensor.from_ndarray(rng.standard_normal((64, 64, 64)))
    i, j, k, l = xe.indices(4)
    A = xe.Tensor()

    def run():
        A(i, j) << B(i, k, l) * Cc(k, j, l)

    ms = _timed(run, 50, xe.synchronize)
    return {"workload": "A(i,j) = B(i,k,l) * C(k,j,l), 64^3, indexed expression (host planning + permute + GEMM)",
            "us_per_eval": round(ms * 1e3, 1), "gflops": round(2 * 64 ** 4 / (ms * 1e-3) / 1e9, 1)}


def bench_permute(h):
    """Permutation kernels at the shapes on the reference's paths, HBM roofline."""
    from xerus_amd import capi

    shapes = [("cfg1 C 64^3 {0,2,1}", (64, 64, 64), (0, 2, 1)),
              ("cfg4 zipper (1,1,256,20,256) {0,1,3,4,2}", (1, 1, 256, 20, 256), (0, 1, 3, 4, 2)),
              ("1024^2 transpose", (1024, 1024), (1, 0)),
              ("20^6 reversal", (20,) * 6, (5, 4, 3, 2, 1, 0)),
              ("4096^2 transpose", (4096, 4096), (1, 0))]
    out = []
    for name, dims, shuf in shapes:
        size = int(np.prod(dims))
        # rotate over enough source / destination pairs that one pass touches >= 1 GiB (the 256 MB
        # last-level cache cannot serve a launch from the previous pass), at most 64 pairs
        nbuf = int(min(64, max(1, -(-(1 << 30) // (16 * size)))))
        base = np.arange(size, dtype=np.float64).reshape(dims)
        srcs = [h.array(base) for _ in range(nbuf)]
        dsts = [h.empty((size,)) for _ in range(nbuf)]
        reps = max(20, nbuf)
        it = iter(range(10 ** 9))

        def one():
            i = next(it) % nbuf
            h.permute(dsts[i], srcs[i], dims, shuf)

        ev = _events(h, capi.KFAM_PERMUTE, one, reps)
        gbs = 16.0 * size / (ev["us_per_launch"] * 1e-6) / 1e9
        out.append({"shape": name, "mbytes": round(16.0 * size / 1e6, 2), "us": round(ev["us_per_launch"], 2),
                    "gbs": round(gbs, 1), "frac_hbm_peak": round(gbs / HBM_PEAK_GBS, 3), "buffers_rotated": nbuf,
                    "timing": "dispatch begin/end events (hipExtLaunchKernelGGL), mean over the rotated launches"})
        for b in srcs + dsts:
            b.free()
    return out


def bench_cfg3(h, xe):
    """BASELINE configs[2]: TTTensor order 10, n 20, rank 128 -- round(128) (certified, non-truncating),
    round(64) (truncating) and (x + y).round(128) (rank 256 -> 128, rank-revealing left sweep)."""
    from xerus_amd import capi

    d, n, r = 10, 20, 128
    dims = [n] * d
    ranks = tt_ranks(d, n, r)
    xc = random_cores(xe, dims, ranks, SEED + 11)
    yc = random_cores(xe, dims, ranks, SEED + 12)
    x = capi.TTDevice.from_cores(h, xc)
    x.move_core(0)
    y = capi.TTDevice.from_cores(h, yc)
    y.move_core(0)
    out = {"workload": f"TT order-{d} n={n} rank-{r}"}

    def round_case(src, target, reps, eps=8 * np.finfo(float).eps):
        ts = []
        for _ in range(reps + 1):
            c = src.clone()
            h.synchronize()
            t0 = time.perf_counter()
            c.round(target, eps)
            h.synchronize()
            ts.append(time.perf_counter() - t0)
            res_ranks = c.r
            out.setdefault("_paths", set()).add(h.last_round_path())
            c.free()
        return float(np.mean(ts[1:])) * 1e3, res_ranks

    ms, rr = round_case(x, 128, 10)
    out.pop("_paths", None)
    f = flops_round(dims, ranks)
    out["round128"] = {"ms": round(ms, 3), "gflops": round(f / (ms * 1e-3) / 1e9, 1), "ranks_out": rr[1:-1]}
    ms, rr = round_case(x, 64, 10)
    out.pop("_paths", None)
    out["round64"] = {"ms": round(ms, 3), "gflops": round(f / (ms * 1e-3) / 1e9, 1), "ranks_out": rr[1:-1],
                      "flops_note": "standard two-sweep flops of the input ranks"}
    # x + y: block-diagonal cores (TTNetwork::operator+=, ttNetwork.cpp:797-847), not canonical
    xs, ys = x.cores(), y.cores()
    sc = []
    for k in range(d):
        X, Y = xs[k], ys[k]
        if k == 0:
            sc.append(np.concatenate([X, Y], axis=2))
        elif k == d - 1:
            sc.append(np.concatenate([X, Y], axis=0))
        else:
            Z = np.zeros((X.shape[0] + Y.shape[0], n, X.shape[2] + Y.shape[2]))
            Z[:X.shape[0], :, :X.shape[2]] = X
            Z[X.shape[0]:, :, X.shape[2]:] = Y
            sc.append(Z)
    s = capi.TTDevice.from_cores(h, sc)
    sr = [1] + [c.shape[2] for c in sc]
    ms, rr = round_case(s, 128, 5)
    out.pop("_paths", None)
    f = flops_round(dims, sr)
    out["sum_round128"] = {"ms": round(ms, 3), "gflops": round(f / (ms * 1e-3) / 1e9, 1), "ranks_in": sr[1:-1],
                           "ranks_out": rr[1:-1]}
    # decaying spectra the certified paths refuse (tests/test_round_general_gpu.py): raw N(0,1) cores whose
    # right rank index is scaled by 0.8^j; round(64) (maxRank cut) and round(1e-8) (eps cut only)
    gc = random_cores(xe, dims, ranks, SEED + 13)
    for k in range(d - 1):
        gc[k] = gc[k] * (0.8 ** np.arange(gc[k].shape[2]))[None, None, :]
    g = capi.TTDevice.from_cores(h, gc)
    f = flops_round(dims, ranks)
    for key, target, eps in (("round64_graded", 64, 8 * np.finfo(float).eps), ("round_eps_graded", [2 ** 62] * (d - 1), 1e-8)):
        out.pop("_paths", None)
        ms, rr = round_case(g, target, 5, eps)
        out[key] = {"ms": round(ms, 3), "gflops": round(f / (ms * 1e-3) / 1e9, 1), "ranks_out": rr[1:-1],
                    "eps": eps, "path": sorted(out.pop("_paths"))}
    out.pop("_paths", None)
    for t in (x, y, s, g):
        t.free()
    return out


def bench_cfg4(h, xe):
    """BASELINE configs[3]: <x,x> of a TTTensor order 12, n 20, rank 256 (zipper), fp64 MFMA roofline."""
    from xerus_amd import capi

    d, n, r = 12, 20, 256
    dims = [n] * d
    ranks = tt_ranks(d, n, r)
    x = capi.TTDevice.from_cores(h, random_cores(xe, dims, ranks, SEED + 13))
    f = flops_dot(dims, ranks, ranks)
    ms = _timed(lambda: x.dot(x), 20, h.synchronize)
    tf = f / (ms * 1e-3) / 1e12
    x.free()
    return {"workload": f"<x,x> TT order-{d} n={n} rank-{r}", "ms": round(ms, 4), "gflop": round(f / 1e9, 3),
            "tflops": round(tf, 2), "frac_fp64_peak": round(tf / FP64_MFMA_PEAK_TFLOPS, 3)}


def bench_svd(h):
    """The dense SVD (xrs_svd, blasWrapper::svd / dgesdd semantics) at the TT edge sizes."""
    rng = np.random.default_rng(3)
    out = {}
    for m in (128, 256, 512):
        A = h.array(rng.standard_normal((m, m)))
        ms = _timed(lambda: h.svd(A), 3, h.synchronize)
        out[str(m)] = {"ms": round(ms, 3)}
        A.free()
    # TT-SVD-shaped unfoldings (min(m, n) <= 128: the bidiagonal route on the QR factor)
    for m, n in ((128, 2560), (64, 1280)):
        A = h.array(rng.standard_normal((m, n)))
        ms = _timed(lambda: h.svd(A), 3, h.synchronize)
        out[f"{m}x{n}"] = {"ms": round(ms, 3)}
        A.free()
    out["route"] = "min(m, n) <= 128: bidiagonalisation + Golub-Kahan eigenpairs, certified (Jacobi fallback); above: block Jacobi"
    return out


def host_cpu_info():
    """nproc, the CPUs this process may run on, the CPU model, and the thread count of the all-cores leg
    (the job's CPU share: OMP_NUM_THREADS when the launcher sets it -- 16 per GPU on the GPU box, where
    nproc shows the whole machine -- else the affinity mask)."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        threads, rule = min(int(env), affinity), "min(OMP_NUM_THREADS, affinity)"
    else:
        threads, rule = affinity, "affinity mask"
    return {"nproc": nproc, "affinity": affinity, "model": model, "threads": max(1, threads), "rule": rule}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, worker=None, timeout=None):
    """`bench.py --gpus N` without a launcher around it: start N rank processes, one per GPU, and relay rank 0's
    JSON line. Runs BEFORE anything touches the GPU -- this process imports neither torch nor xerus_amd and
    never execs: the ranks are ordinary child processes (python bench.py ... with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment, the torch.distributed.run
    contract), so each binds its own device and joins the nccl (RCCL) process group itself. Returns the
    exit status: 0 only if every rank exited 0. `worker` replaces this script (tests: a stub rank)."""
    import subprocess
    import tempfile

    worker = worker or os.path.abspath(__file__)
    port = _free_port()
    procs = []
    with tempfile.TemporaryFile(mode="w+") as out0:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL across processes on this image)
            procs.append(subprocess.Popen([sys.executable, worker] + list(argv), env=env,
                                          stdout=out0 if r == 0 else subprocess.DEVNULL))
        # wait for all; a failed rank ends the job (the others would wait for it in a collective forever)
        t0 = time.time()
        bad = []
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad or all(c == 0 for c in codes):
                break
            if timeout is not None and time.time() - t0 > timeout:
                bad = [(r, "timeout") for r, c in enumerate(codes) if c is None]
                break
            time.sleep(0.05)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        if bad:
            print(f"[bench] rank(s) failed: {bad}", file=sys.stderr)
        out0.seek(0)
        lines = [ln for ln in out0.read().splitlines() if ln.strip()]
    if lines:
        print(lines[-1], flush=True)
    return 0 if not bad and lines else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; N > 1 without WORLD_SIZE in the environment starts N rank processes")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--order", type=int, default=10)
    ap.add_argument("--mode", type=int, default=20)
    ap.add_argument("--rank", type=int, default=256)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-overlap", action="store_true",
                    help="sequential step (<x,y> waited for before the round starts) instead of the async inner product")
    ap.add_argument("--cpu-steps", type=int, default=8)
    ap.add_argument("--no-cfg5", action="store_true", help="skip the sharded order-16 rank-512 round")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the per-config lines (cfg1-cfg4, permutation roofline, SVD); they run at N=1 only")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us (python bench.py --gpus N): become it, before any GPU or torch import
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: measuring {world} rank(s)", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import xerus_amd.xerus as xe
    from xerus_amd import capi

    xe.set_device(local)
    h = capi.Handle(local)
    d, n, r = args.order, args.mode, args.rank
    dims = [n] * d
    ranks = tt_ranks(d, n, r)
    xc = random_cores(xe, dims, ranks, SEED + 2 * rank)
    yc = random_cores(xe, dims, ranks, SEED + 2 * rank + 1)
    x = capi.TTDevice.from_cores(h, xc)
    y = capi.TTDevice.from_cores(h, yc)
    x.move_core(0)
    y.move_core(0)
    assert x.r == ranks and y.r == ranks, (x.r, ranks)

    f_dot = flops_dot(dims, ranks, ranks)
    f_round = flops_round(dims, ranks)
    f_step = f_dot + f_round

    def step_seq(timing=None):
        t0 = time.perf_counter()
        x.dot(y)
        t1 = time.perf_counter()
        x.round(r)
        h.synchronize()
        t2 = time.perf_counter()
        if timing is not None:
            timing["dot"] += t1 - t0
            timing["round"] += t2 - t1

    def step_overlap(timing=None):
        # <x,y> on the handle's side streams (xrs_tt_dot_async) beside x.round(r) on the main stream; the
        # round's release of x's old cores waits for the inner product (stream-ordered fence)
        fut = x.dot_async(y)
        x.round(r)
        fut.result()
        h.synchronize()

    step = step_seq if args.no_overlap else step_overlap

    for _ in range(args.warmup):
        step()

    def barrier():
        h.synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    # phase split (diagnostic, not the headline): the same steps run sequentially, host-timed per call
    timing = {"dot": 0.0, "round": 0.0}
    for _ in range(args.steps):
        step_seq(timing)
    barrier()
    # side key (not the headline, which stays f64 like the reference's value_t): the same <x,y> on fp32 MFMA
    # tiles (xrs_tt_dot_f32), host-timed per call like dot_ms, and its error against the f64 product
    d64 = x.dot(y)
    d32 = x.dot_f32(y)
    for _ in range(2):
        x.dot_f32(y)
    barrier()
    t32 = time.perf_counter()
    for _ in range(args.steps):
        x.dot_f32(y)
    t32 = (time.perf_counter() - t32) / args.steps
    # accuracy: the step's independent x, y (|<x,y>| ~ 2e-7 ||x|| ||y||: error relative to the norms and to the value)
    # and the correlated pair <x,x> (relative to the value)
    nxy = x.frob_norm() * y.frob_norm()
    xx64, xx32 = x.dot(x), x.dot_f32(x)
    dot_f32 = {"ms": round(t32 * 1e3, 4), "tflops": round(f_dot / t32 / 1e12, 3),
               "frac_fp32_peak": round(f_dot / t32 / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
               "rel_err": abs(d32 - d64) / nxy, "rel_err_norms": abs(d32 - d64) / nxy,
               "rel_err_value": abs(d32 - d64) / abs(d64), "value_over_norms": abs(d64) / nxy,
               "xx_rel_err_value": abs(xx32 - xx64) / abs(xx64),
               "timing": "host wall per call (synchronous: includes the read-back and host exponent sum)",
               "path": "xrs_tt_dot_f32: two-ended zipper of xrs_gemm_f32-family launches (v_mfma_f32_16x16x4_f32), fp64 cores "
                       "rounded at load, power-of-two normalised T and environments"}

    # Roofline passes: the same K steps again with a HIP event pair on every GEMM launch (the start / stop
    # events of hipExtLaunchKernelGGL on the stream each launch goes to: the dispatch's own begin / end
    # timestamps). The fork lanes are serialised while timing, so these passes are kept out of the headline
    # timing; their wall times are reported beside it. The kernel's roofline comes
    # from the sequential step (<x,y> waited for before the round starts), where a launch does not share
    # the chip with the other operation's kernels; the overlapped step's per-launch figure is reported
    # beside it (its launch durations include that sharing).
    def events_pass(fn, mask=capi.KFAM_GEMM):
        barrier()
        h.prof_begin(mask)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        barrier()
        el = time.perf_counter() - t0
        return h.prof_end(), el

    prof, elapsed_ev = events_pass(step_seq)
    prof_ov, elapsed_ev_ov = events_pass(step) if step is not step_seq else (prof, elapsed_ev)
    # the separate split-K reduce launches that complete some of those GEMMs (k_splitk_reduce*), same steps
    prof_red, _ = events_pass(step_seq, capi.KFAM_SPLITK)

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = elapsed / args.steps * 1e3
    value = world * f_step * args.steps / elapsed / 1e9
    assert x.r == ranks

    cfg5 = None
    if not args.no_cfg5:
        x.free()
        y.free()
        try:
            cfg5 = bench_cfg5(h, xe, world, rank, dist, barrier, steps=3, warmup=1)
        except Exception as e:   # reported, never fatal for the headline line
            cfg5 = {"error": f"{type(e).__name__}: {e}"}

    extras = {}
    if world == 1 and not args.no_extras:
        for key, fn in [("cfg1", lambda: bench_cfg1(xe)), ("cfg2", lambda: bench_cfg2(h)), ("cfg2_f32", lambda: bench_cfg2_f32(h)),
                        ("cfg3", lambda: bench_cfg3(h, xe)),
                        ("cfg4", lambda: bench_cfg4(h, xe)), ("permute", lambda: bench_permute(h)), ("svd", lambda: bench_svd(h))]:
            try:
                extras[key] = fn()
            except Exception as e:   # reported, never fatal for the headline line
                extras[key] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        launches = max(1, prof["launches"])
        gemm_tflops = prof["flops"] / (prof["ms"] * 1e-3) / 1e12 if prof["ms"] > 0 else 0.0
        traffic = load_traffic()
        roofline = {
            "bound": "mfma",
            "kernel": "GEMM family: k_gemm_glds (LDS-DMA pipeline) + k_gemm_f64 (general tiles), every GEMM launch of the step, fp64 MFMA 16x16x4",
            "achieved": round(gemm_tflops, 3),
            "peak": FP64_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(gemm_tflops / FP64_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
            "traffic_source": traffic.get("source") if traffic else None,
            "launches_per_step": prof["launches"] / args.steps,
            "avg_launch_us": round(prof["ms"] / launches * 1e3, 3),
            "events_pass": ("sequential step (x.dot(y), then x.round) with the handle's fork lanes serialised onto its main "
                            "stream while kernels are timed (xrs_prof_begin); each GEMM launch records its HIP event pair itself "
                            "(hipExtLaunchKernelGGL start/stop events = the dispatch's begin/end timestamps, the interval a "
                            "rocprofv3 kernel trace reports; marker events around a launch add its ~6 us dispatch latency), "
                            "so the per-launch durations agree with a kernel trace of the same pass (tools/roofline_from_trace.py)"),
            "events_pass_ms_per_step": round(elapsed_ev / args.steps * 1e3, 4),
            "incl_splitk_reduce": {
                "achieved": round(prof["flops"] / ((prof["ms"] + prof_red["ms"]) * 1e-3) / 1e12, 3) if prof["ms"] > 0 else 0.0,
                "frac": round(prof["flops"] / ((prof["ms"] + prof_red["ms"]) * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4)
                if prof["ms"] > 0 else 0.0,
                "reduce_launches_per_step": prof_red["launches"] / args.steps,
                "reduce_us_per_launch": round(prof_red["ms"] / max(1, prof_red["launches"]) * 1e3, 3),
                "traffic": traffic.get("hbm_bytes_per_launch_incl_splitk_reduce") if traffic else None,
                "note": "the GEMM family's flops over the GEMM launches' AND the separate split-K reduce launches' summed "
                        "durations (same sequential steps, reduce launches timed in a pass of their own); traffic: the GEMM "
                        "launches' HBM bytes plus the reduce launches' spread over them (same PMC passes)",
            },
            "algorithmic_flops_per_launch": prof["flops"] / launches,
            "algorithmic_bytes_per_launch": prof["bytes"] / launches,
            "chip_level": {
                "achieved": round(f_step / (ms_step * 1e-3) / 1e12, 3),
                "frac": round(f_step / (ms_step * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                "note": "the whole headline step's algorithmic flops / its wall time (launches overlap across streams)",
            },
            "overlapped_step": {
                "achieved": round(prof_ov["flops"] / (prof_ov["ms"] * 1e-3) / 1e12, 3) if prof_ov["ms"] > 0 else 0.0,
                "frac": round(prof_ov["flops"] / (prof_ov["ms"] * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4) if prof_ov["ms"] > 0 else 0.0,
                "avg_launch_us": round(prof_ov["ms"] / max(1, prof_ov["launches"]) * 1e3, 3),
                "events_pass_ms_per_step": round(elapsed_ev_ov / args.steps * 1e3, 4),
                "note": "per-launch durations of the headline (overlapped) step: concurrent <x,y> and round kernels share the chip",
            },
        }
        cpu = None
        if not args.no_cpu and world == 1:   # the CPU baseline is an N = 1 figure (rank 0 of a single-GPU run)
            # CPU baseline leg: the oracle (numpy/scipy-LAPACK restatement of the reference algorithm)
            from oracle import xerus_ref as ref

            try:
                from threadpoolctl import threadpool_limits
            except ImportError:
                threadpool_limits = None
            def cpu_leg(threads, steps):
                xo, yo = ref.TT([c.copy() for c in xc]), ref.TT([c.copy() for c in yc])
                xo.move_core(0)
                yo.move_core(0)
                ctx = threadpool_limits(limits=threads) if threadpool_limits else None
                if ctx:
                    ctx.__enter__()
                try:
                    t0 = time.perf_counter()
                    for _ in range(steps):
                        ref.dot(xo, yo)
                        xo.round(r)
                    return time.perf_counter() - t0
                finally:
                    if ctx:
                        ctx.__exit__(None, None, None)

            host = host_cpu_info()
            t_1 = cpu_leg(1, args.cpu_steps)
            t_all = cpu_leg(host["threads"], args.cpu_steps)
            sample = (f"{args.cpu_steps} full steps (<x,y> + round({r})) of the same order-{d} n={n} r={r} workload and "
                      f"inputs, numpy/scipy-LAPACK restatement of the reference (dgeqp3/dorgqr/dgesdd/dgemm call sequence)")
            cpu = {
                "value": round(f_step * args.cpu_steps / t_all / 1e9, 3),
                "unit": "GFLOP/s",
                "cores": host["threads"],
                "kind": "port",
                "sample": f"{sample}, {host['threads']} BLAS threads (all cores this job may use), {t_all:.2f} s",
                "ms_per_step": round(t_all / args.cpu_steps * 1e3, 2),
                "single_core": {
                    "value": round(f_step * args.cpu_steps / t_1 / 1e9, 3),
                    "cores": 1,
                    "ms_per_step": round(t_1 / args.cpu_steps * 1e3, 2),
                    "sample": f"{sample}, 1 BLAS thread, {t_1:.2f} s",
                },
                "nproc": host["nproc"],
                "affinity_cpus": host["affinity"],
                "cpu_model": host["model"],
                "threads_rule": host["rule"],
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
            "data": "synthetic (TTTensor::random semantics: N(0,1) cores from the product's libstdc++ mt19937_64 "
                    "seeded 0xBAADF00D + 2 rank (+1 for y), move_core(0) on the GPU)",
            "config": {
                "workload": f"TT order-{d} n={n} rank-{r}: <x,y> + x.round({r}) per step",
                "order": d, "mode_size": n, "rank": r, "ranks": ranks,
                "step": ("sequential: x.dot(y), then x.round" if args.no_overlap else
                         "overlapped: x.dot_async(y) on side streams beside x.round on the main stream, both waited for"),
                "dot_ms": round(timing["dot"] / args.steps * 1e3, 4),
                "dot_f32": dot_f32,
                "round_sweep_ms": round(timing["round"] / args.steps * 1e3, 4),
                "sequential_ms_per_step": round((timing["dot"] + timing["round"]) / args.steps * 1e3, 4),
                "gflop_per_step": round(f_step / 1e9, 4),
                "parallelism": f"replicas x{world}",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cfg5": cfg5,
        }
        out.update(extras)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
