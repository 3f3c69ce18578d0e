"""Recompute bench.py's roofline.frac from a rocprofv3 kernel trace of the step-only SEQUENTIAL bench
(tools/gpu_run.sh step `trace`: bench.py --no-cpu --no-cfg5 --no-extras --no-overlap).

The bench runs W warm-up steps, K timed steps, K phase-split steps, the fp32 / fp64 side dots, K steps of the
GEMM HIP-event pass and (r06) K steps of the split-K-reduce event pass, all the same sequential step (<x,y>
waited for, then round). The GEMM family (k_gemm_glds + k_gemm_f64 dispatches; the split-K reduce is not a GEMM
launch, as in bench.py's event mask) of the second-to-last K steps is the GEMM event pass's launch set; the last
K steps' GEMMs (the reduce pass: same launches, untimed by events) are printed as a cross-check. frac = algorithmic flops per launch (bench.py's roofline.algorithmic_flops_per_launch, the
2*M*N*K sum of those launches) / mean trace duration / 78.6 TF/s. Also printed: the chip-level figure (step
algorithmic flops / wall ms_per_step), which counts the whole step, not the GEMMs alone.

Usage: python tools/roofline_from_trace.py TRACE_DIR BENCH_JSON_FILE
"""
import csv
import glob
import json
import os
import sys

PEAK = 78.6e12


def main():
    tdir, bfile = sys.argv[1], sys.argv[2]
    line = [ln for ln in open(bfile) if ln.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    K = b["steps"]
    L = int(round(rf["launches_per_step"]))
    F = rf["algorithmic_flops_per_launch"]
    traces = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for t in traces:
        for r in csv.DictReader(open(t)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    gemm = [(s, e) for s, e, n in rows if ("k_gemm_glds" in n or "k_gemm_f64" in n)]
    need = K * L
    if len(gemm) < 2 * need:
        print(f"only {len(gemm)} GEMM dispatches in the trace, expected >= {2 * need}")
        sys.exit(1)
    windows = {"GEMM events pass (second-to-last K steps)": gemm[-2 * need:-need],
               "split-K reduce events pass (last K steps, its GEMM launches)": gemm[-need:]}
    reds = [(s, e) for s, e, n in rows if "k_splitk_reduce" in n][-int(round(K * rf.get("incl_splitk_reduce", {}).get(
        "reduce_launches_per_step", 0))):] if rf.get("incl_splitk_reduce") else []
    print(f"bench line: steps K={K}, GEMM launches per step L={L}, flops per launch F={F / 1e6:.2f} MFLOP, "
          f"ms_per_step={b['ms_per_step']}, roofline.frac={rf['frac']} (avg_launch_us {rf['avg_launch_us']})")
    for name, w in windows.items():
        durs = [(e - s) * 1e-9 for s, e in w]
        mean = sum(durs) / len(durs)
        print(f"{name}: {len(w)} GEMM dispatches, mean {mean * 1e6:.3f} us -> {F / mean / 1e12:.2f} TF/s, "
              f"frac {F / mean / PEAK:.4f}; GEMM busy per step {sum(durs) / K * 1e3:.4f} ms")
    if reds:
        rd = [(e - s) * 1e-9 for s, e in reds]
        print(f"split-K reduce launches of the last K steps: {len(rd)}, mean {sum(rd) / len(rd) * 1e6:.3f} us "
              f"(bench line: {rf['incl_splitk_reduce']['reduce_us_per_launch']} us)")
    gf = b["config"]["gflop_per_step"] * 1e9
    ms = b["ms_per_step"]
    print(f"chip level: {gf / 1e9:.2f} GFLOP per step / {ms} ms = {gf / (ms * 1e-3) / 1e12:.2f} TF/s = "
          f"{gf / (ms * 1e-3) / PEAK:.4f} of the fp64 peak")


if __name__ == "__main__":
    main()
