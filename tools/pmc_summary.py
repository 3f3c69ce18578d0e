"""Summarise the PMC passes of tools/pmc_bench.sh per kernel family and write profiles/<tag>/pmc_*.

HBM traffic per GEMM launch (k_gemm_glds and k_gemm_f64 dispatches pooled) = calibrated FETCH_SIZE + WRITE_SIZE (rocprofv3 derived counters, KiB).
MI355X_MICROARCH.md (HBM section): FETCH_SIZE reads exactly half of a 16-B/lane streaming read on gfx950;
the 8-B/lane loads and stores of our kernels are calibrated by tools/fetch_calib.hip (pass "calf"/"calw"
in the source directory): the factors measured there (FETCH x2 for 8-B and 16-B loads, WRITE x1 for 8-B
stores) are applied when present. Usage: python tools/pmc_summary.py gpurun_out/pmc2 profiles/r02
"""
import collections
import csv
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)


def load(pass_name):
    files = glob.glob(os.path.join(src, pass_name, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            fam = r["Kernel_Name"].split("<")[0].split("(")[0].replace("void ", "").strip()
            per[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


# calibration: known byte counts of tools/fetch_calib.hip
cal = {"fetch": None, "write": None}
for name, known in (("calf", {"k_read8": 1 << 30, "k_read16": 1 << 30}), ("calw", {"k_write8": 1 << 28})):
    for fam, counters in load(name).items():
        key = fam.split("(")[0]
        for c, v in counters.items():
            if key in known and known[key]:
                factor = known[key] / (sum(v) / len(v) * 1024)
                cal.setdefault("factors", {})[f"{key}:{c}"] = factor
if "factors" in cal:
    cal["fetch"] = cal["factors"].get("k_read8:FETCH_SIZE")
    cal["write"] = cal["factors"].get("k_write8:WRITE_SIZE")

summary = {}
for p in ("fetch", "write", "mfma"):
    for fam, counters in load(p).items():
        for c, v in counters.items():
            summary.setdefault(fam, {})[c] = {"dispatches": len(v), "mean": sum(v) / len(v)}
with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
    json.dump(summary, f, indent=1, sort_keys=True)
# the GEMM family: every GEMM kernel of the step (k_gemm_f64: general tiles; k_gemm_glds: LDS-DMA pipeline),
# pooled per dispatch
g = {}
for p_ in ("fetch", "write", "mfma"):
    for fam, counters in load(p_).items():
        if not fam.startswith("xrs::k_gemm"):
            continue
        for c, v in counters.items():
            g.setdefault(c, []).extend(v)
g = {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in g.items()}
if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
    ff = cal["fetch"] or 1.0
    wf = cal["write"] or 1.0
    fetch, write = g["FETCH_SIZE"]["mean"] * 1024 * ff, g["WRITE_SIZE"]["mean"] * 1024 * wf
    out = {
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "fetch_size_raw_kib": g["FETCH_SIZE"]["mean"],
        "write_size_raw_kib": g["WRITE_SIZE"]["mean"],
        "calibration": {"fetch_factor": ff, "write_factor": wf, "measured": cal.get("factors", {})},
        "dispatches": g["FETCH_SIZE"]["dispatches"],
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over " + os.environ.get(
                      "PMC_CMD", "python3 bench.py --no-cpu --no-cfg5 --no-extras --no-overlap --steps 20 --warmup 3 (tools/gpu_run.sh pmc)") +
                  ", mean per GEMM dispatch (k_gemm_glds + k_gemm_f64), corrected by the 8-B load/store calibration of "
                  "tools/fetch_calib.hip (FETCH x%.3f, WRITE x%.3f); %s/pmc_summary.json" % (ff, wf, dst),
    }
    # the separate split-K reduce launches (k_splitk_reduce, k_splitk_reduce_sym) of the same passes: their bytes
    # summed and spread over the GEMM dispatches (the GEMM family's traffic with its reduce launches included)
    red = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
    nred = 0
    for p_ in ("fetch", "write"):
        for fam, counters in load(p_).items():
            if not fam.startswith("xrs::k_splitk_reduce"):
                continue
            for c, v in counters.items():
                if c in red:
                    red[c] += sum(v)
                    if c == "FETCH_SIZE":
                        nred += len(v)
    if nred:
        rb = red["FETCH_SIZE"] * 1024 * ff + red["WRITE_SIZE"] * 1024 * wf
        out["splitk_reduce"] = {"dispatches": nred, "hbm_bytes_per_reduce": rb / nred,
                                "hbm_bytes_per_gemm_launch": rb / g["FETCH_SIZE"]["dispatches"]}
        out["hbm_bytes_per_launch_incl_splitk_reduce"] = fetch + write + rb / g["FETCH_SIZE"]["dispatches"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in g and "GRBM_GUI_ACTIVE" in g:
        out["mfma_busy_cycles_per_dispatch"] = g["SQ_VALU_MFMA_BUSY_CYCLES"]["mean"]
        out["gui_active_cycles_per_dispatch"] = g["GRBM_GUI_ACTIVE"]["mean"]
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
else:
    print("no GEMM FETCH/WRITE data:", list(summary))
