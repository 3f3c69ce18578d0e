"""Summarise the PMC passes of tools/pmc_bench.sh per kernel family and write profiles/<tag>/pmc_*.

HBM traffic per k_gemm_f64 launch = FETCH_SIZE + WRITE_SIZE (rocprofv3 derived counters, KiB). Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reads exactly half of a 16-B/lane streaming read on gfx950;
the GEMM's global loads are 8-B/lane, for which the guide gives no calibration, so the raw value is
reported with that caveat. Usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r01
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


summary = {}
for p in ("fetch", "write", "mfma"):
    for fam, counters in load(p).items():
        for c, v in counters.items():
            summary.setdefault(fam, {})[c] = {"dispatches": len(v), "mean": sum(v) / len(v)}
with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
    json.dump(summary, f, indent=1, sort_keys=True)
g = summary.get("xrs::k_gemm_f64", {})
if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
    fetch, write = g["FETCH_SIZE"]["mean"] * 1024, g["WRITE_SIZE"]["mean"] * 1024
    out = {
        "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "dispatches": g["FETCH_SIZE"]["dispatches"],
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py --steps 3 --warmup 1, "
                  "mean per k_gemm_f64 dispatch; raw counters (gfx950 FETCH_SIZE halves 16-B/lane reads; "
                  "these 8-B/lane loads are uncalibrated); profiles/r01/pmc_summary.json",
    }
    if "SQ_VALU_MFMA_BUSY_CYCLES" in g and "GRBM_GUI_ACTIVE" in g:
        out["mfma_busy_cycles_per_dispatch"] = g["SQ_VALU_MFMA_BUSY_CYCLES"]["mean"]
        out["gui_active_cycles_per_dispatch"] = g["GRBM_GUI_ACTIVE"]["mean"]
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
else:
    print("no k_gemm_f64 FETCH/WRITE data:", list(summary))
