"""The evidence tooling's arithmetic on synthetic rocprofv3 counter files (no GPU): tools/pmc_summary.py turns
FETCH_SIZE / WRITE_SIZE passes into the bytes per GEMM launch that bench.py reports as roofline.traffic, with the
fetch_calib calibration applied and the split-K reduce launches' bytes spread over the GEMM launches."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(d, name, rows):
    os.makedirs(os.path.join(d, name), exist_ok=True)
    with open(os.path.join(d, name, "p_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for k, c, v in rows:
            w.writerow({"Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})


def test_pmc_summary_traffic(tmp_path):
    src, dst = str(tmp_path / "pmc"), str(tmp_path / "out")
    gib, mib = 1 << 30, 1 << 20
    # calibration: 1 GiB read by 8-B and 16-B loads reports half its bytes; 256 MiB of 8-B stores report them all
    _write(src, "calf", [("k_read8(double const*, double*)", "FETCH_SIZE", gib / 2 / 1024),
                         ("k_read16(double const*, double*)", "FETCH_SIZE", gib / 2 / 1024)])
    _write(src, "calw", [("k_write8(double*)", "WRITE_SIZE", (1 << 28) / 1024)])
    # two GEMM dispatches (10 / 12 MiB fetched as reported, 4 / 6 MiB written) and three reduce dispatches
    gemm = "void xrs::k_gemm_glds<64, 64, 2, 2, 2, false, true, xrs::GemmOne, 32, 2>(xrs::GemmOne)"
    red = "void xrs::k_splitk_reduce<xrs::GemmOne>(xrs::GemmOne)"
    _write(src, "fetch", [(gemm, "FETCH_SIZE", 10 * mib / 1024), (gemm, "FETCH_SIZE", 12 * mib / 1024),
                          (red, "FETCH_SIZE", 1 * mib / 1024), (red, "FETCH_SIZE", 1 * mib / 1024),
                          (red, "FETCH_SIZE", 1 * mib / 1024)])
    _write(src, "write", [(gemm, "WRITE_SIZE", 4 * mib / 1024), (gemm, "WRITE_SIZE", 6 * mib / 1024),
                          (red, "WRITE_SIZE", 0.5 * mib / 1024), (red, "WRITE_SIZE", 0.5 * mib / 1024),
                          (red, "WRITE_SIZE", 0.5 * mib / 1024)])
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src, dst], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0, p.stderr
    t = json.load(open(os.path.join(dst, "pmc_traffic.json")))
    assert abs(t["calibration"]["fetch_factor"] - 2.0) < 1e-12 and abs(t["calibration"]["write_factor"] - 1.0) < 1e-12
    # per GEMM launch: fetch (10 + 12) / 2 MiB x 2, write (4 + 6) / 2 MiB
    assert abs(t["fetch_bytes_per_launch"] - 22 * mib) < 1e-3 and abs(t["write_bytes_per_launch"] - 5 * mib) < 1e-3
    assert abs(t["hbm_bytes_per_launch"] - 27 * mib) < 1e-3
    # reduces: 3 x (1 MiB x 2 + 0.5 MiB) = 7.5 MiB over 2 GEMM launches
    assert t["splitk_reduce"]["dispatches"] == 3
    assert abs(t["splitk_reduce"]["hbm_bytes_per_gemm_launch"] - 3.75 * mib) < 1e-3
    assert abs(t["hbm_bytes_per_launch_incl_splitk_reduce"] - 30.75 * mib) < 1e-3
    assert t["dispatches"] == 2
