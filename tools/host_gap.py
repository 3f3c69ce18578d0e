"""What the host does while the device idles (diagnostics).

python tools/host_gap.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [min_gap_us] [n]
For the n largest gaps between consecutive kernels (any queue) of at least min_gap_us, prints the HIP
API calls of every host thread inside the gap with their durations (rocprofv3 --hip-trace --kernel-trace)."""
import csv
import glob
import sys

d = sys.argv[1]
min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 30.0
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ker = list(csv.DictReader(open(glob.glob(d + "/*_kernel_trace.csv")[0])))
api = list(csv.DictReader(open(glob.glob(d + "/*_hip_api_trace.csv")[0])))
ker.sort(key=lambda r: int(r["Start_Timestamp"]))
api.sort(key=lambda r: int(r["Start_Timestamp"]))
gaps = []
end = int(ker[0]["End_Timestamp"])
for r in ker[1:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s - end >= min_gap * 1e3:
        gaps.append((s - end, end, s, r["Kernel_Name"][:50]))
    end = max(end, e)
gaps.sort(reverse=True)
print("%d gaps >= %.0f us; total %.1f us" % (len(gaps), min_gap, sum(g[0] for g in gaps) / 1e3))
for g, a, b, name in gaps[:nshow]:
    print("\n== gap %.1f us before %s" % (g / 1e3, name))
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e >= a and s <= b and not r["Function"].startswith("__hip"):
            print("  t%-6s %+8.1f us  %-28s %7.1f us" % (r["Thread_Id"][-4:], (s - a) / 1e3, r["Function"][:28], (e - s) / 1e3))
