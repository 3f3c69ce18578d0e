"""Top kernels of a rocprofv3 --stats kernel_stats.csv (diagnostics): python tools/ktop.py <csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} ms {int(r['Calls']):7d} calls {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:120]}")
