"""Per-kernel PMC means from rocprofv3 counter_collection.csv files under a directory (diagnostic).
python tools/pmc_gemm.py DIR  -> one line per (kernel, counter): mean over dispatches."""
import collections
import csv
import glob
import os
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = k.split("(")[0].replace("void ", "").replace("xrs::", "")[:70]
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(per.items()):
    n = max(len(v) for v in cs.values())
    if n < 5:
        continue
    print(k, f"({n} dispatches)")
    for c, v in sorted(cs.items()):
        print(f"    {c:32s} {sum(v) / len(v):14.1f}")
