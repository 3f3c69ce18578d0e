"""Summarise a rocprofv3 kernel-trace CSV: median duration per (kernel, grid) in dispatch order."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.OrderedDict()
for r in rows:
    k = (r['Kernel_Name'].split('(')[0][-60:], r['Grid_Size_X'], r['Grid_Size_Z'])
    agg.setdefault(k, []).append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in agg.items():
    v = sorted(v)
    print("  %-60s grid %7s z %3s n %4d median %9.1f us" % (k[0], k[1], k[2], len(v), v[len(v) // 2] / 1e3))
