"""Per-step kernel timeline of a bench profile: python tools/step_phases.py <kernel_trace.csv> [step_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
pos = [i for i, r in enumerate(rows) if 'potrf_rr_batched' in r['Kernel_Name']]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
a, b = pos[k], pos[k + 1]
t0 = int(rows[a]['Start_Timestamp'])


def nm(r):
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('xrs::', '')
    return n.replace('k_gemm_f64', 'G').replace('__amd_rocclr_', '')[:34]


last = t0
for r in rows[a:b]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print("%8.1f %6.1f gap %6.1f q%s %s g=%s z=%s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - last) / 1e3, r['Queue_Id'], nm(r),
                                                 r['Grid_Size_X'], r['Grid_Size_Z']))
    last = max(last, e)
print("span %.1f us" % ((last - t0) / 1e3))
