"""Timeline of the last N kernel dispatches of a rocprofv3 kernel trace (diagnostics):
python tools/trace_timeline.py <run_kernel_trace.csv> [N]  -> start offset, duration, gap, name"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
end_prev = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "").replace("xrs::", "")[:70]
    print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:7.2f}  gap {(s - end_prev) / 1e3:7.2f}  q{r.get('Queue_Id', '?')}  {short}")
    end_prev = max(end_prev, e)
print(f"total span {(end_prev - t0) / 1e3:.2f} us")
