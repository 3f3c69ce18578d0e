import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6} tot={float(r['TotalDurationNs'])/1e6:8.2f}ms avg={float(r['AverageNs'])/1e3:8.1f}us {100*float(r['TotalDurationNs'])/tot:5.1f}%")
