"""Summarise a rocprofv3 --kernel-trace --stats CSV: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    name = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '')
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>6} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {name[:100]}")
print(f"total {tot/1e6:.1f} ms")
