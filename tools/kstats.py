"""Summarise a rocprofv3 kernel_stats.csv: calls, total ms, avg us, share, short name."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"]
    print(f"{int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1e6:10.2f}ms {float(r['AverageNs']) / 1e3:9.1f}us "
          f"{100 * float(r['TotalDurationNs']) / tot:5.1f}%  {n[:110]}")
print(f"total ms {tot / 1e6:.4f}")
