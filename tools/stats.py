import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    n = r['Name'].split('(')[0][:100]
    print(f"{int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['AverageNs'])/1e3:8.1f}us {100*float(r['TotalDurationNs'])/tot:5.1f}%  {n}")
print('total ms', tot/1e6)
