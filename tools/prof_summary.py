"""Summarise a rocprofv3 rocpd database (or kernel_stats.csv) per kernel name."""
import sqlite3, sys, re, collections
db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
rows = cur.execute("select * from kernels").fetchall()
ci = {c: i for i, c in enumerate(cols)}
name_col = 'kernel_name' if 'kernel_name' in ci else ('name' if 'name' in ci else None)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r[ci[name_col]]
    d = (r[ci['end']] - r[ci['start']]) / 1e3  # us
    n = re.sub(r"\(.*", "", n)
    agg[n][0] += 1; agg[n][1] += d
tot = sum(v[1] for v in agg.values())
print(f"{'calls':>7} {'total_ms':>10} {'avg_us':>9} {'pct':>6}  kernel")
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{c:7d} {t/1e3:10.2f} {t/c:9.1f} {100*t/tot:6.2f}  {n[:150]}")
print(f"total {tot/1e3:.1f} ms")
