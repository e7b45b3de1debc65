"""Tabulate a convbench sweep log: one row per shape, one column per forced kernel choice."""
import re, sys
rows, cols = {}, []
for line in open(sys.argv[1]):
    m = re.match(r"(.*?)\s+f(-?\d+)\s+variant\s+\d+\s+([\d.]+) us\s+([\d.]+) TF/s", line)
    if not m:
        continue
    name, f, us, tf = m.group(1).strip(), m.group(2), float(m.group(3)), float(m.group(4))
    rows.setdefault(name, {})[f] = (us, tf)
    if f not in cols:
        cols.append(f)
print("%-26s" % "shape (us / TF/s)" + "".join("%14s" % ("f" + c) for c in cols))
for name, d in rows.items():
    best = min(d, key=lambda c: d[c][0])
    print("%-26s" % name + "".join(("%7.1f/%-4.0f%s" % (d[c][0], d[c][1], "*" if c == best else " ")).rjust(14) if c in d else " " * 14 for c in cols))
