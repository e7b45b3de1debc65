"""Per-kernel mean PMC values (per dispatch) from tools/pmc_kern.sh passes."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:26s} {sum(v) / len(v):16.1f}  n={len(v)}")
