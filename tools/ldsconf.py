"""Per-kernel LDS bank-conflict share and instruction mix from tools/gpu_ldsconf.sh's counter pass,
sorted by summed dispatch time."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:100]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        if d not in disp[k]:
            disp[k].add(d)
            agg[k]["_us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rows = sorted(agg.items(), key=lambda kv: -kv[1]["_us"])
print(f"{'us':>9} {'n':>5} {'conf/lds':>8} {'valu/w':>7} {'mfma/w':>7} {'lds/w':>6} {'salu/w':>7}  kernel")
for k, c in rows[:40]:
    w = c.get("SQ_WAVES", 0) or 1
    conf = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0))
    print(f"{c['_us']:9.1f} {len(disp[k]):5d} {conf:8.3f} {c.get('SQ_INSTS_VALU', 0) / w:7.0f} "
          f"{c.get('SQ_INSTS_MFMA', 0) / w:7.0f} {c.get('SQ_INSTS_LDS', 0) / w:6.0f} {c.get('SQ_INSTS_SALU', 0) / w:7.0f}  {k}")
