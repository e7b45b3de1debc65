"""Per-kernel averages of the SQ counter passes collected by tools/gpu_sqpmc.sh."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    print(k)
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(avg.items())))
    if "SQ_WAIT_ANY" in avg:
        print(f"   wait_any {avg['SQ_WAIT_ANY'] / wc:.3f}  wait_inst {avg['SQ_WAIT_INST_ANY'] / wc:.3f}  "
              f"active {avg['SQ_ACTIVE_INST_ANY'] / wc:.3f}  wait_inst_lds {avg['SQ_WAIT_INST_LDS'] / wc:.3f}")
    if "GRBM_GUI_ACTIVE" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        print(f"   mfma_busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if "SQ_LDS_IDX_ACTIVE" in avg:
        print(f"   lds_active/gui? bank_conflict/lds_active {avg['SQ_LDS_BANK_CONFLICT'] / max(1, avg['SQ_LDS_IDX_ACTIVE']):.3f}")
