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
        key = r["Kernel_Name"][:90] + " grid=" + r.get("Grid_Size", "?")
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, c in agg.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    print(k)
    print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(avg.items())))
    if "SQ_WAIT_ANY" in avg:
        print(f"   wait_any {avg['SQ_WAIT_ANY'] / wc:.3f}  wait_inst {avg['SQ_WAIT_INST_ANY'] / wc:.3f}  "
              f"active {avg['SQ_ACTIVE_INST_ANY'] / wc:.3f}  wait_inst_lds {avg['SQ_WAIT_INST_LDS'] / wc:.3f}")
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        print(f"   per wave: valu {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}  mfma {avg['SQ_INSTS_MFMA'] / avg['SQ_WAVES']:.0f}  "
              f"lds {avg['SQ_INSTS_LDS'] / avg['SQ_WAVES']:.0f}  salu {avg['SQ_INSTS_SALU'] / avg['SQ_WAVES']:.0f}  "
              f"vmem_rd {avg.get('SQ_INSTS_VMEM_RD', 0) / avg['SQ_WAVES']:.0f}")
    if "GRBM_GUI_ACTIVE" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        print(f"   mfma_busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if "SQ_LDS_IDX_ACTIVE" in avg:
        print(f"   lds_active/gui? bank_conflict/lds_active {avg['SQ_LDS_BANK_CONFLICT'] / max(1, avg['SQ_LDS_IDX_ACTIVE']):.3f}")
