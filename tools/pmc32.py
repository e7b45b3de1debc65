"""Summary of tools/gpu_pmc32.sh: per (source, kernel, grid) mean counters, L2 hit rate, clock."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    src = os.path.relpath(f, root).split(os.sep)[0][:-1]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "conv2_kernel" not in k:
            continue
        key = (src, k[:70], r.get("Grid_Size", "?"))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key in sorted(agg):
    a = {n: sum(v) / len(v) for n, v in agg[key].items()}
    s = f"{key[0]:4s} grid={key[2]:>8s} dur={a['_dur_us']:7.1f}us"
    if "TCC_HIT_sum" in a:
        h, m = a["TCC_HIT_sum"], a["TCC_MISS_sum"]
        s += f" L2hit={h / max(1, h + m):.3f} req={h + m:.3g}"
    if "GRBM_GUI_ACTIVE" in a:
        s += f" clk={a['GRBM_GUI_ACTIVE'] / 8 / (a['_dur_us'] * 1e3):.2f}GHz"
    if "SQ_WAIT_ANY" in a:
        wc = a["SQ_WAVE_CYCLES"] or 1
        s += f" wait_any={a['SQ_WAIT_ANY'] / wc:.2f} wait_inst={a['SQ_WAIT_INST_ANY'] / wc:.2f}"
        s += f" mfma={a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
    if "TCC_EA0_RDREQ_sum" in a:
        s += f" ea_rd={a['TCC_EA0_RDREQ_sum']:.3g} dram={a['TCC_EA0_RDREQ_DRAM_sum']:.3g}"
    print(s + "  " + key[1][-40:])
