"""Summary of tools/gpu_flashpmc.sh: per (source, flash kernel, grid) mean duration and counters."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for src in ("net", "iso"):
    for f in glob.glob(os.path.join(root, src + "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "flash" not in r["Kernel_Name"]:
                continue
            key = (src, r["Kernel_Name"][:60], r.get("Grid_Size", "?"))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            agg[key]["_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, c in sorted(agg.items()):
    a = {k: sum(v) / len(v) for k, v in c.items()}
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    line = f"{key[0]} {key[1]} grid={key[2]} n={len(c['_us'])} dur {a['_us']:.1f} us"
    if "SQ_WAIT_ANY" in a:
        line += (f" | wait_any {a['SQ_WAIT_ANY'] / wc:.3f} wait_inst {a['SQ_WAIT_INST_ANY'] / wc:.3f}"
                 f" active {a['SQ_ACTIVE_INST_ANY'] / wc:.3f} lds_wait {a['SQ_WAIT_INST_LDS'] / wc:.3f}"
                 f" mfma_busy {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if "TCC_HIT_sum" in a:
        h, m = a["TCC_HIT_sum"], a["TCC_MISS_sum"]
        line += f" | L2 hit {h / max(1.0, h + m):.3f} (req {h + m:.0f})"
    print(line)
