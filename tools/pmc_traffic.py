"""Reduce the PMC passes of tools/pmc_bench.sh to per-kernel HBM traffic and MFMA busy.

HBM bytes per dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024:
  * FETCH_SIZE / WRITE_SIZE are in KiB (counter_defs.yaml: .../1024);
  * on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced (16 B/lane) reads,
    `global_load` and `global_load_lds` alike (MI355X_MICROARCH.md, HBM section) -> x2;
    every hot kernel here reads 16 B/lane.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GUI * 1024 SIMDs) (MfmaUtil, gfx950), where GUI is the
per-XCD GRBM_GUI_ACTIVE: rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs (a 90 us
launch shows ~1.8M cycles = 8 x 218k at 2.4 GHz) while MfmaUtil takes reduce(.., max), so
the summed value is divided by 8.
Usage: python tools/pmc_traffic.py gpurun_out/pmc_b out.json [top_n]
"""
import collections
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))


def mean(v):
    return sum(v) / len(v) if v else None


res = {}
for k, c in vals.items():
    fetch, write = mean(c.get("FETCH_SIZE", [])), mean(c.get("WRITE_SIZE", []))
    gui, mf = mean(c.get("GRBM_GUI_ACTIVE", [])), mean(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
    n = len(c.get("FETCH_SIZE", [])) or max(len(v) for v in c.values())
    e = {"dispatches": n, "fetch_kib_raw": fetch, "write_kib": write}
    if fetch is not None and write is not None:
        e["hbm_bytes_per_dispatch"] = 2 * fetch * 1024 + write * 1024
        e["hbm_bytes_total"] = e["hbm_bytes_per_dispatch"] * n
    if gui and mf is not None:
        e["mfma_busy"] = mf / (gui / 8 * 1024)
        e["gui_active_cycles_per_xcd"] = gui / 8
    res[k] = e
json.dump({"method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch (gfx950 FETCH_SIZE x2 "
                     "correction for 16 B/lane reads); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / "
                     "(GRBM_GUI_ACTIVE/8 XCDs * 1024)", "kernels": res}, open(out, "w"), indent=1)
rows = sorted(res.items(), key=lambda kv: -kv[1].get("hbm_bytes_total", 0))
tot = sum(v.get("hbm_bytes_total", 0) for v in res.values())
print(f"total HBM bytes over the run: {tot / 1e9:.2f} GB")
for k, v in rows[:top]:
    print(f"{v['dispatches']:6d}  {v.get('hbm_bytes_per_dispatch', 0) / 1e6:9.2f} MB/disp  "
          f"{v.get('hbm_bytes_total', 0) / 1e9:7.2f} GB  mfma {100 * v.get('mfma_busy', 0):5.1f}%  {k[:90]}")
