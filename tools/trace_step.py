"""One UNet step of a rocprofv3 kernel trace, in dispatch order: duration of each kernel and the
idle gap before it (the step is located as the dispatches between two consecutive sde_step
kernels of the last graph replay). Usage: python tools/trace_step.py run_kernel_trace.csv"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sde_step" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a + 1:b + 1]
tot_d = tot_g = 0.0
prev_end = int(rows[a]["End_Timestamp"])
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d, g = (e - s) / 1e3, (s - prev_end) / 1e3
    tot_d += d; tot_g += g
    prev_end = e
    n = r["Kernel_Name"]
    n = re.sub(r"^_ZN3dac\d+", "", n)[:70]
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{d:8.1f} {g:6.1f}  wg={grid:6d}  {n}")
print(f"step: {len(step)} kernels, busy {tot_d:.1f} us, gaps {tot_g:.1f} us")
