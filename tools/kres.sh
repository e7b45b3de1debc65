#!/bin/bash
# Per-kernel register / LDS / occupancy table of one source file (device compile only).
# Usage: tools/kres.sh csrc/conv_k3.hip [name-filter]
cd "$(dirname "$0")/../da-clip_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize -c "$1" -o /tmp/kres.o --offload-device-only \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name": cur = {"name": v}; rows.append(cur)
    elif cur is not None: cur[k] = v
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print("%-90s V%-4s A%-4s occ%-2s spill%s LDS%s" % (r["name"][:90], r.get("VGPRs"), r.get("AGPRs"), r.get("Occupancy [waves/SIMD]"), r.get("VGPRs Spill"), r.get("LDS Size [bytes/block]")))
' "$2"
