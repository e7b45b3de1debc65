#!/bin/bash
# Per-kernel register / LDS / scratch usage of every translation unit of libdaclip_hip, from the
# compiler's resource remarks (gfx950): tools/kernel_resources.sh > profiles/<round>_kernel_resources.txt
set -o pipefail
cd "$(dirname "$0")/../da-clip_amd"
printf "%-8s %-8s %-8s %-9s %-10s %s\n" VGPRs AGPRs Occ LDS Scratch Kernel
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
    sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
    awk '/Function Name:/ {name=$NF} /VGPRs:/ {v=$NF} /AGPRs:/ {ag=$NF} /ScratchSize/ {sc=$NF} /Occupancy/ {oc=$NF}
         /LDS Size/ {printf "%-8s %-8s %-8s %-9s %-10s %s\n", v, ag, oc, $NF, sc, name}'
done | sort -u -k6
