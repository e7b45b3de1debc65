#!/bin/bash
# Full GPU cycle: tests + smoke + bench + rocprof stats, then the PMC traffic passes.
set -o pipefail
TAG=${1:-r}
bash tools/gpu_cycle.sh $TAG || exit 1
bash tools/pmc_bench.sh $TAG || exit 1
python tools/pmc_traffic.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/pmc_traffic.json 12 > gpurun_out/pmc_$TAG/summary.txt
