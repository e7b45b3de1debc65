#!/bin/bash
# PMC passes over one convbench shape. Each pass is its own rocprofv3 run (counter limits).
set -o pipefail
SHAPE=${1:-"64->64 plain"}
TAG=${2:-p}
FORCE=${3:--1}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE TA_BUSY_avr" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- ./tools/convbench 5 "$SHAPE" - "$FORCE" > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
echo done
