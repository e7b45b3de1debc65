#!/bin/bash
# SQ counter passes over the bench workload (eager launches, T=2): per-kernel stall anatomy.
# Output: gpurun_out/pmck_$TAG/p{1,2}/run_counter_collection.csv ; summary kpmc_$TAG.txt
set -o pipefail
TAG=${1:-k}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmck_$TAG
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  DAC_NO_GRAPH=1 timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmck_$TAG/p$i -o run -- \
    python3 -u bench.py --steps 1 --warmup 0 --T 2 --no-cpu-baseline --no-roofline --no-psnr \
    > gpurun_out/pmck_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmck_$TAG/p$i.log; exit 1; }
done
python3 tools/pmc_kern.py gpurun_out/pmck_$TAG > gpurun_out/kpmc_$TAG.txt
