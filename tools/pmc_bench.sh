#!/bin/bash
# PMC passes over the bench workload (one restore of the bench batch, no eager replay), for each
# dtype in PMC_DTYPES (default "bf16"). Eager launches (DAC_NO_GRAPH=1: same kernels, no graph)
# so every dispatch is sampled. Each pass is its own rocprofv3 run: FETCH_SIZE (3 TCC slots) and
# WRITE_SIZE (2) cannot share a pass. Output: gpurun_out/pmc_$TAG/p<dtype><n>/run_counter_collection.csv
set -o pipefail
TAG=${1:-b}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
for DT in ${PMC_DTYPES:-bf16}; do
  i=0
  for P in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    i=$((i+1))
    # Per-dispatch counters do not depend on T (every step runs the same kernels on the same
    # shapes), so T=10 keeps the serialized PMC run short.
    DAC_NO_GRAPH=1 timeout -s KILL 600 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_$TAG/p$DT$i -o run -- \
      python -u bench.py --steps 1 --warmup 0 --T 10 --dtype $DT --modes none --lines none --no-cpu-baseline --no-roofline --no-psnr ${BENCH_ARGS} \
      > gpurun_out/pmc_$TAG/p$DT$i.log 2>&1 &
    pid=$!
    while kill -0 $pid 2>/dev/null; do sleep 20; echo "pass $DT $i $(date +%T)" >> gpurun_out/pmc_$TAG/heartbeat; done
    wait $pid || { echo "pass $DT $i failed"; tail -5 gpurun_out/pmc_$TAG/p$DT$i.log; exit 1; }
  done
done
echo pmc done
