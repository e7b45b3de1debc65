#!/bin/bash
# 3x3 conv kernel sweep on the GPU: correctness (check mode) then timing per forced choice.
# Usage: tools/conv_sweep.sh TAG "force,list" [shape-filter]
set -o pipefail
TAG=$1; FORCES=$2; FLT=${3:-3x3}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/convbench 2 "$FLT" check "$FORCES" > gpurun_out/sweep_check_$TAG.log 2>&1 || { echo CHECK RUN FAILED; tail -20 gpurun_out/sweep_check_$TAG.log; exit 1; }
grep -c FAIL gpurun_out/sweep_check_$TAG.log && { echo "CHECK FAILURES"; grep FAIL gpurun_out/sweep_check_$TAG.log; }
timeout -k 10 180 ./tools/convbench 20 "$FLT" - "$FORCES" > gpurun_out/sweep_time_$TAG.log 2>&1 || { echo TIME RUN FAILED; tail -20 gpurun_out/sweep_time_$TAG.log; exit 1; }
cat gpurun_out/sweep_time_$TAG.log
