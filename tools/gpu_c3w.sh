# v5 (conv3w) configuration sweep on the 64->64 shapes: tools/gpu_c3w.sh "<cfg> <cfg> ..."
# cfg = waves,TM,stages (DAC_C3W).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/convbench 2 "3x3 64->64" check > gpurun_out/c3w_check.log 2>&1 || { cat gpurun_out/c3w_check.log; exit 1; }
grep -c OK gpurun_out/c3w_check.log
for c in $1; do
  echo "== DAC_C3W=$c"
  DAC_C3W=$c timeout -k 10 60 ./tools/convbench 2 "3x3 64->64" check | grep -c FAIL
  DAC_C3W=$c timeout -k 10 60 ./tools/convbench 100 "3x3 64->64" || exit 1
done
