# conv3w shape sweep: tools/gpu_c3w.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CFGS:-8,4,2 8,4,-3}; do
  echo "== $cfg" 
  DAC_C3W=$cfg timeout -k 10 60 ./tools/convbench 2 "64->64" check || exit 1
  DAC_C3W=$cfg timeout -k 10 60 ./tools/convbench 50 "64->64" || exit 1
done > gpurun_out/c3w_$1.log 2>&1
