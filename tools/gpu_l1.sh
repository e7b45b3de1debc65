# 128x128 64->64 3x3 (the downs.1 ResBlock convs) across v5 shapes and the v4 configurations.
# usage: tools/gpu_l1.sh "<DAC_C3W cfgs>" "<force list>"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/convbench 2 "L1 3x3 64->64" check > gpurun_out/l1_check.log 2>&1 || { cat gpurun_out/l1_check.log; exit 1; }
cat gpurun_out/l1_check.log
for c in $1; do
  echo "== DAC_C3W=$c"
  DAC_C3W=$c timeout -k 10 60 ./tools/convbench 2 "L1 3x3 64->64" check || exit 1
  DAC_C3W=$c timeout -k 10 60 ./tools/convbench 200 "L1 3x3 64->64" || exit 1
done
echo "== forces $2"
timeout -k 10 60 ./tools/convbench 200 "L1 3x3 64->64" - "$2" || exit 1
echo "== all shapes (defaults)"
timeout -k 10 120 ./tools/convbench 100 "" || exit 1
