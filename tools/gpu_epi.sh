# Epilogue change: convbench check + timing of the 3x3 shapes, then in-network A/B against the
# baseline library (DAC_LIB_PATH).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 ./tools/convbench 2 "3x3" check > gpurun_out/epi_check.log 2>&1 || { tail -20 gpurun_out/epi_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/epi_check.log) OK, $(grep -c FAIL gpurun_out/epi_check.log) FAIL"
grep FAIL gpurun_out/epi_check.log | head
timeout -k 10 200 ./tools/convbench 50 "3x3" - -1 | cut -c1-75 || exit 1
bash tools/gpu_ab.sh epi "DAC_LIB_PATH=$GRAFT_REPO_ROOT/da-clip_amd/daclip_amd/libdaclip_hip_base.so" "DAC_X=1" 3
