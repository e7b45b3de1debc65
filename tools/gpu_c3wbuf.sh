# v5 buffer-descriptor DMA (DAC_C3W_BUF): check on the 64->64 shapes, timing both forms, then
# in-network A/B against the baseline library.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/convbench 2 "64->64" check > gpurun_out/c3wbuf_check.log 2>&1 || { tail -20 gpurun_out/c3wbuf_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/c3wbuf_check.log) OK, $(grep -c FAIL gpurun_out/c3wbuf_check.log) FAIL"; grep FAIL gpurun_out/c3wbuf_check.log
for p in 1 2; do for b in 0 1; do echo "== BUF=$b"; DAC_C3W_BUF=$b timeout -k 10 120 ./tools/convbench 50 "3x3 64->64" - | cut -c1-75 || exit 1; done; done
bash tools/gpu_ab.sh c3wbuf "DAC_LIB_PATH=$GRAFT_REPO_ROOT/da-clip_amd/daclip_amd/libdaclip_hip_base.so" "DAC_X=1" 3
