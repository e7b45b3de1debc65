# v4 buffer-resource DMA (FL bit 10): correctness on every 3x3 shape, then flat vs buffer timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/convbench 2 "3x3" check > gpurun_out/buf_check.log 2>&1 || { tail -20 gpurun_out/buf_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/buf_check.log) OK, $(grep -c FAIL gpurun_out/buf_check.log) FAIL"
grep FAIL gpurun_out/buf_check.log | head
echo "== flat"; DAC_CONV3_BUF=0 timeout -k 10 120 ./tools/convbench 100 "3x3" || exit 1
echo "== buffer"; DAC_CONV3_BUF=1 timeout -k 10 120 ./tools/convbench 100 "3x3" || exit 1
