# conv_down fragment overlap: op-level (old vs new convbench, Downsample shapes), check, tests,
# in-graph per-symbol and in-network A/B against libab/base8.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cdpipe
mkdir -p $O
export TMPDIR=/tmp
for b in libab/convbench_base8 tools/convbench; do
  CB_DTYPE=f16 timeout -k 10 120 $b 20 "4x4" - -1 > $O/cb_$(basename $b).log 2>&1 || { echo "CB $b FAILED"; tail $O/cb_$(basename $b).log; exit 1; }
done
paste <(cut -c1-70 $O/cb_convbench_base8.log) <(cut -c40-70 $O/cb_convbench.log)
CB_DTYPE=f16 timeout -k 10 180 tools/convbench 3 "" check -1 > $O/check.log 2>&1 || { echo "CHECK FAILED"; tail $O/check.log; exit 1; }
echo "check: $(grep -c OK $O/check.log) OK, $(grep -ci fail $O/check.log) fail"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_conv_kernels.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_rfcmp.sh cdpipe libab/base8.so 2 conv_down
bash tools/gpu_ab.sh cdpipe "DAC_LIB_PATH=libab/base8.so" "DAC_NONE=1" 3
