# conv2 k-step fragment double-buffer: op-level 1x1 shapes (old vs new convbench), full check,
# tests, in-graph per-symbol times and the in-network A/B against libab/base7.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2pipe
mkdir -p $O
export TMPDIR=/tmp
for b in libab/convbench_base7 tools/convbench; do
  CB_DTYPE=f16 timeout -k 10 120 $b 20 "1x1" - -1 > $O/cb_$(basename $b).log 2>&1 || { echo "CB $b FAILED"; tail $O/cb_$(basename $b).log; exit 1; }
done
paste <(cut -c1-70 $O/cb_convbench_base7.log) <(cut -c40-70 $O/cb_convbench.log) | head -30
CB_DTYPE=f16 timeout -k 10 180 tools/convbench 3 "" check -1 > $O/check.log 2>&1 || { echo "CHECK FAILED"; tail $O/check.log; exit 1; }
echo "check: $(grep -c OK $O/check.log) OK, $(grep -ci fail $O/check.log) fail"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_conv_kernels.py tests/test_normfold.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_rfcmp.sh c2pipe libab/base7.so 2 conv2_kernel
bash tools/gpu_ab.sh c2pipe "DAC_LIB_PATH=libab/base7.so" "DAC_NONE=1" 3
