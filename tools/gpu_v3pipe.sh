# v3 fragment double-buffer: op-level timing old vs new convbench (fp16, the 32^2 3x3 shapes),
# the full convbench check, parity tests, then the in-network A/B against libab/base4.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/v3pipe
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in libab/convbench_base4 tools/convbench; do
    CB_DTYPE=f16 timeout -k 10 120 $b 20 "L3 3x3" - -1 > $O/cb_$(basename $b)_$r.log 2>&1 || { echo "CB $b FAILED"; tail $O/cb_$(basename $b)_$r.log; exit 1; }
    echo "$b: $(grep -E '512->512|768->512' $O/cb_$(basename $b)_$r.log | cut -c1-80 | tr '\n' ' ')"
  done
done
CB_DTYPE=f16 timeout -k 10 180 tools/convbench 3 "" check -1 > $O/check.log 2>&1 || { echo "CHECK FAILED"; tail $O/check.log; exit 1; }
echo "check: $(grep -c OK $O/check.log) OK, $(grep -ci fail $O/check.log) fail"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_conv_kernels.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh v3pipe "DAC_LIB_PATH=libab/base4.so" "DAC_NONE=1" 3
