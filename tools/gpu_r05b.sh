# conv3r first light: op-level check + timing (convbench), then the bench and the new GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 180 tools/convbench 1 "64->64" check -1,33,70 > $O/cb_check.txt 2>&1 || { echo CHECK FAILED rc=$?; tail -20 $O/cb_check.txt; exit 1; }
cat $O/cb_check.txt
timeout -k 10 180 tools/convbench 50 "64->64" - -1,33 > $O/cb_time.txt 2>&1 || { echo TIME FAILED; tail -20 $O/cb_time.txt; exit 1; }
cat $O/cb_time.txt
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -30 $O/bench.log; exit 1; }
tail -c 2500 $O/bench.log
timeout -k 10 900 python -u -m pytest tests/test_wild.py tests/test_text.py tests/test_headline.py tests/test_attention.py tests/test_conv_kernels.py tests/test_restore.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|rel|argmax|headline|passed|failed" $O/tests.log | tail -60
exit $rc
