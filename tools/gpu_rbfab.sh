# rbfuse A/B against an earlier build (tools/gpu_rbfab.sh <tag> <base name under libab/>): op-level (convbench rbf, old vs new binary, fused ==
# pair check), conv tests, in-graph per-symbol times and the in-network A/B against libab/<base>.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for b in libab/convbench_$2 tools/convbench; do
  CB_DTYPE=f16 timeout -k 10 120 $b rbf 20 > $O/rbf_$(basename $b).log 2>&1 || { echo "rbf $b FAILED"; tail $O/rbf_$(basename $b).log; exit 1; }
  echo "$b"; grep -E "128->64|B8" $O/rbf_$(basename $b).log | cut -c1-140
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py tests/test_restore.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh $1 "DAC_LIB_PATH=libab/$2.so" "DAC_NONE=1" 3
