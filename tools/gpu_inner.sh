# Bottom level as 2 x 2 sub-branches (DAC_SPLIT_INNER=1): bit-identity tests, then in-network A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/inner
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split_branches or batch8 or invariance" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh inner "DAC_SPLIT_INNER=0" "DAC_SPLIT_INNER=1" 4
