# Batch-8 vs single-image invariance and the attention group-count identity: tools/gpu_inv8.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/inv8
timeout -k 10 600 python -u -m pytest tests/test_attention.py tests/test_hip_parity.py tests/test_wild.py -m gpu -v --timeout 300 --timeout-method thread -k "invarian or bit_identical or batch8 or attention" > gpurun_out/inv8/tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/inv8/tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/inv8/tests.log | cut -c1-150
