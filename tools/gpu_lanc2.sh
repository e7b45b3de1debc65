# Per-level LinearAttention chunk counts: parity + interleaved in-network A/B: tools/gpu_lanc2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lanc2
timeout -k 10 700 python -u -m pytest tests/test_restore.py tests/test_headline.py tests/test_hip_parity.py tests/test_normfold.py tests/test_wild.py tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lanc2/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/lanc2/tests.log; exit 1; }
tail -1 gpurun_out/lanc2/tests.log
bash tools/gpu_ab.sh lanc "DAC_LA_NC=128" "DAC_LA_NC=0" 3
