set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/vitg
timeout -k 10 600 python -u -m pytest tests/test_hip_parity.py tests/test_wild.py tests/test_text.py -m gpu -x -q -k "encode or degradation or l14" --timeout 300 --timeout-method thread > gpurun_out/vitg/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/vitg/tests.log; exit 1; }
tail -1 gpurun_out/vitg/tests.log
bash tools/gpu_ab.sh splitk "DAC_SPLITK=0" "DAC_SPLITK=1" 3
