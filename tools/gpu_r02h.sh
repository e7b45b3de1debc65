set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/convbench fp8 > gpurun_out/fp8_check.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py tests/test_headline.py -k "fp8 or bf16_close" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r02h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r02h.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --dtype fp8 --no-cpu-baseline --no-psnr --kernel-id 330 > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err
