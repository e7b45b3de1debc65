set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02e.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_r02e.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r02e.json 2> gpurun_out/bench_r02e.err || exit 1
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --kernel-id 999 --no-cpu-baseline --no-psnr > /dev/null 2> gpurun_out/shapeprof_r02e.err
