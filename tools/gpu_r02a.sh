set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r02a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err
