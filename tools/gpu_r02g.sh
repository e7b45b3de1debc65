set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02g.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_r02g.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r02g.json 2> gpurun_out/bench_r02g.err || exit 1
bash tools/gpu_prof.sh g
