set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_hip_parity.py tests/test_headline.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02f.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_r02f.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_prof.sh f
