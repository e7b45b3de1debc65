set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prec_probe.py > gpurun_out/prec_probe.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  --deselect tests/test_headline.py::test_headline_bf16_matches_reference > gpurun_out/pytest_r02b.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r02b.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err
