# Checkpoint measurement: the -m gpu suite, smoke, PMC passes + rocprof kernel stats + the bench
# line (tools/gpu_prof.sh). tools/gpu_checkpoint.sh <tag>; results under gpurun_out/prof_<tag>.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-checkpoint}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/gpu_prof.sh ${1:-checkpoint} || exit 1
exit $rc
