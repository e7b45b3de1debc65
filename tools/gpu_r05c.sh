# Re-entry check of the committed tree: the -m gpu suite, smoke, the default bench line, and the
# per-shape eager conv profile of the fp16 bench batch. Every GPU step time-limited and chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05c}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 300 python -u tools/conv_profile.py --dtype fp16 > $O/convprof_fp16.txt 2>&1 || { echo CONVPROF FAILED; tail -20 $O/convprof_fp16.txt; exit 1; }
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-600
exit $rc
