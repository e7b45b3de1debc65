# Round-6 measurement cycle: the -m gpu suite, smoke, a short bench line with the in-graph
# (stamped) roofline, and rocprofv3 --kernel-trace --stats of that same bench command.
#   tools/gpu_r6.sh <tag> [tests|notests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6}
mkdir -p $O
export TMPDIR=/tmp
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  grep -E "FAILED|ERROR" $O/tests.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit $rc; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
CMD="bench.py --steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr"
timeout -k 10 300 python -u $CMD > $O/bench_short.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench_short.log; exit 1; }
grep '^{' $O/bench_short.log > $O/bench_short.json
cut -c1-600 $O/bench_short.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $CMD > $O/profrun.log 2>&1 || { echo PROF FAILED; tail -20 $O/profrun.log; exit 1; }
grep '^{' $O/profrun.log > $O/bench_under_prof.json
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/kernel_stats_summary.txt
head -25 $O/kernel_stats_summary.txt | cut -c1-160
if [ "${3:-}" = full ]; then
  timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo FULL BENCH FAILED; tail -20 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log > $O/bench.json
  cut -c1-800 $O/bench.json
fi
exit ${rc:-0}
