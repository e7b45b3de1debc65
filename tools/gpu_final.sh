# Round-end measurement: -m gpu suite, smoke, PMC passes (profiles/pmc_traffic.json), rocprofv3
# kernel trace + stats of the short bench command, and the default bench line.
#   tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
grep -E "FAILED|ERROR" $O/tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
PMC_DTYPES=fp16 bash tools/pmc_bench.sh $T || { echo PMC FAILED; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_$T $O/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
cp $O/pmc_traffic.json profiles/pmc_traffic.json
CMD="bench.py --steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $CMD > $O/profrun.log 2>&1 || { echo PROF FAILED; tail -20 $O/profrun.log; exit 1; }
grep '^{' $O/profrun.log > $O/bench_under_rocprof.json
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/kernel_stats_summary.txt
head -8 $O/kernel_stats_summary.txt | cut -c1-150
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo FULL BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
cut -c1-400 $O/bench.json
exit $rc
