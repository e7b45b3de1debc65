# Round-end measurement cycle, every GPU step time-limited and chained:
#   PMC passes (bf16 + fp32 bench workloads) -> profiles/pmc_traffic.json,
#   the -m gpu suite, smoke(), the default bench line (bf16 + fp16 mode), the fp32 line,
#   and a rocprofv3 kernel-stats run. tools/gpu_round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r}
O=gpurun_out/round_$TAG
mkdir -p $O
export TMPDIR=/tmp
PMC_DTYPES="${PMC_DTYPES:-fp16 fp32}" bash tools/pmc_bench.sh $TAG || { echo PMC FAILED; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG profiles/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
timeout -k 10 600 python -u bench.py --dtype fp32 --modes none --lines none > $O/bench_fp32.log 2>&1 || { echo FP32 BENCH FAILED; tail -20 $O/bench_fp32.log; exit 1; }
grep '^{' $O/bench_fp32.log > $O/bench_fp32.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --modes none --lines none > $O/profrun.log 2>&1 || { echo PROF FAILED; tail -20 $O/profrun.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/kernel_stats_summary.txt
cut -c1-400 $O/bench.json $O/bench_fp32.json
