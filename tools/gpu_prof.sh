# Measurement cycle: PMC passes (fp16 bench workload) -> profiles/pmc_traffic.json, rocprofv3
# kernel stats of the bench command, then the default bench line. tools/gpu_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-p}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
PMC_DTYPES="${PMC_DTYPES:-fp16}" bash tools/pmc_bench.sh $TAG || { echo PMC FAILED; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG profiles/pmc_traffic.json > $O/pmc_traffic.txt || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/profrun.log 2>&1 || { echo PROF FAILED; tail -20 $O/profrun.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/kernel_stats_summary.txt
head -40 $O/kernel_stats_summary.txt
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
cut -c1-1500 $O/bench.json
