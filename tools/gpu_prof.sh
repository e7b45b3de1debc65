# rocprofv3 kernel stats over a short bench run: tools/gpu_prof.sh <tag> [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-roofline --no-psnr --no-cpu-baseline --modes none --lines none $2 > gpurun_out/profrun_$1.log 2>&1
rc=$?
f=$(find gpurun_out/prof_$1 -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py "$f" > gpurun_out/kstats_$1.txt
grep '^{' gpurun_out/profrun_$1.log | cut -c1-300
exit $rc
