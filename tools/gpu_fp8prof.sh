# Per-kernel profile of the fp8 handles on the bench workload: tools/gpu_fp8prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fp8prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp8prof/p -o run -- python3 -u bench.py --dtype fp8 --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/fp8prof/run.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/fp8prof/run.log; exit 1; }
grep '^{' gpurun_out/fp8prof/run.log | cut -c1-200
python3 tools/kstats.py gpurun_out/fp8prof/p/run_kernel_stats.csv > gpurun_out/fp8prof/summary.txt
head -25 gpurun_out/fp8prof/summary.txt | cut -c1-140
rm -f gpurun_out/fp8prof/p/run_kernel_trace.csv
