# Per-kernel rocprofv3 stats of the bench workload in bf16 and fp16, back to back on one box,
# to diff the two modes kernel by kernel: tools/gpu_dtype_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for DT in ${DTS:-bf16 fp16 bf16 fp16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1_$DT -o run -- python3 bench.py --steps 3 --warmup 1 --no-roofline --no-psnr --no-cpu-baseline --modes none --lines none --dtype $DT > gpurun_out/profrun_$1_$DT.log 2>&1 || { echo "PROF $DT FAILED"; tail -20 gpurun_out/profrun_$1_$DT.log; exit 1; }
  f=$(find gpurun_out/prof_$1_$DT -name "*kernel_stats.csv" | head -1)
  python3 tools/kstats.py "$f" > gpurun_out/kstats_$1_$DT.txt
  grep '^{' gpurun_out/profrun_$1_$DT.log | cut -c1-200
done
