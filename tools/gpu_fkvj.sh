# flash_kv joint vs per-group walk in the network (rocprof): tools/gpu_fkvj.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fkvj
export TMPDIR=/tmp
for j in 0 1 0 1; do
  DAC_FKV_JOINT=$j timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fkvj/p$j -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/fkvj/p$j.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/fkvj/p$j.log; exit 1; }
  echo "joint=$j"; grep -h "flash_kv" gpurun_out/fkvj/p$j/run_kernel_stats.csv | cut -d, -f1-4
  rm -rf gpurun_out/fkvj/p$j
done
