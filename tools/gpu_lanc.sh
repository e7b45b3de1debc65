# LinearAttention chunk count sweep (la_proj_ctx + la_combine_weff per-kernel times): tools/gpu_lanc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lanc
export TMPDIR=/tmp
for nc in 128 64 32 128 64 32; do
  DAC_LA_NC=$nc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lanc/p$nc -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/lanc/p$nc.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/lanc/p$nc.log; exit 1; }
  echo "nc=$nc"; grep -h "la_proj_ctx\|la_combine" gpurun_out/lanc/p$nc/run_kernel_stats.csv | cut -d, -f1-4
  rm -rf gpurun_out/lanc/p$nc
done
