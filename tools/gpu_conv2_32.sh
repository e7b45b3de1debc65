# In-network sweep of the 1x1 GEMM configuration on the 32x32 level (DAC_CONV2_FORCE32).
set -o pipefail
cd $GRAFT_REPO_ROOT
for f in 0 13 14 15 16 2 4 6 0; do
  DAC_CONV2_FORCE32=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/s7_$f.log 2>&1 || { tail -5 gpurun_out/s7_$f.log; exit 1; }
  echo "force32 $f $(grep '^{' gpurun_out/s7_$f.log | cut -c100-140)"
done
