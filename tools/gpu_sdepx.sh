# Pixel-per-thread SDE step: bit-identity test + per-kernel times of both forms: tools/gpu_sdepx.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sdepx
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -m gpu -v -k "sde_step_pixel" --timeout 200 --timeout-method thread > gpurun_out/sdepx/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/sdepx/tests.log; exit 1; }
tail -1 gpurun_out/sdepx/tests.log
for a in 0 1; do
  DAC_SDE_PX=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sdepx/p$a -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/sdepx/p$a.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/sdepx/p$a.log; exit 1; }
  echo "px=$a"; grep -h "sde_step" gpurun_out/sdepx/p$a/run_kernel_stats.csv | cut -d, -f1-4
  rm -rf gpurun_out/sdepx/p$a
done
