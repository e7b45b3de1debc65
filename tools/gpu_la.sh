# LinearAttention stale reference max: parity (restore / headline fixtures, LA op tests) and an
# interleaved in-network A/B: tools/gpu_la.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/la
timeout -k 10 600 python -u -m pytest tests/test_restore.py tests/test_headline.py tests/test_hip_parity.py tests/test_normfold.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/la/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/la/tests.log; exit 1; }
tail -1 gpurun_out/la/tests.log
grep -i "psnr\|delta" gpurun_out/la/tests.log | head -20
export TMPDIR=/tmp
for arm in 0 1 0 1; do
  DAC_LA_STALE=$arm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/la/prof$arm -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/la/prof$arm.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/la/prof$arm.log; exit 1; }
  echo "stale=$arm"; grep -h "la_proj_ctx\|la_apply\|la_combine" gpurun_out/la/prof$arm/run_kernel_stats.csv | cut -d, -f1-6
  rm -rf gpurun_out/la/prof$arm
done
bash tools/gpu_ab.sh lastale "DAC_LA_STALE=0" "DAC_LA_STALE=1" 2
