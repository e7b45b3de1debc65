# Norm folds A/B in the bench workload, then the whole -m gpu suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --modes none > gpurun_out/s2_on.log 2>&1 || { tail -20 gpurun_out/s2_on.log; exit 1; }
grep '^{' gpurun_out/s2_on.log | cut -c1-330
DAC_NO_LN_FOLD=1 DAC_NO_GN_IN_LN=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --modes none > gpurun_out/s2_off.log 2>&1 || { tail -20 gpurun_out/s2_off.log; exit 1; }
grep '^{' gpurun_out/s2_off.log | cut -c1-330
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?
tail -5 gpurun_out/s2_tests.log
exit $rc
