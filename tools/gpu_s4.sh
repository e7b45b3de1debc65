# GEGLU tile without scratch: convbench timing + lnf check, bench with/without the GEGLU fold,
# GPU tests touching the SpatialTransformer.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 120 ./tools/convbench 50 "geglu" || exit 1
timeout -k 10 180 ./tools/convbench lnf 10 || exit 1
for m in 29 31 29 31; do
  DAC_FOLD=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none > $O/b_$m.log 2>&1 || { tail -20 $O/b_$m.log; exit 1; }
  echo "fold $m $(grep '^{' $O/b_$m.log | cut -c100-140)"
done
DAC_FOLD=31 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_parity.py tests/test_restore.py tests/test_normfold.py -k "256 or bf16_close or fp16_close or restore or norm_folds" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc
