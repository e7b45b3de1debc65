# LN-fold (shifted moments) check and the conv / norm-fold GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/convbench lnf 5 > gpurun_out/lnf.log 2>&1; rc=$?
cat gpurun_out/lnf.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 2 ] || [ $rc -eq 3 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_normfold.py tests/test_restore.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_lnf.log 2>&1
rc=$?
tail -25 gpurun_out/t_lnf.log
exit $rc
