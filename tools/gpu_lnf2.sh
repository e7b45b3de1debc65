# LN-fold moments split across the WGN waves: op-level (convbench lnf vs host fp64, both builds),
# the norm-fold / conv / parity / mixed tests, then the in-network A/B against libab/base3.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lnf2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/convbench lnf 20 > $O/lnf.log 2>&1 || { echo "convbench lnf FAILED"; tail $O/lnf.log; exit 1; }
cut -c1-170 $O/lnf.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py tests/test_normfold.py tests/test_hip_parity.py tests/test_mixed.py tests/test_restore.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh lnf2 "DAC_LIB_PATH=libab/base3.so" "DAC_NONE=1" 3
