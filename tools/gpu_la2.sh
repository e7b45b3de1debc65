# LinearAttention LDS swizzles: op-level timing (convbench la, old vs new build's checksums are
# printed for comparison), the network parity tests that run LinearAttention, the bank-conflict
# pass, then the in-network A/B against libab/v3swz.so (the build before this change).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/la2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/convbench la 20 > $O/la.log 2>&1 || { echo "convbench la FAILED"; tail $O/la.log; exit 1; }
cat $O/la.log | cut -c1-160
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_normfold.py tests/test_mixed.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ldsconf.sh la2 > $O/ldsc.txt 2>&1 || { echo "ldsconf failed"; tail $O/ldsc.txt; exit 1; }
grep -E "la_|conv3_kernel" $O/ldsc.txt | cut -c1-150
bash tools/gpu_ab.sh la2 "DAC_LIB_PATH=libab/v3swz.so" "DAC_NONE=1" 3
