# rbfuse fragment offsets held in VGPRs: op-level check (convbench rbf: fused == conv3r pair, bit
# for bit; fp16 and bf16), the conv / parity tests, then the in-network A/B against libab/base2.so
# (the build before the change).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rbf3
mkdir -p $O
export TMPDIR=/tmp
for dt in f16 bf16; do
  CB_DTYPE=$dt timeout -k 10 120 tools/convbench rbf 20 > $O/rbf_$dt.log 2>&1 || { echo "convbench rbf $dt FAILED"; tail $O/rbf_$dt.log; exit 1; }
  cut -c1-150 $O/rbf_$dt.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py tests/test_hip_parity.py tests/test_mixed.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh rbf3 "DAC_LIB_PATH=libab/base2.so" "DAC_NONE=1" 3
