# Session check: folded-norm GEMM checks, parity tests touching the SpatialTransformer, restore
# bars, 128^2 v5 sweep, v4 stagger sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
#(lnf/gns checks passed)
#(attn_bench: see DESIGN)
DAC_NO_LN_FOLD=0 DAC_NO_GN_IN_LN=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_parity.py tests/test_restore.py tests/test_conv_kernels.py tests/test_attention.py tests/test_normfold.py -k "normfold or norm_folds or 256 or bf16_close or fp16_close or restore or folded or prenorm or attention" > gpurun_out/s1_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|dPSNR|rel" gpurun_out/s1_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
bash tools/gpu_l1.sh "8,2,2 8,2,3 4,4,3 4,4,4 6,4,2" "40,48,41,49,12" || exit 1
bash tools/gpu_stag.sh "0 4 8 12 16 24 -8 -16 0"
