# log2-domain flash_kv: attention tests + microbench, then the full validation / A/B:
# tools/gpu_fkv.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention.py -v --timeout 120 --timeout-method thread > gpurun_out/fkv_$1_tests.log 2>&1 || { tail -30 gpurun_out/fkv_$1_tests.log; exit 1; }
tail -2 gpurun_out/fkv_$1_tests.log
timeout -k 10 120 python3 -u tools/attn_bench.py 50 > gpurun_out/attn_$1.log 2>&1 || { cat gpurun_out/attn_$1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_$1.log
bash tools/gpu_val_ab.sh $1
