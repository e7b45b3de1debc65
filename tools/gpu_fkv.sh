# flash_kv joint group walk A/B + the batch-invariance checks: tools/gpu_fkv.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fkv
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_parity.py tests/test_wild.py -k "invarian" -v --timeout 200 --timeout-method thread > $O/inv.log 2>&1 || { echo INV FAILED; tail -30 $O/inv.log; exit 1; }
tail -3 $O/inv.log
timeout -k 10 300 python -u -m pytest tests/test_attention.py -v --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1 || { echo ATTN FAILED; tail -30 $O/attn_tests.log; exit 1; }
tail -3 $O/attn_tests.log
for i in 1 2; do
  DAC_FKV_JOINT=0 timeout -k 10 120 python -u tools/attn_bench.py 200 > $O/ab0_$i.log 2>&1 || exit 1
  DAC_FKV_JOINT=1 timeout -k 10 120 python -u tools/attn_bench.py 200 > $O/ab1_$i.log 2>&1 || exit 1
done
grep -H "variant=8\|variant=11\|variant=12" $O/ab*.log
