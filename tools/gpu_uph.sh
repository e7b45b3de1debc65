# Row-phase upsample conv: op-level check + timing, in-network A/B (DAC_UPH), restore tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/uph_${1:-a}
mkdir -p $O
timeout -k 10 120 tools/convbench uph 20 > $O/cb.log 2>&1; rc=$?; cat $O/cb.log; [ $rc -eq 0 ] || { echo CONVBENCH FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_restore.py tests/test_headline.py tests/test_hip_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep -h "restore_fp16\|restore_bf16" gpurun_out/restore_metrics.jsonl | tail -2 | cut -c1-200
bash tools/gpu_ab.sh uph "DAC_UPH=1" "DAC_UPH=2" 3
