# fp8 ResBlock pair (conv3q.hip): op-level check + timing, the fp8 tests, and the fp8 / fp16
# bench lines on one box. tools/gpu_q8.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/q8_${1:-a}
mkdir -p $O
timeout -k 10 120 tools/convbench q8 10 > $O/cb.log 2>&1; rc=$?; cat $O/cb.log; [ $rc -eq 0 ] || { echo CONVBENCH FAILED rc=$rc; exit 1; }
timeout -k 10 600 python -u -m pytest tests -k "fp8" -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|restore_fp8|headline" $O/tests.log | tail -12
timeout -k 10 500 python -u bench.py --dtype fp8 --batch 8 --modes none --lines none --no-cpu-baseline --no-roofline > $O/b8.log 2>&1 || { echo BENCH8 FAILED; tail -20 $O/b8.log; exit 1; }
timeout -k 10 500 python -u bench.py --modes none --lines none --no-cpu-baseline --no-roofline --no-psnr > $O/b16.log 2>&1 || { echo BENCH16 FAILED; tail -20 $O/b16.log; exit 1; }
DAC_Q8=0 timeout -k 10 500 python -u bench.py --dtype fp8 --batch 8 --modes none --lines none --no-cpu-baseline --no-roofline --no-psnr > $O/b8off.log 2>&1 || { echo BENCH8OFF FAILED; tail -20 $O/b8off.log; exit 1; }
for f in b8 b16 b8off; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['dtype'], d['value'], d['ms_per_step'], d.get('psnr',{}).get('delta_db'))"; done
