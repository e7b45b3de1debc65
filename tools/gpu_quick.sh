# Quick GPU check: convbench check+time on a shape filter, bf16 parity tests, bench line.
# tools/gpu_quick.sh <tag> <convbench-filter> [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/convbench 2 "$2" check > gpurun_out/q_check_$1.log 2>&1 || { echo CHECK FAILED; cat gpurun_out/q_check_$1.log; exit 1; }
cat gpurun_out/q_check_$1.log
timeout -k 10 120 ./tools/convbench 50 "$2" > gpurun_out/q_time_$1.log 2>&1 || exit 1
cat gpurun_out/q_time_$1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${3:+-k "$3"} > gpurun_out/q_test_$1.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/q_test_$1.log; exit 1; }
tail -2 gpurun_out/q_test_$1.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q_bench_$1.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/q_bench_$1.log; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/q_bench_$1.log') if l.startswith('{')][0]);print('BENCH',d['value'],d['ms_per_step'],d['psnr']['delta_db'] if d.get('psnr') else None)"
