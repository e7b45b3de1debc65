# Full -m gpu suite and a bench line with the current defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s6_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s6_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/s6_tests.log | head; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --modes fp16 > gpurun_out/s6_bench.log 2>&1 || { tail gpurun_out/s6_bench.log; exit 1; }
grep '^{' gpurun_out/s6_bench.log | cut -c1-200
