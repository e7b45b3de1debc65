#!/bin/bash
# One GPU cycle: parity tests -> bench -> rocprof kernel stats. Each step time-limited.
set -o pipefail
TAG=${1:-r}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -3 gpurun_out/test_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
grep '^{' gpurun_out/bench_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-psnr > gpurun_out/profrun_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/profrun_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -2
