# Iteration check: GPU tests (optional -k filter), bench line, rocprof kernel stats summary.
# tools/gpu_iter.sh <tag> [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${2:+-k "$2"} > gpurun_out/i_test_$1.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/i_test_$1.log; exit 1; }
tail -2 gpurun_out/i_test_$1.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/i_bench_$1.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/i_bench_$1.log; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/i_bench_$1.log') if l.startswith('{')][0]);print('BENCH',d['value'],d['ms_per_step'],d['psnr']['delta_db'] if d.get('psnr') else None)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iprof_$1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline > gpurun_out/iprof_$1.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/iprof_$1.log; exit 1; }
python3 tools/kstats.py gpurun_out/iprof_$1/run_kernel_stats.csv > gpurun_out/ikstats_$1.txt
head -30 gpurun_out/ikstats_$1.txt
