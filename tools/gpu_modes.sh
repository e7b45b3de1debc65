# Bench lines of the other BASELINE configs on one GPU: fp8 (configs[4]) and Wild-IR (configs[3]).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --dtype fp8 --kernel-id 330 > gpurun_out/bench_fp8.log 2>&1 || { tail -20 gpurun_out/bench_fp8.log; exit 1; }
grep '^{' gpurun_out/bench_fp8.log
timeout -k 10 400 python -u bench.py --model wild-ir --no-cpu-baseline > gpurun_out/bench_wild.log 2>&1 || { tail -20 gpurun_out/bench_wild.log; exit 1; }
grep '^{' gpurun_out/bench_wild.log
