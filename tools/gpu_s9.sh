# Wild-IR (configs[3]) and fp8 (configs[4]) bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --model wild-ir --no-cpu-baseline --modes none > gpurun_out/s9_wild.log 2>&1 || { tail -20 gpurun_out/s9_wild.log; exit 1; }
grep '^{' gpurun_out/s9_wild.log > gpurun_out/s9_wild.json
timeout -k 10 600 python -u bench.py --dtype fp8 --no-cpu-baseline --modes none > gpurun_out/s9_fp8.log 2>&1 || { tail -20 gpurun_out/s9_fp8.log; exit 1; }
grep '^{' gpurun_out/s9_fp8.log > gpurun_out/s9_fp8.json
cut -c1-300 gpurun_out/s9_wild.json gpurun_out/s9_fp8.json
