# In-network A/B of two environment settings on the bench workload (interleaved, short runs):
# tools/gpu_ab.sh <tag> "<env A>" "<env B>" [reps] [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_$1
for r in $(seq 1 ${4:-3}); do
  for arm in A B; do
    if [ $arm = A ]; then E="$2"; else E="$3"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none $5 > gpurun_out/ab_$1/$arm$r.log 2>&1 || { echo "$arm$r FAILED"; tail -5 gpurun_out/ab_$1/$arm$r.log; exit 1; }
    echo "$arm ($E) $(grep '^{' gpurun_out/ab_$1/$arm$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
