# Three-arm interleaved A/B/C of environment settings on the bench workload:
# tools/gpu_ab3.sh <tag> "<env A>" "<env B>" "<env C>" [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_$1
for r in $(seq 1 ${5:-3}); do
  for arm in A B C; do
    case $arm in A) E="$2";; B) E="$3";; C) E="$4";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/ab_$1/$arm$r.log 2>&1 || { echo "$arm$r FAILED"; tail -5 gpurun_out/ab_$1/$arm$r.log; exit 1; }
    echo "$arm ($E) $(grep '^{' gpurun_out/ab_$1/$arm$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
