# In-network comparison of N environment settings: per arm one rocprofv3 kernel-stats run of a
# short bench (per-kernel averages of the kernels matching FILTER) and the bench value, arms
# interleaved over REPS rounds. tools/gpu_arms.sh <tag> "<filter regex>" "<env 1>" "<env 2>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; FILT=$2; shift 2
O=gpurun_out/arms_$TAG
mkdir -p $O
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o run -- python3 -u bench.py --steps 2 --warmup 1 --T 20 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/p$i.log 2>&1 || { echo "arm $i prof FAILED"; tail -5 $O/p$i.log; exit 1; }
  echo "== arm $i ($E) $(grep '^{' $O/p$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  python3 tools/kstats.py $(find $O/p$i -name "*kernel_stats.csv" | head -1) > $O/k$i.txt
  grep -E "$FILT" $O/k$i.txt | head -12
  tail -1 $O/k$i.txt
done
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/b$i$r.log 2>&1 || { echo "arm $i bench FAILED"; tail -5 $O/b$i$r.log; exit 1; }
    echo "bench arm $i r$r ($E) $(grep '^{' $O/b$i$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
