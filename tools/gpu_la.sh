# LinearAttention op-level A/B: tools/convbench_old (committed linattn) vs tools/convbench (with
# the q-softmax shift given as $1, 0 = per-pixel max), plus a per-kernel rocprofv3 split of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/la
mkdir -p $O
export TMPDIR=/tmp
QS=${1:-40}
for r in 1 2; do
  echo "== old r$r"; timeout -k 10 60 ./tools/convbench_old la 50 || exit 1
  echo "== new qshift 0 r$r"; timeout -k 10 60 ./tools/convbench la 50 0 || exit 1
  echo "== new qshift $QS r$r"; timeout -k 10 60 ./tools/convbench la 50 $QS || exit 1
done
for b in convbench_old convbench; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$b -o run -- ./tools/$b la 50 $QS > $O/$b.log 2>&1 || { echo "$b prof failed"; tail -5 $O/$b.log; exit 1; }
  echo "== $b kernels"; python3 tools/kstats.py $(find $O/$b -name "*kernel_stats.csv" | head -1) | grep -E "la_" | head -12
done
