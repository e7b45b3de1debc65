# conv3r timing A/B: convbench c3r from two builds (tools/convbench_old vs tools/convbench), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3rab
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 tools/convbench_old c3r 30 > $O/old$r.txt 2>&1 || { echo OLD FAILED; tail $O/old$r.txt; exit 1; }
  timeout -k 10 120 tools/convbench c3r 30 > $O/new$r.txt 2>&1 || { echo NEW FAILED; tail $O/new$r.txt; exit 1; }
  echo "== old $r"; cat $O/old$r.txt; echo "== new $r"; cat $O/new$r.txt
done
