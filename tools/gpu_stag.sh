# v4 first-round stagger sweep (DAC_V4_STAGGER) on the v4 3x3 shapes: tools/gpu_stag.sh "<values>"
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in $1; do
  echo "== DAC_V4_STAGGER=$v"
  for s in "L0 3x3 128->64" "L1 3x3 128->128" "L1 3x3 192->128" "L2 3x3 256->256"; do
    DAC_V4_STAGGER=$v timeout -k 10 60 ./tools/convbench 100 "$s" || exit 1
  done
done
DAC_V4_STAGGER=8 timeout -k 10 60 ./tools/convbench 2 "L0 3x3 128->64" check || exit 1
