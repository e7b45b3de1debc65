# Per-shape eager conv profile (tools/conv_profile.py, fp16 bench batch) under N env settings.
# tools/gpu_cprof_arms.sh <tag> "<filter regex>" "<env 1>" "<env 2>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; FILT=$2; shift 2
O=gpurun_out/cpa_$TAG
mkdir -p $O
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u tools/conv_profile.py --dtype fp16 > $O/c$i.txt 2>&1 || { echo "arm $i FAILED"; tail -5 $O/c$i.txt; exit 1; }
  echo "== arm $i ($E)"; grep -E "$FILT" $O/c$i.txt
done
