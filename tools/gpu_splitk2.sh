# Wild-IR split-K sweep: 3x3 split count (DAC_SPLITK32) x 1x1 split on/off (DAC_SPLITK32_1X1).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/splitk2
mkdir -p $O
B="--model wild-ir --steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for cfg in "0 1" "2 1" "4 1" "8 1" "4 0" "2 0"; do
    set -- $cfg
    DAC_SPLITK32=$1 DAC_SPLITK32_1X1=$2 timeout -k 10 200 python -u bench.py $B > $O/w$1_$2.$rep.log 2>&1 || { echo W FAILED; tail $O/w$1_$2.$rep.log; exit 1; }
    echo "wild k3=$1 k1=$2 $(grep '^{' $O/w$1_$2.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
