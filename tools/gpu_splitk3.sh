# Wild-IR split-K extent: 3x3 split at levels up to DAC_SPLITK_PX pixels per image.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/splitk3
mkdir -p $O
B="--model wild-ir --steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for px in 1024 4096 16384; do
    DAC_SPLITK_PX=$px timeout -k 10 200 python -u bench.py $B > $O/w$px.$rep.log 2>&1 || { echo W FAILED; tail $O/w$px.$rep.log; exit 1; }
    echo "wild px=$px $(grep '^{' $O/w$px.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
