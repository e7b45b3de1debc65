# N-major XCD tile order (DAC_NMAJOR bits: 1 v3, 2 1x1 GEMMs, 4 v4) vs the default, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/nmajor
mkdir -p $O
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2 3; do
  for m in 0 1 2 7; do
    DAC_NMAJOR=$m timeout -k 10 200 python -u bench.py $B > $O/u$m.$rep.log 2>&1 || { echo "FAILED $m"; tail -5 $O/u$m.$rep.log; exit 1; }
    echo "nmajor=$m $(grep '^{' $O/u$m.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
