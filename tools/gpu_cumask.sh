# CU-mask probe: the split section's two branches on disjoint CU halves (DAC_CUMASK 1/2/3) vs 0.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cumask
mkdir -p $O
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for m in 0 1 2 3; do
    DAC_CUMASK=$m timeout -k 10 200 python -u bench.py $B > $O/u$m.$rep.log 2>&1 || { echo U FAILED; tail $O/u$m.$rep.log; exit 1; }
    echo "univ cumask=$m $(grep '^{' $O/u$m.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
