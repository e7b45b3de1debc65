# Re-check of earlier tuning choices under the current kernels: each knob against the default,
# arms interleaved (round 6).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs
mkdir -p $O
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2 3; do
  for E in "X=0" "DAC_CONV3H=1" "DAC_UPH=2" "DAC_C3I_ST=4" "DAC_SPLIT_LVL=2" "DAC_CONV2_FORCE32=0"; do
    env $E timeout -k 10 200 python -u bench.py $B > $O/r.log 2>&1 || { echo "FAILED $E"; tail -5 $O/r.log; exit 1; }
    echo "$E $(grep '^{' $O/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
