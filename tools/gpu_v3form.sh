# v3 (512-wide 32x32 3x3 convs) wave-layout probe: DAC_V3_FORM 0 (8 waves 4x2, default), 1 (4 waves
# 2x2 of 64x64), 2 (8 waves 2x4 of 64x32), op-level (convbench, fp16) and in the network.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/v3form
mkdir -p $O
for f in 0 1 2; do
  DAC_V3_FORM=$f CB_DTYPE=f16 timeout -k 10 120 tools/convbench 20 "L3 3x3" check -1 > $O/cb$f.log 2>&1 || { echo CB FAILED; tail $O/cb$f.log; exit 1; }
  echo "form $f"; cat $O/cb$f.log | cut -c1-160
done
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for f in 0 1 2; do
    DAC_V3_FORM=$f timeout -k 10 200 python -u bench.py $B > $O/u$f.$rep.log 2>&1 || { echo U FAILED; tail $O/u$f.$rep.log; exit 1; }
    echo "univ form=$f $(grep '^{' $O/u$f.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
