# (Removed experiment: the DAC_CONV3_KP form measured slower and is no longer in the library)
# v3 wave-pair split-K (DAC_CONV3_KP=2: 8 waves as 2 x 2 x 2 of 64 x 64 tiles, each pair over half
# of every stage's k-steps) against the 4 x 2 waves of 32 x 64: op-level check + time, in-network
# interleaved A/B, and the fp16 parity tests with the new form.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/v3kp
mkdir -p $O
for dt in f16 bf16; do
  for kp in 1 2; do
    DAC_CONV3_KP=$kp CB_DTYPE=$dt timeout -k 10 120 tools/convbench 20 "L3 3x3" check -1 > $O/cb_${dt}_$kp.log 2>&1 || { echo CB FAILED; tail $O/cb_${dt}_$kp.log; exit 1; }
    echo "$dt kp=$kp"; cut -c1-120 $O/cb_${dt}_$kp.log
  done
done
for r in 1 2; do
  for kp in 1 2; do
    DAC_CONV3_KP=$kp CB_DTYPE=f16 timeout -k 10 120 tools/convbench 50 "L3 3x3" - -1 > $O/t_${kp}_$r.log 2>&1 || { echo T FAILED; tail $O/t_${kp}_$r.log; exit 1; }
    echo "time kp=$kp"; cut -c1-100 $O/t_${kp}_$r.log
  done
done
B="--steps 4 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none"
for r in 1 2 3; do
  for kp in 1 2; do
    DAC_CONV3_KP=$kp timeout -k 10 300 python -u bench.py $B > $O/n_${kp}_$r.log 2>&1 || { echo N FAILED; tail -5 $O/n_${kp}_$r.log; exit 1; }
    echo "net kp=$kp $(grep '^{' $O/n_${kp}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
DAC_CONV3_KP=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mixed.py tests/test_restore.py > $O/par.log 2>&1
e=$?; tail -3 $O/par.log; exit $e
