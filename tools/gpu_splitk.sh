# Split-K A/B at the 32x32 level (DAC_SPLITK32): Wild-IR (default 4 vs 0) and universal-IR
# (default 0 vs 2 / 4), interleaved; plus the Wild-IR / invariance GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/splitk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wild.py tests/test_hip_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "wild or invariance or batch" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for k in 0 4; do
    DAC_SPLITK32=$k timeout -k 10 200 python -u bench.py --model wild-ir $B > $O/w$k.$rep.log 2>&1 || { echo W FAILED; tail $O/w$k.$rep.log; exit 1; }
    echo "wild k=$k $(grep '^{' $O/w$k.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
  for k in 0 2; do
    DAC_SPLITK32=$k timeout -k 10 200 python -u bench.py $B > $O/u$k.$rep.log 2>&1 || { echo U FAILED; tail $O/u$k.$rep.log; exit 1; }
    echo "univ k=$k $(grep '^{' $O/u$k.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
