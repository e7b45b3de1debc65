# la_apply<64> blocks per CU (DAC_LA_PERCU): its 144 registers leave 3 waves per SIMD, i.e. 3
# resident 4-wave blocks per CU, while the grid was sized for 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lapercu
mkdir -p $O
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2 3; do
  for k in 4 3 6; do
    DAC_LA_PERCU=$k timeout -k 10 200 python -u bench.py $B > $O/u$k.$rep.log 2>&1 || { echo U FAILED; tail $O/u$k.$rep.log; exit 1; }
    echo "univ percu=$k $(grep '^{' $O/u$k.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
