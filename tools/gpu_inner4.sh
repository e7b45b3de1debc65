# Inner fork effect measured eagerly (DAC_NO_GRAPH=1, T=20), arms interleaved; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/inner4
mkdir -p $O
for rep in 1 2 3; do
  for v in 0 1; do
    DAC_NO_GRAPH=1 DAC_SPLIT_INNER=$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --T 20 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline > $O/e$v.$rep.log 2>&1 || { echo "FAILED inner=$v"; exit 1; }
    echo "eager inner=$v $(grep '^{' $O/e$v.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
