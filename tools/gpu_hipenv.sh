# HIP runtime knobs against the default: graph packet capture, hardware queues per process.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hipenv
mkdir -p $O
B="--steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline"
for rep in 1 2; do
  for E in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "GPU_MAX_HW_QUEUES=8"; do
    env $E timeout -k 10 200 python -u bench.py $B > $O/r.log 2>&1 || { echo "FAILED $E"; tail -5 $O/r.log; exit 1; }
    echo "$E $(grep '^{' $O/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
