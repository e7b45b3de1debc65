# In-graph per-symbol launch times (bench roofline stamps) of two builds, interleaved:
# tools/gpu_rfcmp.sh <tag> <libA> [reps] [comma-separated symbol substrings]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rf_$1
mkdir -p $O
F=${4:-conv3_kernel,rbfuse,conv3i}
for r in $(seq 1 ${3:-2}); do
  for arm in A B; do
    E=""; [ $arm = A ] && E="DAC_LIB_PATH=$2"
    env $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --modes none --lines none --no-cpu-baseline --no-psnr > $O/$arm$r.log 2>&1 || { echo "$arm$r FAILED"; tail -5 $O/$arm$r.log; exit 1; }
    grep '^{' $O/$arm$r.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); r=d["roofline"]; keys=sys.argv[1].split(",")
print("'$arm$r'", d["value"], "conv_busy", r.get("conv_busy_ms_per_restore"), " ".join("%s=%.1f" % (s["symbol"][13:44], s["mean_us"]) for s in r["symbols"] if any(k in s["symbol"] for k in keys)))' "$F"
  done
done
