# fp16 parity of alternative builds (DAC_LIB_PATH): the headline restore fixture's dPSNR and the
# mixed8 batch's per-image dPSNR, one bench run per build. tools/gpu_numerics.sh <tag> <lib>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/num_$1
mkdir -p $O
shift
for lib in "$@"; do
  n=$(basename $lib .so)
  env $([ "$lib" = cur ] || echo DAC_LIB_PATH=$lib) timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --lines mixed8 --modes none --no-cpu-baseline --no-roofline > $O/$n.log 2>&1 || { echo "$n FAILED"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); l=d["lines"][0]; print("'$n'", d["value"], "headline dPSNR", d["psnr"]["delta_db"], "mixed8", l["psnr"]["delta_db"])'
done
