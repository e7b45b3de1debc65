# (Removed experiment: no gain; DESIGN.md §9. The two-tile form is not in conv_edge.hip.)
# conv7 (init conv) variants against libab/base.so / libab/convbench_base:
# against libab/base.so / libab/convbench_base: op-level check + time, in-graph times, equal PSNR.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c7ct
mkdir -p $O
for r in 1 2; do
  for arm in base new; do
    CB=tools/convbench; [ $arm = base ] && CB=libab/convbench_base
    CB_DTYPE=f16 timeout -k 10 120 $CB 50 "init" check -1 > $O/cb_${arm}_$r.log 2>&1 || { echo CB FAILED; tail $O/cb_${arm}_$r.log; exit 1; }
    echo "$arm"; cut -c1-150 $O/cb_${arm}_$r.log
  done
done
bash tools/gpu_rfcmp.sh c7ct libab/base.so 3 conv7 || exit 1
for arm in A B; do
  E=""; [ $arm = A ] && E="DAC_LIB_PATH=libab/base.so"
  env $E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --modes none --lines mixed8 --no-cpu-baseline --no-roofline > $O/p$arm.log 2>&1 || { echo P FAILED; tail -5 $O/p$arm.log; exit 1; }
  grep '^{' $O/p$arm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$arm'", d["value"], d["psnr"]["delta_db"], d["psnr"]["u8_mismatch"], d["lines"][0]["psnr"]["delta_db"])'
done
