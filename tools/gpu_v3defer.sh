# (Removed experiment, measured within noise; DESIGN.md §9. The deferral is no longer in conv_impl.h.)
# v3 with the last fragment group's MFMAs deferred past the next stage barrier, against libab/base.so
# (the previous source): op-level check, in-graph per-symbol times, and equal restore PSNR deltas.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/v3defer
mkdir -p $O
for dt in f16 bf16; do
  CB_DTYPE=$dt timeout -k 10 120 tools/convbench 20 "L3 3x3" check -1 > $O/cb_$dt.log 2>&1 || { echo CB FAILED; tail $O/cb_$dt.log; exit 1; }
  echo "$dt"; cut -c1-130 $O/cb_$dt.log
done
bash tools/gpu_rfcmp.sh v3defer libab/base.so 3 conv3_kernel || exit 1
for arm in A B; do
  E=""; [ $arm = A ] && E="DAC_LIB_PATH=libab/base.so"
  env $E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --modes none --lines mixed8 --no-cpu-baseline --no-roofline > $O/p$arm.log 2>&1 || { echo P FAILED; tail -5 $O/p$arm.log; exit 1; }
  grep '^{' $O/p$arm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$arm'", d["value"], json.dumps(d.get("psnr")), json.dumps([l.get("psnr") for l in d.get("lines", [])])[:600])'
done
