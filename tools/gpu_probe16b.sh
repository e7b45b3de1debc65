# fp16 precision probe, part 2 (mixed-fixture images): IEEE-half weight rounding emulated per UNet
# role on the fp32 path (DAC_EMU_FP16=1 + DAC_EMU_W role mask), and the real fp16 handle with the
# split-precision edge layers of the bf16 handles (DAC_F16_EDGES=1). tools/gpu_probe16b.sh <imgs>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/probe16b
mkdir -p $O
run() { timeout -k 10 120 python -u tools/prec_probe.py "$@" >> $O/probe.jsonl 2>> $O/err.log || { echo "probe $* failed"; tail -5 $O/err.log; exit 1; }; }
for i in ${1:-3 7}; do
  export PROBE_MIXED=$i
  DAC_F16_EDGES=1 run fp16 fp16 edges_fp16_img$i
  for m in 1 2 4 8 16 32 64 128 256; do
    DAC_EMU_FP16=1 DAC_EMU_W=$m run fp32 fp32 W${m}_img$i
  done
done
cat $O/probe.jsonl
