# fp16 precision probe on one mixed-fixture image (PROBE_MIXED=<i>): the fp32 UNet with IEEE-half
# rounding emulated per role (DAC_EMU_FP16=1, DAC_EMU_W / DAC_EMU_A role masks, engine.cpp), and
# the real fp16 handle. tools/gpu_probe16.sh <image index>
set -o pipefail
cd $GRAFT_REPO_ROOT
export PROBE_MIXED=${1:-3} DAC_EMU_FP16=1
O=gpurun_out/probe16_$PROBE_MIXED
mkdir -p $O
run() { timeout -k 10 120 python -u tools/prec_probe.py "$@" >> $O/probe.jsonl 2>> $O/err.log || { echo "probe $* failed"; tail -5 $O/err.log; exit 1; }; }
run fp16 fp16 real_fp16
run fp32 fp32 fp32
run fp16 fp32 enc16
DAC_EMU_W=511 run fp32 fp32 W511
DAC_EMU_A=511 DAC_EMU_W=511 run fp32 fp32 AW511
for m in 511 1 2 4 8 16 32 64 128 256; do
  DAC_EMU_A=$m run fp32 fp32 A$m
done
cat $O/probe.jsonl
