# Precision attribution on the restoration fixture (tools/prec_probe.py), one process per config.
#   tools/gpu_prec.sh "<label>:<emu_w>:<emu_a>:<enc>:<unet>[:fp16]" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in "$@"; do
  IFS=: read label w a e u h <<< "$c"
  env ${w:+DAC_EMU_W=$w} ${a:+DAC_EMU_A=$a} ${h:+DAC_EMU_FP16=1} PROBE_SAVE=1 timeout -k 10 120 python -u tools/prec_probe.py ${e:-fp32} ${u:-fp32} $label \
    >> gpurun_out/prec.jsonl 2> gpurun_out/prec_err.log || { echo "FAILED: $c"; tail -5 gpurun_out/prec_err.log; exit 1; }
done
cat gpurun_out/prec.jsonl
