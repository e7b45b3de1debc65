# fp16 precision probe, part 3: which final_res_block weights carry the low-light image's fp16
# error (IEEE-half weight rounding of final_res_block emulated on the fp32 path, one sub-module
# kept fp32 at a time with DAC_EMU_WSKIP). tools/gpu_probe16c.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/probe16c
mkdir -p $O
export PROBE_MIXED=3
run() { timeout -k 10 120 python -u tools/prec_probe.py "$@" >> $O/probe.jsonl 2>> $O/err.log || { echo "probe $* failed"; tail -5 $O/err.log; exit 1; }; }
DAC_EMU_FP16=1 DAC_EMU_W=64 run fp32 fp32 W64_all
for s in mlp block1 block2 res_conv; do
  DAC_EMU_FP16=1 DAC_EMU_W=64 DAC_EMU_WSKIP=$s run fp32 fp32 W64_skip_$s
done
DAC_EMU_FP16=1 DAC_EMU_W=64 DAC_EMU_WSKIP=block1,block2,res_conv run fp32 fp32 W64_only_mlp
cat $O/probe.jsonl
