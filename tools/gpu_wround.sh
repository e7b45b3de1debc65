# Per-layer sum-keeping weight rounding (DAC_WROUND_KEY) on the fp16 restore fixture and the mixed
# batch: per-image dPSNR for the default, final_res_block.block1 only, final_res_block, and all layers.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wround
mkdir -p $O
i=0
for E in "DAC_WROUND=1" "DAC_WROUND_KEY=final_res_block.block1" "DAC_WROUND_KEY=final_res_block." "DAC_WROUND=2" "DAC_WROUND_KEY=final_res_block.block1 DAC_WROUND=1"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --modes ${MODES:-none} --lines mixed8 --no-cpu-baseline --no-roofline > $O/w$i.log 2>&1 || { echo "$E FAILED"; tail -5 $O/w$i.log; exit 1; }
  grep '^{' $O/w$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["psnr"]; l=d["lines"][0]["psnr"]; print("'"$E"'", "fixture", p["delta_db"], p["u8_mismatch"], "mixed", l["delta_db"], "max", l["max_abs_delta_db"], "mean", l["mean_delta_db"]); [print("   mode", m.get("dtype"), json.dumps(m.get("psnr"))[:300]) for m in d.get("modes", [])]'
done
