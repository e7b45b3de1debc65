# v3 ring depth: 64-byte chunks in a 3 / 4-stage ring (DAC_V3_ST) against the 128-byte double
# buffer: op-level check + timing (fp16, 32^2 shapes), then in-network A/B/C.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/v3st
mkdir -p $O
export TMPDIR=/tmp
for st in 0 3 4; do
  DAC_V3_ST=$st CB_DTYPE=f16 timeout -k 10 120 tools/convbench 20 "L3 3x3" check -1 > $O/cb_$st.log 2>&1 || { echo "CB st=$st FAILED"; tail $O/cb_$st.log; exit 1; }
  echo "st=$st: $(grep -E '512->512|768->512|256->512' $O/cb_$st.log | cut -c1-120 | tr '\n' ' ')"
done
bash tools/gpu_ab3.sh v3st "DAC_V3_ST=0" "DAC_V3_ST=3" "DAC_V3_ST=4" 3
