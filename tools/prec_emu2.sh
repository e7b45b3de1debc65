# Candidate precision fixes, emulated on the fp32 engine (engine.cpp DAC_EMU_* / DAC_WROUND).
cd $GRAFT_REPO_ROOT
for spec in "0x19a 0x1ff 0" "0x19b 0x1ff 0" "0x1ba 0x1ff 0" "0x1de 0x1ff 0" "0x1ff 0x1ff 1" "0x1ff 0 1" "0x4 0 1" "0x40 0 1"; do
  set -- $spec
  echo "W=$1 A=$2 WROUND=$3"
  DAC_EMU_W=$1 DAC_EMU_A=$2 DAC_WROUND=$3 timeout -k 10 120 python -u tools/prec_probe.py fp32/fp32 2>&1 | grep combo || exit 1
done
echo "real bf16, WROUND=1"
DAC_WROUND=1 timeout -k 10 120 python -u tools/prec_probe.py fp32/bf16 2>&1 | grep combo
