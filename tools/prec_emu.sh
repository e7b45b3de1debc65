# Precision probe: fp32 engine with selected UNet roles rounded to bf16 (DAC_EMU_W / DAC_EMU_A,
# engine.cpp), headline fixture restore; one process per setting (the masks are read once).
cd $GRAFT_REPO_ROOT
for spec in "0x1ff 0" "0 0x1ff" "0x1ff 0x1ff" "0 1" "0 2" "0 4" "0 8" "0 16" "0 32" "0 64" "0 128" "0x1ff 0x1df"; do
  set -- $spec
  echo "W=$1 A=$2"
  DAC_EMU_W=$1 DAC_EMU_A=$2 timeout -k 10 120 python -u tools/prec_probe.py fp32/fp32 2>&1 | grep combo || exit 1
done
