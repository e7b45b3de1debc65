# Weight-rounding sensitivity per UNet role (DAC_EMU_W, engine.cpp), fp32 engine, headline restore.
cd $GRAFT_REPO_ROOT
for w in 1 2 4 8 16 32 64 128 256 0x1dd 0x1fd; do
  echo "W=$w A=0"
  DAC_EMU_W=$w DAC_EMU_A=0 timeout -k 10 120 python -u tools/prec_probe.py fp32/fp32 2>&1 | grep combo || exit 1
done
