# Which final-stage weights need more than bf16 (WROUND=1 everywhere else), emulated on fp32.
cd $GRAFT_REPO_ROOT
for skip in "final_res_block.res_conv" "final_res_block.block1" "final_res_block.block2" "final_conv" "init_conv" \
            "final_res_block.res_conv,final_conv,init_conv" "final_res_block,final_conv,init_conv" \
            "final_res_block,final_conv" "final_res_block.res_conv,final_conv"; do
  echo "skip=$skip"
  DAC_EMU_W=0x1ff DAC_EMU_A=0x1ff DAC_WROUND=1 DAC_EMU_WSKIP=$skip timeout -k 10 120 python -u tools/prec_probe.py fp32/fp32 2>&1 | grep combo || exit 1
done
