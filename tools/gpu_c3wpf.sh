# v5 next-segment L2 prefetch (DAC_C3W_PF) A/B on the 64->64 shapes: check, then interleaved timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DAC_C3W_PF=1 timeout -k 10 120 ./tools/convbench 2 "64->64" check > gpurun_out/c3wpf_check.log 2>&1 || { tail -20 gpurun_out/c3wpf_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/c3wpf_check.log) OK, $(grep -c FAIL gpurun_out/c3wpf_check.log) FAIL"
for p in 1 2; do
  for pf in 0 1; do
    echo "== pass $p PF=$pf"
    DAC_C3W_PF=$pf timeout -k 10 120 ./tools/convbench 50 "64->64" - -1,61 || exit 1
  done
done
