# Which DAC_FOLD mask breaks fp16 batch invariance on the restoration fixture (bit 2 = the GEGLU fold, since removed from the engine).
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 0 29 2 31 1 8 24; do
  DAC_FOLD=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_restore.py -k "restore_matches_reference and fp16" > gpurun_out/s5_$m.log 2>&1
  echo "fold $m: $(tail -1 gpurun_out/s5_$m.log)"
done
