# v4 A-halo L2 prefetch (FL bit 12 / 13, convbench forces 54 / 55) against the default buffer
# form (48): correctness on every 3x3 shape, then two interleaved timing passes; LN-fold check.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 ./tools/convbench 2 "3x3" check 48,54,55 > gpurun_out/pf_check.log 2>&1 || { tail -20 gpurun_out/pf_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/pf_check.log) OK, $(grep -c FAIL gpurun_out/pf_check.log) FAIL"
grep FAIL gpurun_out/pf_check.log | head
for p in 1 2; do
  echo "== pass $p"
  timeout -k 10 200 ./tools/convbench 50 "3x3" - 48,54,55 | grep -v "f-1 \|f48 .*variant 2[1-4]" || exit 1
done
timeout -k 10 120 ./tools/convbench lnf 5 || exit 1
