# convbench A/B on the 3x3 shapes: correctness of the listed forces, two interleaved timing
# passes, the LN-fold / GroupNorm-in-A check. tools/gpu_cb.sh <tag> <forces> [shape filter]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
F=${3:-3x3}
timeout -k 10 200 ./tools/convbench 2 "$F" check $2 > gpurun_out/cb_$1_check.log 2>&1 || { tail -20 gpurun_out/cb_$1_check.log; exit 1; }
echo "check: $(grep -c OK gpurun_out/cb_$1_check.log) OK, $(grep -c FAIL gpurun_out/cb_$1_check.log) FAIL"
grep FAIL gpurun_out/cb_$1_check.log | head
for p in 1 2; do
  echo "== pass $p"
  timeout -k 10 200 ./tools/convbench 50 "$F" - $2 || exit 1
done
timeout -k 10 120 ./tools/convbench lnf 5 || exit 1
