# Validate the tree (convbench checks, the -m gpu suite, smoke) and A/B two environment settings
# of this library: tools/gpu_val_env.sh <tag> "<env A>" "<env B>"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/val_$1
mkdir -p $O
timeout -k 10 300 ./tools/convbench 2 "" check > $O/cb_check.log 2>&1 || { tail -20 $O/cb_check.log; exit 1; }
echo "convbench check: $(grep -c OK $O/cb_check.log) OK, $(grep -c FAIL $O/cb_check.log) FAIL"; grep FAIL $O/cb_check.log | head
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep FAILED $O/tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke.log; }
bash tools/gpu_ab.sh $1 "$2" "$3" 3
