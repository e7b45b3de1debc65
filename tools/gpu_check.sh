# Full GPU validation of the current tree: LN-fold op check, the -m gpu suite, smoke(), and the
# default bench line. tools/gpu_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chk_$1
O=gpurun_out/chk_$1
timeout -k 10 120 ./tools/convbench lnf 5 > $O/lnf.log 2>&1; echo "lnf rc=$?"; head -3 $O/lnf.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; grep FAILED $O/tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 - $O/bench.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read())
print("main", d["dtype"], d["value"], d["ms_per_step"], "psnr", (d.get("psnr") or {}).get("delta_db"), "frac", (d.get("roofline") or {}).get("frac"))
for m in d.get("modes", []): print("mode", m["dtype"], m["value"], (m.get("psnr") or {}).get("delta_db"))
for m in d.get("lines", []): print("line", m["line"], m["dtype"], m["value"], m["ms_per_step"], (m.get("psnr") or {}).get("delta_db"), m.get("wall_s"))
PY
