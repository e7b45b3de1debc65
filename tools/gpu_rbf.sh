set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rbf}
mkdir -p $O
timeout -k 10 300 tools/convbench rbf 20 > $O/rbf.txt 2>&1; rc=$?; cat $O/rbf.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_conv_kernels.py -m gpu -v --timeout 150 --timeout-method thread > $O/ck.log 2>&1; rc=$?; tail -3 $O/ck.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --modes none --lines none --no-cpu-baseline > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][0]); print(d['value'], d['psnr']['delta_db'], d['roofline']['kernel'], d['roofline']['frac']); [print(c) for c in d['roofline'].get('classes',[])]"
