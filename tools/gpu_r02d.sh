set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prec_probe.py fp32/bf16 bf16/bf16 > gpurun_out/prec_probe_c.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_r02c.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --kernel-id 999 --no-cpu-baseline --no-psnr > gpurun_out/shapeprof_r02.json 2> gpurun_out/shapeprof_r02.err || exit 1
timeout -k 10 300 tools/convbench 50 "L3 1x1" - 100,101,102,103,104,105,106,107,108,109,110 > gpurun_out/cb_l3_1x1.log 2>&1
