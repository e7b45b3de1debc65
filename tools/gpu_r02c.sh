set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prec_probe.py fp32/bf16 bf16/bf16 > gpurun_out/prec_probe_c.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_r02c.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r02c.log
exit $rc
