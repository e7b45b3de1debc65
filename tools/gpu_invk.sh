set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/invk
export TMPDIR=/tmp
for B in 8 16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/invk/p$B -o run -- python3 -u tools/inv_kernels.py $B > gpurun_out/invk/p$B.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/invk/p$B.log; exit 1; }
  cut -d, -f1-2 gpurun_out/invk/p$B/run_kernel_stats.csv | sort > gpurun_out/invk/k$B.txt
done
diff gpurun_out/invk/k8.txt gpurun_out/invk/k16.txt || true
