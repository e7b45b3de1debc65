# One UNet step of the bench graph in dispatch order (rocprofv3 kernel trace + tools/trace_step.py),
# under an optional env setting. tools/gpu_trace.sh <tag> ["<env>"]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/trace_$1
mkdir -p $O
export TMPDIR=/tmp
env ${2:-X=1} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 -u bench.py --steps 1 --warmup 1 --T 10 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/run.log 2>&1 || { echo "FAILED"; tail -5 $O/run.log; exit 1; }
python3 tools/trace_step.py $(find $O/p -name "*kernel_trace.csv" | head -1) > $O/step.txt
cat $O/step.txt
