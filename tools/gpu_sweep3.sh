# 3x3 conv configuration sweep (check + time) on a shape filter: tools/gpu_sweep3.sh <tag> <filter> <forces>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/convbench 2 "$2" check "$3" > gpurun_out/s3c_$1.log 2>&1 || { cat gpurun_out/s3c_$1.log; exit 1; }
grep -c FAIL gpurun_out/s3c_$1.log && grep FAIL gpurun_out/s3c_$1.log
timeout -k 10 200 ./tools/convbench 40 "$2" - "$3" > gpurun_out/s3t_$1.log 2>&1 || exit 1
cat gpurun_out/s3t_$1.log
