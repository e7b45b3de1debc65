# 1x1 GEMM configuration sweep in convbench: tools/gpu_sweep1x1.sh <tag> <filter> <forces>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 ./tools/convbench 50 "$2" - "$3" > gpurun_out/sweep1x1_$1.log 2>&1
