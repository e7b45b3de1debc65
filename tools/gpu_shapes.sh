# Per-shape conv timing (eager replay with events per launch): tools/gpu_shapes.sh <tag> [dtype]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conv_profile.py --dtype ${2:-bf16} > gpurun_out/shapes_$1.log 2>&1
