# Isolated timing of the 32x32-level 1x1 GEMM shapes over every conv2 configuration (convbench).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c2sweep}
mkdir -p $O
timeout -k 10 240 tools/convbench 50 "L3 1x1" - -1,101,102,103,104,105,106,107,108,110,111,112,113,114,115,116 > $O/sweep.txt 2>&1 || { echo SWEEP FAILED; tail -20 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
timeout -k 10 240 tools/convbench 50 "L3 3x3" - > $O/sweep3.txt 2>&1 || { echo SWEEP3 FAILED; exit 1; }
cat $O/sweep3.txt
