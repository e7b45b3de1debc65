# conv3r op-level check + timing sweep (stagger delay 70..79 = (k-70)*8 x 64 cycles; 33 = v5).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c3r}
mkdir -p $O
timeout -k 10 180 tools/convbench 1 "64->64" check -1,33 > $O/cb_check.txt 2>&1 || { echo CHECK FAILED rc=$?; tail -20 $O/cb_check.txt; exit 1; }
cat $O/cb_check.txt
timeout -k 10 300 tools/convbench 50 "3x3 64->64" - 33,70,72,74,75,76,77,78,33,70,74,76 > $O/cb_time.txt 2>&1 || { echo TIME FAILED; tail -20 $O/cb_time.txt; exit 1; }
cat $O/cb_time.txt
