# Same-box A/B: HEAD engine (tools/ab) vs the restructured section (inner fork off), and the inner
# fork eagerly (DAC_NO_GRAPH=1) to localise a crash seen under graph capture.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/inner2
mkdir -p $O
DAC_SPLIT_INNER=1 DAC_NO_GRAPH=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --T 5 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline > $O/eager_inner.log 2>&1; echo "eager inner rc=$?"; grep '^{' $O/eager_inner.log | cut -c1-120
bash tools/gpu_ab.sh inner2 "DAC_LIB_PATH=$GRAFT_REPO_ROOT/tools/ab/libdaclip_hip_base.so" "DAC_SPLIT_INNER=0" 3
