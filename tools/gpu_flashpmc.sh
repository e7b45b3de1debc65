# flash_kv in the network vs alone: SQ stall and L2 hit counters of the
# SpatialTransformer attention kernel in the bench workload (eager launches, T = 2) and in
# tools/attn_bench.py at the split section's batch (4) with the engine's prescaled-q variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/flashpmc
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  DAC_NO_GRAPH=1 timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/net$i -o run -- python3 -u bench.py --steps 1 --warmup 0 --T 2 --no-cpu-baseline --no-roofline --no-psnr --modes none --lines none > $O/net$i.log 2>&1 || { echo "net pass $i failed"; tail -5 $O/net$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/iso$i -o run -- python3 -u tools/attn_bench.py 20 4 8 > $O/iso$i.log 2>&1 || { echo "iso pass $i failed"; tail -5 $O/iso$i.log; exit 1; }
done
python3 tools/flashpmc.py $O | tee $O/summary.txt
