# L2 hit rate / clock / stall counters of the 32x32-level 1x1 GEMMs: in the network (eager bench,
# T=2) against the same shapes in convbench (back to back, L2-warm). tools/gpu_pmc32.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc32_${1:-a}
mkdir -p $O
export TMPDIR=/tmp
P1="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  DAC_NO_GRAPH=1 timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/net$i -o run -- \
    python3 -u bench.py --steps 1 --warmup 0 --T 2 --no-cpu-baseline --no-roofline --no-psnr --modes none --lines none \
    > $O/net$i.log 2>&1 || { echo "net pass $i failed"; tail -5 $O/net$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/cb$i -o run -- ./tools/convbench 5 "L3 1x1" - > $O/cb$i.log 2>&1 || { echo "cb pass $i failed"; tail -5 $O/cb$i.log; exit 1; }
done
python3 tools/pmc32.py $O > $O/summary.txt
cat $O/summary.txt
