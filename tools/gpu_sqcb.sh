# SQ stall / issue counters of convbench launches (one shape filter, listed forces):
# tools/gpu_sqcb.sh <tag> <shape filter> <forces> <kernel regex>
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/sqc_$1
mkdir -p $D
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
P3="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$4" --output-format csv -d $D/p$i -o run -- ./tools/convbench 5 "$2" - $3 > $D/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $D/log$i.txt; exit 1; }
done
python3 tools/sqpmc.py $D
