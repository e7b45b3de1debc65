# v3 LDS swizzle change: op-level check (every convbench shape, fp16 and bf16), the bank-conflict
# counters of the 512-channel 32² conv, then the in-network A/B against libab/base.so (old swizzle).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/swz
mkdir -p $O
export TMPDIR=/tmp
for dt in f16 bf16; do
  CB_DTYPE=$dt timeout -k 10 180 tools/convbench 3 "" check -1 > $O/cb_$dt.log 2>&1 || { echo "CB $dt FAILED"; tail $O/cb_$dt.log; exit 1; }
  echo "convbench $dt: $(grep -c . $O/cb_$dt.log) lines, $(grep -ci fail $O/cb_$dt.log) fail"
done
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
CB_DTYPE=f16 timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- ./tools/convbench 5 "L3 3x3" - -1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python3 tools/sqpmc.py $O > $O/sq.txt 2>&1; head -30 $O/sq.txt | cut -c1-200
bash tools/gpu_ab.sh swz "DAC_LIB_PATH=libab/base.so" "DAC_NONE=1" 3
