# Attention microbench + SQ counters: tools/gpu_attn.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/attn_bench.py 50 > gpurun_out/attn_$1.log 2>&1 || { cat gpurun_out/attn_$1.log; exit 1; }
cat gpurun_out/attn_$1.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/attnpmc_$1/p1 -o run -- python3 -u tools/attn_bench.py 2 > gpurun_out/attnpmc_$1_p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/attnpmc_$1/p2 -o run -- python3 -u tools/attn_bench.py 2 > gpurun_out/attnpmc_$1_p2.log 2>&1 || exit 1
python3 tools/pmc_kern.py gpurun_out/attnpmc_$1 > gpurun_out/attnpmc_$1.txt
cat gpurun_out/attnpmc_$1.txt
