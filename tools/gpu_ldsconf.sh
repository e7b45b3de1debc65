# LDS bank conflicts and instruction mix of every kernel in the bench (eager replay, T=2), one
# SQ counter pass: tools/gpu_ldsconf.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/ldsc_$1
mkdir -p $D
export TMPDIR=/tmp DAC_NO_GRAPH=1
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d $D/p2 -o run -- python3 -u bench.py --steps 1 --warmup 0 --T 2 --no-cpu-baseline --no-roofline --no-psnr --modes none --lines none > $D/log.txt 2>&1 || { echo "pass failed"; tail -5 $D/log.txt; exit 1; }
python3 tools/ldsconf.py $D
