# fp16 vs bf16 kernel stats of the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof16 -o run -- python3 -u bench.py --steps 2 --warmup 1 --dtype fp16 --no-cpu-baseline --no-psnr --no-roofline --modes none > $O/p16.log 2>&1 || { tail -20 $O/p16.log; exit 1; }
python3 tools/kstats.py $(find $O/prof16 -name "*kernel_stats.csv" | head -1) > $O/k16.txt
head -40 $O/k16.txt | cut -c1-150
