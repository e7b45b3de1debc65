# Norm folds A/B: op checks, bench runs per DAC_FOLD mask, rocprof kernel stats of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 180 ./tools/convbench lnf 10 && timeout -k 10 120 ./tools/convbench gns || exit 1
for m in 0 25 1 4 8 24 29 0 25; do
  DAC_FOLD=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/b_$m.log 2>&1 || { tail -20 $O/b_$m.log; exit 1; }
  echo "fold $m $(grep '^{' $O/b_$m.log | cut -c100-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/k.txt
grep -E "ln_kernel|conv2_kernel|gn_" $O/k.txt | cut -c1-150
