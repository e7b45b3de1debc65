# Norm folds A/B: alternating bench runs and a rocprof kernel-stats run of each arm.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s3
mkdir -p $O
for arm in off on off on; do
  if [ $arm = off ]; then export DAC_NO_LN_FOLD=1 DAC_NO_GN_IN_LN=1; else export DAC_NO_LN_FOLD=0 DAC_NO_GN_IN_LN=0; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none > $O/b_$arm.log 2>&1 || { tail -20 $O/b_$arm.log; exit 1; }
  echo "$arm $(grep '^{' $O/b_$arm.log | cut -c100-175)"
done
for arm in off on; do
  if [ $arm = off ]; then export DAC_NO_LN_FOLD=1 DAC_NO_GN_IN_LN=1; else export DAC_NO_LN_FOLD=0 DAC_NO_GN_IN_LN=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none > $O/p_$arm.log 2>&1 || { tail -20 $O/p_$arm.log; exit 1; }
  python3 tools/kstats.py $(find $O/prof_$arm -name "*kernel_stats.csv" | head -1) > $O/k_$arm.txt
done
head -45 $O/k_on.txt | cut -c1-150
echo ====
head -45 $O/k_off.txt | cut -c1-150
