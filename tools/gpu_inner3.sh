# Where does the graph-captured inner fork crash? (T, B) sweep, each its own process.
cd $GRAFT_REPO_ROOT
O=gpurun_out/inner3
mkdir -p $O
for cfg in "1 4" "1 8" "2 8" "5 8"; do
  set -- $cfg
  DAC_SPLIT_INNER=1 AMD_LOG_LEVEL=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --T $1 --batch $2 --modes none --lines none --no-cpu-baseline --no-psnr --no-roofline > $O/t$1b$2.log 2>&1
  echo "T=$1 B=$2 rc=$? $(grep '^{' $O/t$1b$2.log | cut -c60-110)"
done
