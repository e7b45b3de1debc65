# In-network sweep of the 1x1 configuration used at the 32x32 level (DAC_CONV2_FORCE32).
cd $GRAFT_REPO_ROOT
for f in 0 11 12 13 8; do
  echo "force32=$f $(DAC_CONV2_FORCE32=$f timeout -k 10 120 python3 bench.py --steps 3 --no-cpu-baseline --no-psnr --no-roofline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
