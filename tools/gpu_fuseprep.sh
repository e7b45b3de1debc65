# sde_step writing the next step's UNet input (DAC_FUSE_PREP=1, default) against a separate
# unet_prep launch per step (=0): loop tests, equal dPSNR, interleaved bench pairs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fuseprep
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_restore.py tests/test_headline.py tests/test_mixed.py tests/test_variants.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for f in 0 1; do
    DAC_FUSE_PREP=$f timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --modes none --lines none --no-cpu-baseline --no-roofline $([ $r = 1 ] || echo --no-psnr) > $O/b${f}_$r.log 2>&1 || { echo "B$f FAILED"; tail -5 $O/b${f}_$r.log; exit 1; }
    grep '^{' $O/b${f}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d.get("psnr") or {}; print("fuse='$f'", d["value"], d["ms_per_step"], p.get("delta_db"), p.get("u8_mismatch"))'
  done
done
