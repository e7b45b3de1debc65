# Two library builds A/B (base = daclip_amd/libdaclip_hip_base.so via DAC_LIB_PATH): per-kernel
# rocprof times for a kernel pattern, then interleaved in-network pairs: tools/gpu_lib_ab.sh <pattern>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/libab
export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/da-clip_amd/daclip_amd/libdaclip_hip_base.so
for arm in base new base new; do
  if [ $arm = base ]; then export DAC_LIB_PATH=$BASE; else unset DAC_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/libab/p$arm -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-roofline --modes none --lines none > gpurun_out/libab/p$arm.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/libab/p$arm.log; exit 1; }
  echo "$arm"; grep -h "$1" gpurun_out/libab/p$arm/run_kernel_stats.csv | cut -d, -f1-4
  rm -rf gpurun_out/libab/p$arm
done
unset DAC_LIB_PATH
bash tools/gpu_ab.sh libab "DAC_LIB_PATH=$BASE" "DAC_NONE=1" 2
