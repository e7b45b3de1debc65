# LinearAttention x-tile swizzle that keeps each thread's channels: parity equal to the
# conflicted-layout build (libab/novslot.so), bank conflicts, A/B against it.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_numerics.sh la3 cur libab/novslot.so || exit 1
bash tools/gpu_ldsconf.sh la3 > gpurun_out/ldsc_la3.txt 2>&1 || { echo "ldsconf failed"; tail gpurun_out/ldsc_la3.txt; exit 1; }
grep -E "la_proj|la_apply" gpurun_out/ldsc_la3.txt | cut -c1-130
bash tools/gpu_ab.sh la3 "DAC_LIB_PATH=libab/novslot.so" "DAC_NONE=1" 3
