# Full measurement cycle for the committed profiles: PMC traffic passes -> profiles/pmc_traffic.json,
# then GPU tests, smoke, the default bench line (reads that JSON), and a rocprofv3 stats run.
# tools/gpu_profiles.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r}
mkdir -p gpurun_out
bash tools/pmc_bench.sh $TAG || { echo PMC FAILED; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_$TAG profiles/pmc_traffic.json > gpurun_out/pmc_traffic_$TAG.txt || exit 1
mkdir -p gpurun_out/profiles_out && cp profiles/pmc_traffic.json gpurun_out/profiles_out/
bash tools/gpu_cycle.sh $TAG
