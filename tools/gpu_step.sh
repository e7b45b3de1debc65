# One GPU iteration: selected gpu tests (assertion failures do not stop the run; a timeout,
# abort or crash does) and then a short bench line.
#   tools/gpu_step.sh <tag> "<pytest args>" [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
if [ -n "$2" ]; then
  eval timeout -k 10 900 python -u -m pytest $2 -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?
  tail -25 gpurun_out/t_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST rc=$rc: stopping"; exit $rc; fi
fi
if [ "$3" != "none" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $3 > gpurun_out/b_$TAG.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/b_$TAG.log; exit 1; }
  grep '^{' gpurun_out/b_$TAG.log
fi
