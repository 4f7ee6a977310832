# GPU-box check: new-op tests first (fail fast), then the whole -m gpu suite, then a bench line.
#   gpurun -- bash tools/gpu_run.sh <tag> [pytest -k expr for the first step]
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-x}
if [ -n "$2" ]; then
  timeout -k 10 150 python -u -m pytest tests -m gpu -x -q -k "$2" --timeout 120 --timeout-method thread > gpurun_out/first_$tag.log 2>&1; rc=$?
  echo "first rc=$rc"; tail -15 gpurun_out/first_$tag.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests_$tag.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$tag.json; tail -3 gpurun_out/bench_$tag.err
