set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_s3.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests_s3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_s3.json; tail -3 gpurun_out/bench_s3.err
