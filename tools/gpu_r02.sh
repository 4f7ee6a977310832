#!/bin/bash
# Round-2 GPU check: selected tests (fail fast), then bench N=1 and the world-1 DDP
# (segmented-overlap) bench, then a kernel trace of the DDP bench for the timeline.
#   gpurun -- bash tools/gpu_r02.sh <tag> "<pytest -k expr>" [trace]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
tag=${1:-x}
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "$2" --timeout 150 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t_$tag.log | tail -30
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b1_$tag.json 2> gpurun_out/b1_$tag.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/b1_$tag.json; tail -3 gpurun_out/b1_$tag.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --force-ddp > gpurun_out/bddp_$tag.json 2> gpurun_out/bddp_$tag.err; rc=$?
echo "bench ddp rc=$rc"; cat gpurun_out/bddp_$tag.json; tail -3 gpurun_out/bddp_$tag.err
[ $rc -eq 0 ] || exit $rc
if [ "$3" = "trace" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr_$tag -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --force-ddp --steps 3 --warmup 2 > $R/gpurun_out/tr_$tag.log 2>&1; rc=$?
  echo "trace rc=$rc"
fi
exit $rc
