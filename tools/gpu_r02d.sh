#!/bin/bash
# all GPU tests, bench with kernel trace, dW split sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|^E |FAILED|Error" gpurun_out/t_$tag.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b1_$tag.json 2> gpurun_out/b1_$tag.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/b1_$tag.json
[ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr_$tag -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 5 --warmup 3 > $R/gpurun_out/tr_$tag.log 2>&1 ); rc=$?
echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "$2" = "sweep" ]; then
  timeout -k 10 400 python tools/dw_sweep.py > gpurun_out/dw_sweep_$tag.txt 2>&1; rc=$?
  echo "sweep rc=$rc"; cat gpurun_out/dw_sweep_$tag.txt
fi
exit $rc
