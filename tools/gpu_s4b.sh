#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; cd $R; OUT=$R/gpurun_out/s4b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "graphed_step" > $OUT/t.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/t.log | head -20; tail -3 $OUT/t.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/t.log; tail -1 $OUT/t.log
