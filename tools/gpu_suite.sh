#!/bin/bash
# round-end check: full GPU suite + smoke()
set -u
R=$GRAFT_REPO_ROOT; cd $R; OUT=$R/gpurun_out/final; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "^E |FAILED" $OUT/t.log | head -20; tail -3 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
