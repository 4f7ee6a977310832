#!/bin/bash
# full GPU suite, bench, steady-state kernel summary
set -u
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/s3j
OUT=$R/gpurun_out/s3j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { grep -E "^E |FAILED" $OUT/t.log | head -20; tail -3 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 40 > $OUT/b.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['ms_per_step'], d['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 5 --warmup 3 > $OUT/tr.log 2>&1 || exit 1
python3 $R/tools/step_summary.py $OUT/tr/run_results.db 5 > $OUT/summary.txt && head -3 $OUT/summary.txt && grep -E "adam|ln_bwd|reduce_multi" $OUT/summary.txt
