#!/bin/bash
# BN finalize batched loads + grouped-dW split divisor variants
set -u
R=$GRAFT_REPO_ROOT; cd $R; OUT=$R/gpurun_out/s4c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or conv or module or graph" > $OUT/t.log 2>&1 || { grep -E "^E |FAILED" $OUT/t.log | head -20; tail -3 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in def def; do
  if [ $v = def ]; then unset LASR_DW_GROUP_SPLIT_DIV; else export LASR_DW_GROUP_SPLIT_DIV=$v; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 60 > $OUT/b_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));print('$v', d['ms_per_step'], d['value'])"
done
unset LASR_DW_GROUP_SPLIT_DIV
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 5 --warmup 3 > $OUT/tr.log 2>&1 || exit 1
python3 $R/tools/step_summary.py $OUT/tr/run_results.db 5 > $OUT/summary.txt && head -3 $OUT/summary.txt && grep -E "bn_|reduce_multi|dw_group" $OUT/summary.txt
