#!/bin/bash
# A/B of the grouped weight-gradient tiles (LASR_DW_WIDE): tests under each variant, then the
# bench line of each.  Output under gpurun_out/$1/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${1:-dwwide}; mkdir -p "$OUT"; cd "$R"
V1="LASR_DW_WIDE=3"
V2="LASR_DW_WIDE=2 LASR_DW_GROUP_SPLIT_DIV=4,1"
for v in "$V1" "$V2"; do
  tag=$(echo "$v" | tr ' =,' '___')
  env $v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "dw_group or parity_bf16 or config2_full_model_bf16" > "$OUT/tests_$tag.log" 2>&1 || exit 1
done
for v in "LASR_DW_WIDE=2" "$V1" "$V2"; do
  tag=$(echo "$v" | tr ' =,' '___')
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || exit 1
done
echo done
