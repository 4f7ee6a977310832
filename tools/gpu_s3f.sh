#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CASES=("(prod)" "dd bias" "dX dd (nn)" "dd res" "fc2 fwd" "dX fc1 (nn" "qkv")
for v in 0 1; do
  echo "=== LASR_GEMM_DIRECT=$v"
  LASR_GEMM_DIRECT=$v timeout -k 10 200 python -u tools/gemm_graph_bench.py --cold "${CASES[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in 0 1 0 1; do LASR_GEMM_DIRECT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/d_$v.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/d_$v.json'));print('direct', $v, d['ms_per_step'])"; done
