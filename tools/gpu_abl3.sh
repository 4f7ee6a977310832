#!/bin/bash
# GEMM ablation (LASR_EXP variants in liteasr_amd/lib/exp) + product bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CASES=("fc1" "dd bias" "dX dd (nn)" "dd res" "fc2 fwd" "dX fc1 (nn" "dW fc1" "dW dd")
echo "=== product"
timeout -k 10 200 python -u tools/gemm_graph_bench.py --cold "${CASES[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
for n in 2 3 6 7; do
  echo "=== LASR_EXP=$n"
  LITEASR_HIP_LIB=$PWD/liteasr_amd/lib/exp/lib$n.so timeout -k 10 200 python -u tools/gemm_graph_bench.py --cold "${CASES[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_ks.json 2> gpurun_out/b_ks.err || exit 1
cat gpurun_out/b_ks.json
