set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 1 2 4 7; do
  echo "=== LASR_EXP=$n"
  LITEASR_HIP_LIB=$PWD/tools/exp/lib$n.so timeout -k 10 200 python -u tools/gemm_graph_bench.py "fc1" "dd bias" "fc2 fwd" "dW fc1" "square" "ctc head" 2>&1 | grep -v amdgpu.ids || exit 1
done
