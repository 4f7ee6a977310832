set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 0 1 2 4 7; do
  echo "=== LASR_EXP=$n"
  GEMM_TORCH_REF=0 LITEASR_HIP_LIB=$PWD/tools/exp/lib$n.so timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
