set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "=== base + torch"
timeout -k 10 200 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/abl_base.txt || exit 1
for n in 1 2 4 7; do
  echo "=== LASR_EXP=$n"
  GEMM_TORCH_REF=0 LITEASR_HIP_LIB=$PWD/tools/abl/lib$n.so timeout -k 10 200 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/abl_$n.txt || exit 1
done
