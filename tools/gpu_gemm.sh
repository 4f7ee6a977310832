set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
GEMM_TORCH_REF=0 timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids
