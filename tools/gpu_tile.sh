set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/gemm_graph_bench.py "$@" 2>&1 | grep -v amdgpu.ids
