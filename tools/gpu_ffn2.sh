#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "ffn_fused" --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
echo "ffn tests rc=$rc"; grep -E "passed|failed|^E " gpurun_out/t_$tag.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ffn_bench.py > gpurun_out/ffnb_$tag.log 2>&1; rc=$?
echo "ffn bench rc=$rc"; grep -v amdgpu.ids gpurun_out/ffnb_$tag.log
exit $rc
