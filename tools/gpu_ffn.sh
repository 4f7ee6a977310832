#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "ffn_fused" --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
echo "ffn tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|^E " gpurun_out/t_$tag.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ffn_bench.py > gpurun_out/ffnb_$tag.log 2>&1; rc=$?
echo "ffn bench rc=$rc"; grep -v amdgpu.ids gpurun_out/ffnb_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "parity or graphed or ddp or encoder_reuse" --timeout 200 --timeout-method thread > gpurun_out/t2_$tag.log 2>&1; rc=$?
echo "model tests rc=$rc"; tail -5 gpurun_out/t2_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/b1_$tag.json 2> gpurun_out/b1_$tag.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/b1_$tag.json
exit $rc
