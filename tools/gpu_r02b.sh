#!/bin/bash
# tests (given -k), then the bf16 error measurement
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -k "$2" --timeout 300 --timeout-method thread > gpurun_out/t_$tag.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|^E " gpurun_out/t_$tag.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u tools/bf16_errs.py > gpurun_out/bf16_$tag.log 2>&1; rc=$?
echo "bf16 rc=$rc"; cat gpurun_out/bf16_$tag.log | tail -12
exit $rc
