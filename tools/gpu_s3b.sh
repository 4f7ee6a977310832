#!/bin/bash
# kernel tests, GEMM ablation, bench + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3b_t.log 2>&1; rc=$?
echo "kernel tests rc=$rc"; tail -3 gpurun_out/s3b_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s3b_b.json 2> gpurun_out/s3b_b.err || exit 1
cat gpurun_out/s3b_b.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tr_s3b -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --steps 5 --warmup 3 > $R/gpurun_out/tr_s3b.log 2>&1 ) || exit 1
CASES=("fc1" "dd bias" "dX dd (nn)" "dd res" "fc2 fwd" "dX fc1 (nn" "dW fc1" "dW dd")
for n in 2 3 6 7; do
  echo "=== LASR_EXP=$n"
  LITEASR_HIP_LIB=$PWD/liteasr_amd/lib/exp/lib$n.so timeout -k 10 200 python -u tools/gemm_graph_bench.py --cold "${CASES[@]}" 2>&1 | grep -v amdgpu.ids || exit 1
done
