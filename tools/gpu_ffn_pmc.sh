#!/bin/bash
# PMC pass over tools/ffn_bench.py (fused vs two-GEMM FFN): wave-state split + L2 hit rate
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_ffn -o run -- python3 $R/tools/ffn_bench.py > $R/gpurun_out/pmc_ffn.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 $R/gpurun_out/pmc_ffn.log
find $R/gpurun_out/pmc_ffn -name "*.csv" | head
exit $rc
