#!/bin/bash
# SQ counter passes over 2 eager steps of the bench (one pass per counter set; no tracing
# domains beside --pmc), summarised per kernel for the attention / GEMM kernels of interest.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${1:-pmcattn}; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU"
S2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_WR"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d "$OUT/p$i" -o run -- python3 "$R/bench.py" --graph off --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > "$OUT/p$i.log" 2>&1 || exit 1
  python3 "$R/tools/pmc_kernels.py" "$(find "$OUT/p$i" -name '*.db' | head -1)" relattn_ row_dx_ln gemm_bf16_glds_kernel gemm_dw_group conv1_bwd ctc_alpha > "$OUT/pmc_kernels_$i.json" || exit 1
  rm -rf "$OUT/p$i"
done
echo done
