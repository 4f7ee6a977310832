mkdir -p gpurun_out/r4k
for v in NONE LASR_DEC_ROW_LN LASR_FUSED_DEC_ATTN LASR_EPI_SPEC LASR_FUSED_LN2 LASR_ROW_LN LASR_BATCH_POS_PROJ; do
  echo "== $v" >> gpurun_out/r4k/c4b.log
  env $v=0 timeout -k 10 200 python -u -m pytest -q -s --timeout 180 --timeout-method thread -m gpu tests/test_model_gpu.py -k "config4_full_model_fp32" 2>&1 | grep -E "fp32 parity|passed|failed" >> gpurun_out/r4k/c4b.log || true
done
