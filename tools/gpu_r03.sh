#!/bin/bash
# Round-3 GPU pass: GPU tests, the default bench line, a kernel trace of the bench.
# Usage: tools/gpu_r03.sh TAG [tests|bench|trace ...]; output under gpurun_out/TAG/.
# Every step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r03}; shift
STEPS=${*:-tests bench trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { echo "=== $*" >&2; "$@"; rc=$?; echo "=== rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for s in $STEPS; do
  case $s in
    tests) cd "$R" && run timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 ;;
    testsall) cd "$R" && timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1; echo "=== rc=$?" >&2 ;;
    rowln_ab) cd "$R" && for v in 0 1; do LASR_ROW_LN=$v timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 150 --timeout-method thread -k "large_width_chunk_bf16_emulated or config2_full_model_bf16_emulated" -s > "$OUT/rowln_ab_$v.log" 2>&1 || true; done ;;
    libab) cd "$R" && for v in base new base new; do lib=liteasr_amd/lib/libliteasr_hip.so; [ $v = base ] && lib=liteasr_amd/lib/ab/libliteasr_hip_base.so
             LITEASR_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 > "$OUT/bench_lib_$v.json" 2> "$OUT/bench_lib_$v.err" || exit 1
             grep "^{" "$OUT/bench_lib_$v.json" >> "$OUT/libab.jsonl"; done ;;
    convdx) cd "$R" && for v in ${AB_VALUES:-0 1 0 1}; do env ${AB_VAR:-LASR_DX_ROWTAB}=$v timeout -k 10 120 python3 tools/conv2_bench.py >> "$OUT/conv2_dx_ab.json" 2>> "$OUT/conv2_bench.err" || exit 1; done ;;
    convdx_old) cd "$R" && for v in 0 1 0 1; do LASR_DX_ROWTAB=$v run timeout -k 10 120 python3 tools/conv2_bench.py >> "$OUT/conv2_dx_ab.json" 2>> "$OUT/conv2_bench.err"; done ;;
    conv) cd "$R" && for v in ${CONV_VARIANTS:-0 1}; do LASR_CONV_WIDE=$v run timeout -k 10 120 python3 tools/conv2_bench.py >> "$OUT/conv2_bench.json" 2>> "$OUT/conv2_bench.err"; done
          run timeout -k 10 60 python3 -c "import torch; a=torch.load('/tmp/conv2_dw_0.pt'); b=torch.load('/tmp/conv2_dw_1.pt'); print('dw rel', ((a['dw']-b['dw']).abs().max()/a['dw'].abs().max()).item(), 'db rel', ((a['db']-b['db']).abs().max()/a['db'].abs().max()).item())" >> "$OUT/conv2_bench.json" ;;
    benchab) cd "$R" && for v in ${WIDE_VARIANTS:-0 1}; do LASR_GEMM_WIDE=$v run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 > "$OUT/bench_wide$v.json" 2> "$OUT/bench_wide$v.err"; done ;;
    variants) cd "$R" && run timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "variants" -s > "$OUT/variants.log" 2>&1 ;;
    envab) cd "$R" && for v in ${AB_VALUES:-0 1}; do env ${AB_VAR}=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 > "$OUT/bench_${AB_VAR}_$v.json" 2> "$OUT/bench_${AB_VAR}_$v.err" || exit 1
             grep "^{" "$OUT/bench_${AB_VAR}_$v.json" | sed "s/^{/{\"ab\": \"${AB_VAR}=$v\", /" >> "$OUT/envab.jsonl"; done ;;
    model) cd "$R" && run timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_trainer_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/model.log" 2>&1 ;;
    conv1) cd "$R" && run timeout -k 10 120 python3 tools/conv1_bench.py > "$OUT/conv1_bench.json" 2> "$OUT/conv1_bench.err" ;;
    kgpu) cd "$R" && run timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_nodes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/kgpu.log" 2>&1 ;;
    smoke) cd "$R" && run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) cd "$R" && run timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    benchq) cd "$R" && run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > "$OUT/benchq.json" 2> "$OUT/benchq.err" ;;
    long) cd "$R" && run timeout -k 10 300 python3 bench.py --config long --no-cpu-baseline > "$OUT/bench_long.json" 2> "$OUT/bench_long.err" ;;
    large) cd "$R" && run timeout -k 10 300 python3 bench.py --config large --no-cpu-baseline --no-roofline > "$OUT/bench_large.json" 2> "$OUT/bench_large.err" ;;
    ddp1) cd "$R" && run timeout -k 10 300 python3 bench.py --force-ddp --no-cpu-baseline --no-roofline > "$OUT/bench_ddp1.json" 2> "$OUT/bench_ddp1.err" ;;
    trace) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > "$OUT/trace.log" 2>&1
           db=$(find "$OUT/trace" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary.txt" 2>&1 ;;
    pmc) for c in ${PMC_CASES:-family dw hot}; do
           cd /tmp && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$c" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case $c > "$OUT/pmc_fetch_$c.log" 2>&1
           run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$c" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case $c > "$OUT/pmc_write_$c.log" 2>&1
           grep "^{" "$OUT/pmc_fetch_$c.log" | tail -1 > "$OUT/roofline_meta_$c.json"
           run python3 "$R/tools/pmc_traffic.py" "$(find "$OUT/pmc_fetch_$c" -name '*.db' | head -1)" "$(find "$OUT/pmc_write_$c" -name '*.db' | head -1)" "$OUT/roofline_meta_$c.json" "$OUT/roofline_pmc_$c.json"
           rm -rf "$OUT/pmc_fetch_$c" "$OUT/pmc_write_$c"  # counter databases: gpurun_out stays under its cap
         done ;;
    pmcsave) for c in family dw hot; do cp "$OUT/roofline_pmc_$c.json" "$R/profiles/r03/roofline_pmc_${c}_$TAG.json" || exit 1; done ;;
    mfma) cd /tmp && run timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o run -- python3 "$R/bench.py" --graph off --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$OUT/pmc_mfma.log" 2>&1
          run python3 "$R/tools/pmc_mfma.py" "$(find "$OUT/pmc_mfma" -name '*counter_collection.csv' | head -1)" > "$OUT/pmc_mfma_summary.json"
          rm -rf "$OUT/pmc_mfma" ;;
    tracelong) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_long" -o run -- python3 "$R/bench.py" --config long --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/trace_long.log" 2>&1
           db=$(find "$OUT/trace_long" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary_long.txt" 2>&1 ;;
    tracefam) cd /tmp && run timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_family" -o run -- python3 "$R/bench.py" --roofline-only 50 --roofline-case family > "$OUT/trace_family.log" 2>&1
           grep "^{" "$OUT/trace_family.log" | tail -1 > "$OUT/trace_family_meta.json"
           run python3 "$R/tools/family_trace.py" "$(find "$OUT/trace_family" -name '*.db' | head -1)" "$OUT/trace_family_meta.json" > "$OUT/family_trace_summary.json" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
