#!/bin/bash
# GPU pass (round 6).  Usage: tools/gpu_r05.sh TAG STEP...; output under gpurun_out/TAG/.
# Every step has its own time limit; the script stops at the first failure.
set -u -o pipefail
TAG=${1:-r06}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
run() { echo "=== $*" >&2; "$@"; rc=$?; echo "=== rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for s in "$@"; do
  cd "$R"
  case $s in
    tests) run timeout -k 10 900 $PYT tests > "$OUT/tests.log" 2>&1 ;;
    new) run timeout -k 10 900 $PYT tests/test_native_reducer_gpu.py tests/test_switches_gpu.py tests/test_nodes_gpu.py \
           "tests/test_model_gpu.py::test_parity_config4_full_model_fp32" "tests/test_model_gpu.py::test_parity_config4_full_model_bf16_emulated" \
           "tests/test_kernels_gpu.py::test_gemm_ksub2_bit_identical" -s > "$OUT/new.log" 2>&1 ;;
    attncheck) # bitwise A/B of the attention kernels: ab_prev/'s library vs the tree's
           run timeout -k 10 300 python3 tools/with_lib.py $R/ab_prev/liteasr_amd/lib/libliteasr_hip.so tools/attn_check.py dump "$OUT/attn_base.pt" > "$OUT/attn_check.log" 2>&1
           run timeout -k 10 300 python3 tools/attn_check.py dump "$OUT/attn_new.pt" >> "$OUT/attn_check.log" 2>&1
           run python3 tools/attn_check.py cmp "$OUT/attn_new.pt" "$OUT/attn_base.pt" > "$OUT/attn_check.jsonl" 2>&1
           rm -f "$OUT/attn_base.pt" "$OUT/attn_new.pt" ;;
    epiab) # FFN fc1 epilogue ablation: the tree's library and the LASR_EXP builds in liteasr_amd/lib/exp
           for rep in 1 2; do for v in tree ${EXP_LIBS:-8 16 24}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             run timeout -k 10 120 python3 tools/with_lib.py $lib tools/epi_ab.py >> "$OUT/epi_ab.jsonl" 2>> "$OUT/epi_ab.err"; done; done ;;
    envlist) # whole step, one tree, the environments of ENV_LIST ("VAR=val ...;VAR=val;..."), two passes
           IFS=';' read -ra ENVS <<< "${ENV_LIST:-}"
           for rep in 1 2; do for i in "${!ENVS[@]}"; do e=${ENVS[$i]}
             env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 ${AB_ARGS:-} > "$OUT/envlist_$i.json" 2> "$OUT/envlist_$i.err" || exit 1
             grep "^{" "$OUT/envlist_$i.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=(d['config'].get('allreduce') or {}); t=a.get('timeline_last_step') or {}; print(json.dumps({'env': '$e', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'segment_ms': t.get('segment_ms')}))" >> "$OUT/envlist.jsonl"; done; done ;;
    conv2ab) # subsampling conv2 GEMMs: the tree's library vs liteasr_amd/lib/exp/lib$N.so (EXP_LIBS="32 ...")
           for rep in 1 2; do for v in tree ${EXP_LIBS:-}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             run timeout -k 10 120 python3 tools/with_lib.py $lib tools/conv2_bench.py ${CONV2_SHAPE:-} | sed "s/^{/{\"v\": \"$v\", /" >> "$OUT/conv2_ab.jsonl" || exit 1; done; done ;;
    envab) # whole step, one tree, two environments alternating (ENV_A / ENV_B: "VAR=val ...")
           for v in A B A B; do e=$ENV_A; [ $v = B ] && e=$ENV_B
             env $e timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-roofline --no-chunk-compare --steps 40 ${AB_ARGS:-} > "$OUT/envab_$v.json" 2> "$OUT/envab_$v.err" || exit 1
             grep "^{" "$OUT/envab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'env': '$e', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median')}))" >> "$OUT/envab.jsonl"; done ;;
    dyn) run timeout -k 10 900 $PYT tests/test_kernels_gpu.py -k "u2_prep or embed_and_prep or prep" \
           tests/test_model_gpu.py -k "dynamic or config4 or graphed or chunk" -s > "$OUT/dyn.log" 2>&1 ;;
    hold) run timeout -k 10 300 $PYT tests/test_fusions_gpu.py tests/test_kernels_gpu.py -k "held or chained or reduce_multi or dw_group" > "$OUT/hold.log" 2>&1
          run timeout -k 10 600 $PYT tests/test_native_reducer_gpu.py tests/test_trainer_gpu.py tests/test_model_gpu.py >> "$OUT/hold.log" 2>&1 ;;
    fus) run timeout -k 10 600 $PYT tests/test_fusions_gpu.py -s > "$OUT/fus.log" 2>&1 ;;
    fc1sweep) run timeout -k 10 300 python3 tools/fc1_tile_sweep.py > "$OUT/fc1_sweep_small.jsonl" 2> "$OUT/fc1_sweep.err"
           run timeout -k 10 300 python3 tools/fc1_tile_sweep.py 7968 2048 512 > "$OUT/fc1_sweep_large.jsonl" 2>> "$OUT/fc1_sweep.err" ;;
    flagab) # whole step under FLAG_A / FLAG_B module overrides (tools/flag_ab.py), alternating, AB_ARGS
           for v in A B A B; do f=$FLAG_A; [ $v = B ] && f=$FLAG_B
             run timeout -k 10 400 python3 tools/flag_ab.py $f -- bench.py --no-cpu-baseline --no-roofline --no-chunk-compare --steps 40 ${AB_ARGS:-} > "$OUT/flagab_$v.json" 2> "$OUT/flagab_$v.err"
             grep "^{" "$OUT/flagab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'flags': '$f', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'launches': (d.get('graph_nodes_per_step') or {}).get('kernel')}))" >> "$OUT/flagab.jsonl"; done ;;
    dwdirect) run timeout -k 10 600 $PYT tests/test_kernels_gpu.py -k "dw_group" > "$OUT/dwdirect.log" 2>&1 ;;
    attnab2) # attention kernels: ab_lib/base.so (the library before the change) vs the tree's: bitwise
           # outputs (attn_check) and graph-replayed times, alternating
           run timeout -k 10 300 python3 tools/with_lib.py $R/ab_lib/${VARIANT:-base}.so tools/attn_check.py dump "$OUT/attn_base.pt" > "$OUT/attn_check.log" 2>&1
           run timeout -k 10 300 python3 tools/attn_check.py dump "$OUT/attn_new.pt" >> "$OUT/attn_check.log" 2>&1
           run python3 tools/attn_check.py cmp "$OUT/attn_new.pt" "$OUT/attn_base.pt" > "$OUT/attn_check.jsonl" 2>&1
           rm -f "$OUT/attn_base.pt" "$OUT/attn_new.pt"
           for v in base new base new; do
             if [ $v = base ]; then run timeout -k 10 300 python3 tools/with_lib.py $R/ab_lib/${VARIANT:-base}.so tools/attn_bench.py > "$OUT/attn_ab_$v.tmp"
             else run timeout -k 10 300 python3 tools/attn_bench.py > "$OUT/attn_ab_$v.tmp"; fi
             sed "s/^{/{\"lib\": \"$v\", /" "$OUT/attn_ab_$v.tmp" >> "$OUT/attn_ab.jsonl"; rm -f "$OUT/attn_ab_$v.tmp"; done ;;
    libab) # whole step: the tree's library vs ab_lib/$VARIANT.so (tools/with_lib.py), alternating, AB_ARGS
           for v in tree var tree var; do
             if [ $v = var ]; then run timeout -k 10 400 python3 tools/with_lib.py $R/ab_lib/$VARIANT.so bench.py --no-cpu-baseline --no-roofline --no-chunk-compare --steps 40 ${AB_ARGS:-} > "$OUT/libab_$v.json" 2> "$OUT/libab_$v.err"
             else run timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-roofline --no-chunk-compare --steps 40 ${AB_ARGS:-} > "$OUT/libab_$v.json" 2> "$OUT/libab_$v.err"; fi
             grep "^{" "$OUT/libab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'variant': '${VARIANT:-}', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'launches': (d.get('graph_nodes_per_step') or {}).get('kernel')}))" >> "$OUT/libab.jsonl"; done ;;
    flaglist) # whole step under each entry of FLAG_LIST ("mod.attr=v mod.attr=v;...;..."; an empty entry
           # = the tree as is) and ENV_LIST alike, two passes, AB_ARGS
           IFS=';' read -ra FL <<< "${FLAG_LIST:-}"
           for rep in 1 2; do for i in "${!FL[@]}"; do f=${FL[$i]}
             run timeout -k 10 400 python3 tools/flag_ab.py $f -- bench.py --no-cpu-baseline --no-roofline --no-chunk-compare --steps 40 ${AB_ARGS:-} > "$OUT/flaglist_$i.json" 2> "$OUT/flaglist_$i.err"
             grep "^{" "$OUT/flaglist_$i.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'flags': '$f', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'launches': (d.get('graph_nodes_per_step') or {}).get('kernel')}))" >> "$OUT/flaglist.jsonl"; done; done ;;
    largedyn) run timeout -k 10 500 python3 bench.py --config large --no-cpu-baseline --no-roofline > "$OUT/bench_large_dyn.json" 2> "$OUT/bench_large_dyn.err" ;;
    switches) run timeout -k 10 900 $PYT tests/test_switches_gpu.py > "$OUT/switches.log" 2>&1 ;;
    new5) run timeout -k 10 900 $PYT tests/test_native_reducer_gpu.py "tests/test_nodes_gpu.py::test_decoder_layer_node" \
           "tests/test_model_gpu.py::test_parity_config4_full_model_fp32" -s > "$OUT/new5.log" 2>&1 ;;
    ctc) run timeout -k 10 600 $PYT tests -k "ctc or CTC" > "$OUT/ctc.log" 2>&1 ;;
    attn) run timeout -k 10 600 $PYT tests/test_kernels_gpu.py -k "relattn or decoder_attention or attn" > "$OUT/attn.log" 2>&1 ;;
    attnbench) run timeout -k 10 300 python3 tools/attn_bench.py > "$OUT/attn_bench.jsonl" 2> "$OUT/attn_bench.err" ;;
    attnab) # attention kernels: the library in ab/ (same ABI) vs the tree's, alternating
           for v in base new base new; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v = base ] && lib=$R/ab_prev/liteasr_amd/lib/libliteasr_hip.so
             run timeout -k 10 300 python3 tools/with_lib.py $lib tools/attn_bench.py > "$OUT/attn_ab_$v.tmp"
             sed "s/^{/{\"lib\": \"$v\", /" "$OUT/attn_ab_$v.tmp" >> "$OUT/attn_ab.jsonl"; rm -f "$OUT/attn_ab_$v.tmp"; done ;;
    attnexp) # attention kernels: the tree's library vs liteasr_amd/lib/exp/lib$N.so ablation builds (EXP_LIBS), twice
           for rep in 1 2; do for v in tree ${EXP_LIBS:-}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             run timeout -k 10 300 python3 tools/with_lib.py $lib tools/attn_bench.py > "$OUT/attn_exp_$v.tmp"
             sed "s/^{/{\"lib\": \"$v\", /" "$OUT/attn_exp_$v.tmp" >> "$OUT/attn_exp.jsonl"; rm -f "$OUT/attn_exp_$v.tmp"; done; done ;;
    ctcexp) # CTC kernels at small and long: the tree's library vs lib/exp/lib$N.so (EXP_LIBS), twice
           for rep in 1 2; do for v in tree ${EXP_LIBS:-}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             run timeout -k 10 200 python3 tools/with_lib.py $lib tools/ctc_bench.py > "$OUT/ctc.tmp" 2>> "$OUT/ctcexp.err"
             sed "s/^{/{\"lib\": \"$v\", /" "$OUT/ctc.tmp" >> "$OUT/ctcexp.jsonl"; rm -f "$OUT/ctc.tmp"; done; done ;;
    toolab) # TOOL (a script printing JSON lines) under the tree's library, ab_prev/'s and lib/exp/lib$N.so (EXP_LIBS), twice
           for rep in 1 2; do for v in tree prev ${EXP_LIBS:-}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so
             [ $v = prev ] && lib=$R/ab_prev/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && [ $v != prev ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             run timeout -k 10 200 python3 tools/with_lib.py $lib $TOOL > "$OUT/toolab.tmp" 2>> "$OUT/toolab.err"
             sed "s/^{/{\"lib\": \"$v\", /" "$OUT/toolab.tmp" >> "$OUT/toolab.jsonl"; rm -f "$OUT/toolab.tmp"; done; done ;;
    caseab) # bench.py roofline cases (RCASES "small:dw large:dw ..."): the tree's library vs lib/exp/lib$N.so (EXP_LIBS), twice
           for rep in 1 2; do for v in tree ${EXP_LIBS:-}; do lib=$R/liteasr_amd/lib/libliteasr_hip.so; [ $v != tree ] && lib=$R/liteasr_amd/lib/exp/lib$v.so
             for rc in ${RCASES:-small:dw}; do cfg=${rc%%:*}; cs=${rc##*:}
               run timeout -k 10 200 python3 tools/with_lib.py $lib bench.py --config $cfg --roofline-only 20 --roofline-case $cs > "$OUT/caseab.tmp" 2>> "$OUT/caseab.err"
               grep "^{" "$OUT/caseab.tmp" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'cfg': '$cfg', 'case': '$cs', 'kernel': d.get('kernel'), 'us': d.get('us_per_launch_eager')}))" >> "$OUT/caseab.jsonl"; done; done; done ;;
    stepab) # whole step: the previous commit's tree (ab_prev/: `git archive` + its built library) vs this
           # tree, alternating (AB_ARGS: e.g. --config large)
           for v in base new base new; do d=$R; [ $v = base ] && d=$R/ab_prev
             (cd $d && run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 ${AB_ARGS:-}) > "$OUT/step_ab_$v.json" 2> "$OUT/step_ab_$v.err" || exit 1
             grep "^{" "$OUT/step_ab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'args': '${AB_ARGS:-}', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'utt_s': d['value']}))" >> "$OUT/step_ab.jsonl"; done ;;
    attnprof) cd /tmp
           for cs in ${ATTN_CASES:-small long}; do
             run timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/attn_trace" -o run -- python3 "$R/tools/attn_bench.py" $cs > "$OUT/attn_trace.log" 2>&1
             cp "$(find "$OUT/attn_trace" -name '*kernel_stats.csv' | head -1)" "$OUT/attn_kernel_stats_$cs.csv"; rm -rf "$OUT/attn_trace"; done
           S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU"
           S2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA"
           for cs in ${ATTN_CASES:-small long}; do i=0; for set in "$S1" "$S2"; do i=$((i+1))
             run timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/ap$i" -o run -- python3 "$R/tools/attn_bench.py" $cs > "$OUT/ap$i.log" 2>&1
             run python3 "$R/tools/pmc_kernels.py" "$(find "$OUT/ap$i" -name '*.db' | head -1)" flash_ > "$OUT/attn_pmc_${cs}_$i.json"; rm -rf "$OUT/ap$i"; done; done ;;
    kgpu) run timeout -k 10 600 $PYT tests/test_kernels_gpu.py tests/test_row_ln_gpu.py > "$OUT/kgpu.log" 2>&1 ;;
    model) run timeout -k 10 900 $PYT tests/test_model_gpu.py tests/test_nodes_gpu.py -s > "$OUT/model.log" 2>&1 ;;
    smoke) run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) run timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    benchprof) # rocprofv3 --kernel-trace --stats of the default bench command (the summary kept under profiles/)
           cd /tmp && run timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/benchprof" -o run -- python3 "$R/bench.py" > "$OUT/rocprofv3_bench.log" 2>&1
           grep "^{" "$OUT/rocprofv3_bench.log" | tail -1 > "$OUT/rocprofv3_bench.json"
           cp "$(find "$OUT/benchprof" -name '*kernel_stats.csv' | head -1)" "$OUT/rocprofv3_kernel_stats_bench.csv"; rm -rf "$OUT/benchprof" ;;
    benchq) run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 > "$OUT/benchq.json" 2> "$OUT/benchq.err" ;;
    long) run timeout -k 10 300 python3 bench.py --config long --no-cpu-baseline > "$OUT/bench_long.json" 2> "$OUT/bench_long.err" ;;
    large) run timeout -k 10 400 python3 bench.py --config large --no-cpu-baseline > "$OUT/bench_large.json" 2> "$OUT/bench_large.err" ;;
    ddp1) run timeout -k 10 300 python3 bench.py --force-ddp --no-cpu-baseline --no-roofline > "$OUT/bench_ddp1.json" 2> "$OUT/bench_ddp1.err" ;;
    ddpab) # world-1 A/B in one call: plain step, torch DDP, native DDP (no collective at world 1),
           # native DDP with the 1-rank RCCL all-reduces forced (their cost beside the backward)
           for rep in 1 2; do for v in plain torch native forced; do
             case $v in plain) a="";; torch) a="--force-ddp";; native) a="--force-ddp --comm native";;
               forced) a="--force-ddp --comm native --single-rank-collectives";; esac
             run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 $a > "$OUT/ddpab_$v.json" 2> "$OUT/ddpab_$v.err"
             grep "^{" "$OUT/ddpab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['config']['allreduce'] or {}; t=a.get('timeline_last_step') or {}; print(json.dumps({'arm': '$v', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'segment_ms': t.get('segment_ms'), 'exposed_comm_ms': t.get('exposed_comm_ms')}))" >> "$OUT/ddpab.jsonl"; done; done ;;
    ddp1n) run timeout -k 10 300 python3 bench.py --force-ddp --comm native --no-cpu-baseline --no-roofline > "$OUT/bench_ddp1_native.json" 2> "$OUT/bench_ddp1_native.err" ;;
    famsq) cd /tmp  # SQ counter sets over the family roofline case (the stall breakdown)
           S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU"
           S2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA"
           i=0; for set in "$S1" "$S2"; do i=$((i+1))
             run timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/fs$i" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --roofline-only 10 --roofline-case family > "$OUT/fs$i.log" 2>&1
             run python3 "$R/tools/pmc_kernels.py" "$(find "$OUT/fs$i" -name '*.db' | head -1)" gemm_bf16_glds_kernel row_res_ln row_dx_ln_bwd > "$OUT/family_sq_${PMC_CONFIG:-small}_$i.json"; rm -rf "$OUT/fs$i"; done ;;
    tracefam) cd /tmp && run timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_family" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --roofline-only 50 --roofline-case family > "$OUT/trace_family.log" 2>&1
           grep "^{" "$OUT/trace_family.log" | tail -1 > "$OUT/trace_family_meta.json"
           run python3 "$R/tools/family_trace.py" "$(find "$OUT/trace_family" -name '*.db' | head -1)" "$OUT/trace_family_meta.json" > "$OUT/family_trace_summary_${PMC_CONFIG:-small}.json"; rm -rf "$OUT/trace_family" ;;
    splitk) run timeout -k 10 300 python3 tools/splitk_sweep.py > "$OUT/splitk_small.jsonl" 2> "$OUT/splitk.err"
           run timeout -k 10 300 python3 tools/splitk_sweep.py 7968 512 2048 > "$OUT/splitk_large.jsonl" 2>> "$OUT/splitk.err" ;;
    tileab) run timeout -k 10 200 python3 tools/tile_ab.py > "$OUT/tile_ab.jsonl" 2> "$OUT/tile_ab.err" ;;
    blaslt) run timeout -k 10 120 python3 tools/blaslt_ref.py > "$OUT/blaslt.jsonl" 2> "$OUT/blaslt.err" ;;
    trace) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > "$OUT/trace.log" 2>&1
           db=$(find "$OUT/trace" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary.txt" 2>&1
           python3 "$R/tools/step_summary.py" "$db" 5 --grid > "$OUT/step_summary_grid.txt" 2>&1
           python3 "$R/tools/step_summary.py" "$db" 5 --order > "$OUT/step_order.txt" 2>&1; rm -f "$db" ;;
    tracelong) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_long" -o run -- python3 "$R/bench.py" --config long --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > "$OUT/trace_long.log" 2>&1
           db=$(find "$OUT/trace_long" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary_long.txt" 2>&1
           python3 "$R/tools/step_summary.py" "$db" 5 --order > "$OUT/step_order_long.txt" 2>&1; rm -f "$db" ;;
    tracelarge) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_large" -o run -- python3 "$R/bench.py" --config large --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > "$OUT/trace_large.log" 2>&1
           db=$(find "$OUT/trace_large" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary_large.txt" 2>&1
           python3 "$R/tools/step_summary.py" "$db" 5 --grid > "$OUT/step_summary_grid_large.txt" 2>&1
           python3 "$R/tools/step_summary.py" "$db" 5 --order > "$OUT/step_order_large.txt" 2>&1; rm -f "$db" ;;
    profile) cd /tmp && run timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/prof_markers" -o run -- python3 "$R/bench.py" --profile --no-cpu-baseline --no-roofline --steps 3 --warmup 1 > "$OUT/profile.log" 2>&1 ;;
    pmc) for c in ${PMC_CASES:-family dw hot}; do
           cd /tmp && run timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$c" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --roofline-only 20 --roofline-case $c > "$OUT/pmc_fetch_$c.log" 2>&1
           run timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$c" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --roofline-only 20 --roofline-case $c > "$OUT/pmc_write_$c.log" 2>&1
           grep "^{" "$OUT/pmc_fetch_$c.log" | tail -1 > "$OUT/roofline_meta_$c.json"
           run python3 "$R/tools/pmc_traffic.py" "$(find "$OUT/pmc_fetch_$c" -name '*.db' | head -1)" "$(find "$OUT/pmc_write_$c" -name '*.db' | head -1)" "$OUT/roofline_meta_$c.json" "$OUT/roofline_pmc_${c}_${PMC_CONFIG:-small}.json"
           rm -rf "$OUT/pmc_fetch_$c" "$OUT/pmc_write_$c"
         done ;;
    mfma) cd /tmp && run timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --graph off --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$OUT/pmc_mfma.log" 2>&1
          run python3 "$R/tools/pmc_mfma.py" "$(find "$OUT/pmc_mfma" -name '*counter_collection.csv' | head -1)" ${PMC_CONFIG:-small} > "$OUT/pmc_mfma_summary_${PMC_CONFIG:-small}.json"
          rm -rf "$OUT/pmc_mfma" ;;
    mfmacase) cd /tmp && run timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mc" -o run -- python3 "$R/bench.py" --config ${PMC_CONFIG:-small} --roofline-only 10 --roofline-case attn > "$OUT/pmc_mc.log" 2>&1
          grep "^{" "$OUT/pmc_mc.log" | tail -1 > "$OUT/mc_meta.json"
          run python3 "$R/tools/pmc_mfma.py" "$(find "$OUT/pmc_mc" -name '*counter_collection.csv' | head -1)" --case "$OUT/mc_meta.json" > "$OUT/pmc_mfma_case_attn_${PMC_CONFIG:-small}.json"
          rm -rf "$OUT/pmc_mc" ;;
    libab) # whole-step A/B against the round-3 tree (ab_r03/: `git archive 42f6a8d` + its built
           # library; the Python layer changed ABI this round, so the base runs its own tree)
           for v in ${AB_ORDER:-base new base new}; do d=$R; [ $v = base ] && d=$R/ab_r03
             (cd $d && run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 40 ${AB_ARGS:-}) > "$OUT/ab_$v.json" 2> "$OUT/ab_$v.err"
             grep "^{" "$OUT/ab_$v.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tree': '$v', 'ms': d['ms_per_step'], 'median': d.get('ms_per_step_median'), 'utt_s': d['value']}))" >> "$OUT/libab.jsonl"; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
