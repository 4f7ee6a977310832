#!/bin/bash
# Round-2 (second session) measurement pass on the GPU box: kernel-trace stats of the default bench command,
# then separate PMC passes (FETCH_SIZE / WRITE_SIZE, no trace domains) of the two roofline
# kernels (the grouped FFN weight-gradient launch of one layer, and the hottest instance, the FFN fc1 forward).
# Output under gpurun_out/<tag>/; each GPU step has its own time limit, stop at the first failure.
set -u
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() { echo "=== $*"; "$@"; rc=$?; echo "=== rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_trace.log" 2>&1
for c in dw hot; do
  run timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$c" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case $c > "$OUT/pmc_fetch_$c.log" 2>&1
  run timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$c" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case $c > "$OUT/pmc_write_$c.log" 2>&1
  grep "^{" "$OUT/pmc_fetch_$c.log" | tail -1 > "$OUT/roofline_meta_$c.json"
  python3 "$R/tools/pmc_traffic.py" "$OUT/pmc_fetch_$c/run_results.db" "$OUT/pmc_write_$c/run_results.db" "$OUT/roofline_meta_$c.json" "$OUT/roofline_pmc_$c.json" || exit 1
done
run timeout -k 10 400 python3 "$R/bench.py" > "$OUT/bench_full.json" 2> "$OUT/bench_full.err"
# world-1 RCCL group through the DDP reducer: overlap timeline (segment / bucket events) and
# a kernel trace showing where the bucket all-reduce kernels land among the backward kernels
run timeout -k 10 300 python3 "$R/bench.py" --force-ddp --no-cpu-baseline --no-roofline > "$OUT/bench_ddp1.json" 2> "$OUT/bench_ddp1.err"
run timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace_ddp1" -o run -- python3 "$R/bench.py" --force-ddp --no-cpu-baseline --no-roofline --steps 3 --warmup 2 > "$OUT/trace_ddp1.log" 2>&1
# the other configs on the same code path
run timeout -k 10 300 python3 "$R/bench.py" --config large --no-cpu-baseline --no-roofline > "$OUT/bench_large.json" 2> "$OUT/bench_large.err"
run timeout -k 10 300 python3 "$R/bench.py" --config long --no-cpu-baseline --no-roofline > "$OUT/bench_long.json" 2> "$OUT/bench_long.err"
run timeout -k 10 300 python3 "$R/tools/paraformer_bench.py" > "$OUT/paraformer_bench.json" 2> "$OUT/paraformer_bench.err"
echo done
