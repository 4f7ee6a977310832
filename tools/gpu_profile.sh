#!/bin/bash
# GPU-box measurement pass: kernel-trace stats of the default bench command and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, no trace domains) of the roofline
# kernel.  Output under gpurun_out/<tag>/.  Each GPU step has its own time limit and the
# script stops at the first failure.
set -u
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() { echo "=== $*"; "$@"; rc=$?; echo "=== rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_trace.log" 2>&1
run timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 "$R/bench.py" --roofline-only 20 > "$OUT/pmc_fetch.log" 2>&1
run timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 "$R/bench.py" --roofline-only 20 > "$OUT/pmc_write.log" 2>&1
grep "^{" "$OUT/pmc_fetch.log" | tail -1 > "$OUT/roofline_meta.json"
echo done
