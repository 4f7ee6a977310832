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
    smoke) cd "$R" && run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) cd "$R" && run timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    benchq) cd "$R" && run timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline > "$OUT/benchq.json" 2> "$OUT/benchq.err" ;;
    long) cd "$R" && run timeout -k 10 300 python3 bench.py --config long --no-cpu-baseline > "$OUT/bench_long.json" 2> "$OUT/bench_long.err" ;;
    large) cd "$R" && run timeout -k 10 300 python3 bench.py --config large --no-cpu-baseline --no-roofline > "$OUT/bench_large.json" 2> "$OUT/bench_large.err" ;;
    ddp1) cd "$R" && run timeout -k 10 300 python3 bench.py --force-ddp --no-cpu-baseline --no-roofline > "$OUT/bench_ddp1.json" 2> "$OUT/bench_ddp1.err" ;;
    trace) cd /tmp && run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > "$OUT/trace.log" 2>&1
           db=$(find "$OUT/trace" -name "*.db" | head -1); python3 "$R/tools/step_summary.py" "$db" > "$OUT/step_summary.txt" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
