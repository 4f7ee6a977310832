#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/s3i
OUT=$R/gpurun_out/s3i
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pf" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case dw > "$OUT/pf.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pw" -o run -- python3 "$R/bench.py" --roofline-only 20 --roofline-case dw > "$OUT/pw.log" 2>&1 || exit 1
grep "^{" "$OUT/pf.log" | tail -1 > "$OUT/meta.json"
python3 "$R/tools/pmc_traffic.py" "$OUT/pf/run_results.db" "$OUT/pw/run_results.db" "$OUT/meta.json" "$OUT/pmc_dw.json" || exit 1
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print(d['ms_per_step'], r['avg_launch_us'], r['frac'], r['hottest_instance']['avg_launch_us'])"
