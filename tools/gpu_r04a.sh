set -u
R=$GRAFT_REPO_ROOT; cd $R; OUT=$R/gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 120 python3 tools/blaslt_ref.py > $OUT/blaslt.jsonl 2> $OUT/blaslt.err || { tail -5 $OUT/blaslt.err; exit 1; }
cat $OUT/blaslt.jsonl
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
