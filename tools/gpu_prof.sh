set -o pipefail
# kernel-trace of the default bench: gpurun -- bash tools/gpu_prof.sh <tag>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$1 -o run -- python3 bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3 ${2:+--config $2} > gpurun_out/tr_$1.log 2>&1; rc=$?
echo "prof rc=$rc"
find gpurun_out/tr_$1 -name "*.db" > gpurun_out/tr_$1.path
exit $rc
