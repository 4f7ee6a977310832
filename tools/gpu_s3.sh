#!/bin/bash
# session-3 experiment runner: ./tools/gpu_s3.sh <tag> <python tool args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 600 python -u "$@" > gpurun_out/$tag.txt 2>&1; rc=$?
echo "rc=$rc"; cat gpurun_out/$tag.txt | grep -v amdgpu.ids
exit $rc
