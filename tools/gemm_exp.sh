#!/bin/bash
# Build GEMM ablation variants of the library (CPU side): tools/exp/lib<N>.so with LASR_EXP=N.
set -e
cd "$(dirname "$0")/.."
make -j8 >/dev/null
objs=$(ls build/obj/*.o | grep -v gemm.o)
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DLASR_EXP=$n -c liteasr_amd/csrc/gemm.hip -o build/obj_exp_gemm_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/exp/lib$n.so $objs build/obj_exp_gemm_$n.o
done
