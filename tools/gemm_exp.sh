#!/bin/bash
# Build GEMM ablation variants of the library (CPU side): liteasr_amd/lib/exp/lib<N>.so with
# LASR_EXP=N compiled into every GEMM translation unit (gemm.hip, gemm_l0..3.hip).
# bit 1: skip the MFMAs, bit 2: skip the epilogue stores, bit 4: skip the glds loads, bit 8: no
# dropout draws in the Swish-gate epilogue, bit 16: no activation math there.
set -e
cd "$(dirname "$0")/.."
make -j8 >/dev/null
mkdir -p liteasr_amd/lib/exp
objs=$(ls build/obj/*.o | grep -v "/gemm.o\|/gemm_l[0-9].o")
for n in "$@"; do
  mkdir -p build/exp$n
  for f in gemm gemm_l0 gemm_l1 gemm_l2 gemm_l3; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DLASR_EXP=$n -c liteasr_amd/csrc/$f.hip -o build/exp$n/$f.o 2>/dev/null &
  done
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o liteasr_amd/lib/exp/lib$n.so $objs build/exp$n/*.o
done
