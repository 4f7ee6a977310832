#!/bin/bash
# Build GEMM ablation variants of the library (CPU side): liteasr_amd/lib/exp/lib<N>.so with
# LASR_EXP=N compiled into every GEMM translation unit (gemm.hip, gemm_l0..3.hip).
# EXP_FILES (default: the GEMM units) names other translation units to build this way
# (e.g. EXP_FILES=ctc, whose LASR_EXP bits are listed in ctc.hip).
# GEMM bits: bit 1: skip the MFMAs, bit 2: skip the epilogue stores, bit 4: skip the glds loads, bit 8: no
# dropout draws in the Swish-gate epilogue, bit 16: no activation math there.
set -e
cd "$(dirname "$0")/.."
make -j8 >/dev/null
mkdir -p liteasr_amd/lib/exp
FILES=${EXP_FILES:-gemm gemm_l0 gemm_l1 gemm_l2 gemm_l3}
pat=$(for f in $FILES; do printf '/%s.o\\|' $f; done); pat=${pat%\\|}
objs=$(ls build/obj/*.o | grep -v "$pat")
for n in "$@"; do
  mkdir -p build/exp$n
  rm -f build/exp$n/*.o
  for f in $FILES; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DLASR_EXP=$n -c liteasr_amd/csrc/$f.hip -o build/exp$n/$f.o 2>/dev/null &
  done
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o liteasr_amd/lib/exp/lib$n.so $objs build/exp$n/*.o
done
