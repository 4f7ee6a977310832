"""Launch census of one training step, on the CPU (no GPU needed).

Runs bench.py's model and loss forward + backward on CPU tensors with every HIP launch
replaced by a recorder (the planner, lasr_gemm_plan, is host code and really runs), then
prints the step's GEMMs grouped by (M, N, K, batch, planned tile, split, call site).  Tool
for deciding where a kernel change pays; numbers are meaningless, shapes and counts are not.

  python tools/step_census.py [--config small] [--sort count|flops]
"""

from __future__ import annotations

import argparse
import collections
import ctypes as C
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from liteasr_amd import _native as N  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if fr.filename.endswith(("kernels.py", "_native.py", "step_census.py")):
            continue
        return f"{os.path.basename(fr.filename)}:{fr.lineno}:{fr.name}"
    return "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="small")
    ap.add_argument("--sort", default="flops")
    args = ap.parse_args()
    cfgd = bench.CONFIGS[args.config]
    real_call = N.call
    lib = N.load()
    rec = collections.Counter()
    gemms = collections.Counter()
    flops = collections.Counter()

    def call(name, *a):
        if name == "lasr_gemm_plan" or name.startswith("lasr_dropout"):
            return real_call(name, *a)
        rec[name] += 1
        if name == "lasr_gemm":
            g = a[0]._obj
            tm, tn, sp, fl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
            real_call("lasr_gemm_plan", C.byref(g), C.byref(tm), C.byref(tn), C.byref(sp), C.byref(fl))
            key = (g.M, g.N, g.K, g.batch, f"{tm.value}x{tn.value}", sp.value, g.c_dtype, site())
            gemms[key] += 1
            flops[key] += 2 * g.M * g.N * g.K * g.batch
        elif name == "lasr_gemm_dw_group":
            arr, n = a[0], a[1]
            for i in range(n):
                g = arr[i]
                key = (g.M, g.N, g.K, g.batch, "group", -g.split_k, g.c_dtype, "dw_group")
                gemms[key] += 1
                flops[key] += 2 * g.M * g.N * g.K * g.batch
        return 0

    N.call = call
    K.stream = lambda: 0
    torch.cuda.is_current_stream_capturing = lambda: False
    from liteasr_amd.models import _fused

    _fused._require_hip = lambda model, xs: None
    torch.manual_seed(0)
    dev = torch.device("cpu")
    model = bench.build(cfgd, "bf16", 0.1, dev)
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig

    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=bench.V, smoothing=0.1, ctc_weight=cfgd["w"]))
    batch = bench.synthetic(cfgd, 0, dev)
    loss = crit(model, *batch)
    loss.backward()
    del lib
    order = sorted(gemms, key=lambda k: -(flops[k] if args.sort == "flops" else gemms[k]))
    print(f"{'M':>7} {'N':>6} {'K':>6} {'bat':>4} {'tile':>8} {'sp':>3} {'cdt':>3} {'n':>4} {'GFLOP':>8}  site")
    for k in order:
        M, Nn, Kd, b, tile, sp, cdt, s = k
        print(f"{M:7d} {Nn:6d} {Kd:6d} {b:4d} {tile:>8} {sp:3d} {cdt:3d} {gemms[k]:4d} {flops[k] / 1e9:8.2f}  {s}")
    print()
    for name, n in rec.most_common():
        print(f"{n:5d} {name}")


if __name__ == "__main__":
    main()
