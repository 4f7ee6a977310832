"""Tile A/B for the step's N = d, K = ff GEMMs (FFN fc2 forward with the fp32 residual epilogue,
FFN fc1 input gradient), each tile forced through the per-call tile override and timed as a replayed
hipGraph of `iters` launches (as bench.py times the roofline family).  Prints one JSON line per
(shape, tile).
    python tools/tile_ab.py [M N K]"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402


def graph_time(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    M, D, F = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (7968, 256, 2048)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, F, device=dev, generator=g).bfloat16()
    w2 = (torch.randn(D, F, device=dev, generator=g) * F ** -0.5).bfloat16()
    b2 = torch.randn(D, device=dev, generator=g) * 0.02
    res = torch.randn(M, D, device=dev, generator=g)
    out = torch.empty(M, D, device=dev)
    dz = torch.randn(M, F, device=dev, generator=g).bfloat16()
    w1 = (torch.randn(F, D, device=dev, generator=g) * F ** -0.5).bfloat16()
    dln = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    def cases(**kw):
        return {
            "fc2_fwd": lambda: K.linear(x, w2, out, bias=b2, res=res, res_scale=0.5, drop_p=0.1, drop_seed=3, **kw),
            "fc1_dx": lambda: K.gemm(dz, w1, dln, **kw),
        }
    ref = {}
    for tile in [(0, 0), (64, 64), (128, 64), (64, 128), (128, 128)]:
        for name, fn in cases(tile=tile if tile[0] else None).items():
            us = graph_time(fn)
            o = (out if name == "fc2_fwd" else dln).float()
            if tile == (0, 0):
                ref[name] = o.clone()
            same = bool(torch.equal(o, ref[name]))
            print(json.dumps({"case": name, "M": M, "N": D, "K": F, "tile": f"{tile[0]}x{tile[1]}" if tile[0] else "planner",
                              "us": round(us, 2), "bit_identical_to_planner": same}), flush=True)
    # K split in slices (fixed-order fp32 reduction that applies the epilogue): fewer k steps
    # per workgroup, more workgroups
    for sp in (2, 4):
        split_cases = {
            "fc2_fwd": lambda: K.gemm(x, w2.t(), out, bias=b2, res=res, res_scale=0.5, drop_p=0.1, drop_seed=3,
                                      split_k=sp),
            "fc1_dx": lambda: K.gemm(dz, w1, dln, split_k=sp),
        }
        for name, fn in split_cases.items():
            us = graph_time(fn)
            o = (out if name == "fc2_fwd" else dln).float()
            err = ((o - ref[name]).abs().max() / ref[name].abs().max()).item()
            print(json.dumps({"case": name, "M": M, "N": D, "K": F, "tile": f"planner split {sp}",
                              "us": round(us, 2), "rel_err_vs_unsplit": err}), flush=True)
    # ring stage depth: 32-deep (64-B row segments per operand row and stage) vs 64-deep (128 B)
    for ks in (1, 2):
        for name, fn in cases(ksub=ks).items():
            us = graph_time(fn)
            o = (out if name == "fc2_fwd" else dln).float()
            print(json.dumps({"case": name, "M": M, "N": D, "K": F, "tile": f"planner ksub {ks}", "us": round(us, 2),
                              "bit_identical_to_planner": bool(torch.equal(o, ref[name]))}), flush=True)


if __name__ == "__main__":
    main()
