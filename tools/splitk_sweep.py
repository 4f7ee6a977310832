"""Big tiles with a K split for the step's N = d, K = d_ff GEMMs (FFN fc2 forward with the fp32
residual epilogue, FFN fc1 input gradient): each (tile, split) forced through the per-call tile
override and an explicit split_k (the fixed-order split-K reduction applies the epilogue), timed
as a replayed hipGraph of 50 launches (tile_ab.graph_time).  The question: do 256-row tiles,
which read fewer L2 -> LDS bytes per flop than the planner's 64 x 64 / 128 x 64, win once a K
split fills the chip?  One JSON line per (case, tile, split); the error column is relative to
the planner's unsplit output.
    python tools/splitk_sweep.py [M N K]"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402
from tools.tile_ab import graph_time  # noqa: E402


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
            "fc2_fwd": (lambda: K.linear(x, w2, out, bias=b2, res=res, res_scale=0.5, drop_p=0.1, drop_seed=3, **kw),
                        out),
            "fc1_dx": (lambda: K.gemm(dz, w1, dln, **kw), dln),
        }

    ref = {}
    for name, (fn, o) in cases().items():
        us = graph_time(fn)
        ref[name] = o.float().clone()
        print(json.dumps({"case": name, "M": M, "N": D, "K": F, "tile": "planner", "split": 1, "us": round(us, 2)}),
              flush=True)
    for tile in [(128, 64), (128, 128), (128, 256), (256, 128), (256, 256)]:
        if tile[1] > D:
            continue
        for sp in (1, 2, 4, 8):
            ntiles = ((M + tile[0] - 1) // tile[0]) * ((D + tile[1] - 1) // tile[1])
            if sp > 1 and ntiles * sp > 1024:
                continue
            kw = {"tile": tile}
            if sp > 1:
                kw["split_k"] = sp
            for name, (fn, o) in cases(**kw).items():
                try:
                    us = graph_time(fn)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"case": name, "tile": f"{tile[0]}x{tile[1]}", "split": sp, "error": str(e)[:120]}),
                          flush=True)
                    continue
                err = ((o.float() - ref[name]).abs().max() / ref[name].abs().max()).item()
                print(json.dumps({"case": name, "M": M, "N": D, "K": F, "tile": f"{tile[0]}x{tile[1]}", "split": sp,
                                  "workgroups": ntiles * sp, "us": round(us, 2), "rel_err_vs_planner": err}),
                      flush=True)


if __name__ == "__main__":
    main()
