"""Tile A/B for the encoder attention backward's two positional GEMMs over the head-major
pre-shift score gradient dBDh [H][B][T][ldS] (nets/functional.py attention backward):
  dqv = dBD @ p per (b, h)         batched B*H, M = T, N = d_k, K = T
  dp  = dBD^T @ qv per head        batched H, M = T, N = d_k, K = B*T (split over K)
each tile forced through the per-call override, timed as a replayed hipGraph (tile_ab.py's
graph_time); outputs compared with the planner's bit for bit.
    python tools/attn_gemm_tile_ab.py [small|large|long ...]"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd.nets.functional import _heads, ld_scores  # noqa: E402
from tools.tile_ab import graph_time  # noqa: E402

SHAPES = {"small": (32, 249, 4, 64), "large": (32, 249, 16, 32), "long": (8, 999, 4, 64)}


def run(name):
    B, T, H, dk = SHAPES[name]
    d, M = H * dk, B * T
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(3)
    ldS = ld_scores(T)
    dBDh = torch.randn(H, B, T, ldS, device=dev, generator=g).bfloat16()
    p = torch.randn(T, d, device=dev, generator=g).bfloat16()
    qv = torch.randn(M, d, device=dev, generator=g).bfloat16()
    p4 = p.view(T, H, dk).permute(1, 0, 2).unsqueeze(0).expand(B, H, T, dk)
    dqv = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    dp = torch.empty(T, d, device=dev, dtype=torch.bfloat16)

    def cases(**kw):
        return {
            "dqv": (lambda: K.gemm(dBDh.permute(1, 0, 2, 3)[..., :T], p4, _heads(dqv, B, T, H, dk), alpha=0.125,
                                   **kw), dqv),
            "dp": (lambda: K.gemm(dBDh.view(H, M, ldS)[..., :T].transpose(-1, -2), qv.view(M, H, dk).permute(1, 0, 2),
                                  dp.view(T, H, dk).permute(1, 0, 2), alpha=0.125, split_k=0, **kw), dp),
        }

    ref = {}
    for tile in [(0, 0), (64, 64), (128, 64), (64, 128), (128, 128)]:
        for case, (fn, out) in cases(tile=tile if tile[0] else None).items():
            try:
                us = graph_time(fn)
            except Exception as e:  # (a tile the operands' layout does not take)
                print(json.dumps({"shape": name, "case": case, "tile": f"{tile[0]}x{tile[1]}", "error": str(e)[:120]}),
                      flush=True)
                continue
            if tile == (0, 0):
                ref[case] = out.clone()
            print(json.dumps({"shape": name, "case": case, "B": B, "T": T, "H": H, "dk": dk,
                              "tile": f"{tile[0]}x{tile[1]}" if tile[0] else "planner", "us": round(us, 2),
                              "bit_identical_to_planner": bool(torch.equal(out, ref[case]))}), flush=True)


if __name__ == "__main__":
    for s in sys.argv[1:] or ["small", "large", "long"]:
        run(s)
