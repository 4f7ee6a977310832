"""Tile / ring-depth sweep of the FFN fc1 GEMMs at a config's shape (M = B*T', N = ff, K = d):
the forward (bias + Swish + stored gate + dropout) and the backward dz (x stored gate), each
tile forced through the per-call override, timed as a replayed hipGraph of 50 launches, with
an output hash (a tile never changes an output's summation order: the hashes must agree).
    python tools/fc1_tile_sweep.py [M F D]"""

import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd._native import ACT_GATE, ACT_SWISH  # noqa: E402
from tools.epi_ab import graph_us  # noqa: E402


def main():
    M, F, D = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (7968, 2048, 256)
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    dev = "cuda"
    ln = torch.randn(M, D, device=dev).bfloat16()
    w1 = (torch.randn(F, D, device=dev) * 0.05).bfloat16()
    w2 = (torch.randn(D, F, device=dev) * 0.05).bfloat16()
    b1 = torch.randn(F, device=dev) * 0.1
    h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    g = torch.empty_like(h)
    gb = torch.randn(M, D, device=dev).bfloat16()
    dz = torch.empty_like(h)

    def hsh(*ts):
        torch.cuda.synchronize()
        m = hashlib.sha256()
        for t in ts:
            m.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
        return m.hexdigest()[:16]

    for tile in [None, (128, 128), (256, 128), (128, 256), (64, 256), (256, 256), (64, 128), (128, 64)]:
        for ks in (0, 1, 2):
            kw = dict(tile=tile, ksub=ks)
            cases = {
                "fc1_fwd": (lambda: K.linear(ln, w1, h, bias=b1, act=ACT_SWISH, zout=g, zout_mode=1, drop_p=0.1,
                                             drop_seed=11, **kw), (h, g)),
                "fc1_dz": (lambda: K.gemm(gb, w2, dz, alpha=K.dropout_scale(0.1), aux=g, aux_act=ACT_GATE, **kw), (dz,)),
            }
            for name, (fn, outs) in cases.items():
                try:
                    fn()
                    hv = hsh(*outs)
                    us = graph_us(fn)
                except Exception as e:  # a tile / depth the planner rejects for this shape
                    print(json.dumps({"case": name, "tile": str(tile), "ksub": ks, "error": str(e)[:120]}), flush=True)
                    continue
                plan = K.gemm_plan(ln if name == "fc1_fwd" else gb, (w1.t() if name == "fc1_fwd" else w2),
                                   h if name == "fc1_fwd" else dz, flags=True, tile=tile, ksub=ks)
                print(json.dumps({"case": name, "M": M, "N": F, "K": D, "tile": str(tile), "ksub": ks,
                                  "plan": plan, "us": round(us, 2), "hash": hv}), flush=True)


if __name__ == "__main__":
    main()
