"""Why the N = d GEMMs run slower inside the step than in the isolated roofline replays
(fc2 forward + residual: ~26 us in the step trace vs ~21 us replayed alone at small): the same
fc2 launch timed as a replayed hipGraph under four cache states of its 32.6 MB A operand.
  hot      -- 50 launches on one A (A stays in the 256 MB MALL / partly in L2)
  rotate   -- 48 launches cycling over 12 distinct A buffers (391 MB, more than the MALL)
  producer -- fc1 forward writes A, then fc2 reads it (the step's order); minus fc1 alone
  flush    -- a 320 MB fill between launches; minus the fill alone
One JSON line per state.  python tools/cache_state_probe.py [M D F]"""

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
    h = torch.randn(M, D, device=dev, generator=g).bfloat16()
    w1 = (torch.randn(F, D, device=dev, generator=g) * D ** -0.5).bfloat16()
    w2 = (torch.randn(D, F, device=dev, generator=g) * F ** -0.5).bfloat16()
    b2 = torch.randn(D, device=dev, generator=g) * 0.02
    res = torch.randn(M, D, device=dev, generator=g)
    out = torch.empty(M, D, device=dev)
    xs = [torch.randn(M, F, device=dev, generator=g).bfloat16() for _ in range(12)]
    scratch = torch.empty(80 * 1024 * 1024, device=dev)  # 320 MB

    def fc2(x):
        K.linear(x, w2, out, bias=b2, res=res, res_scale=0.5, drop_p=0.1, drop_seed=3)

    def fc1(x):
        K.linear(h, w1, x)

    ab = {"bytes": M * F * 2 + D * F * 2 + 2 * M * D * 4}
    t_hot = graph_time(lambda: fc2(xs[0]), iters=48)
    it = iter(range(10 ** 9))
    t_rot = graph_time(lambda: fc2(xs[next(it) % 12]), iters=48)
    t_fc1 = graph_time(lambda: fc1(xs[0]), iters=48)
    t_pair = graph_time(lambda: (fc1(xs[0]), fc2(xs[0])), iters=48)
    t_fill = graph_time(lambda: scratch.fill_(1.0), iters=24)
    t_fill_fc2 = graph_time(lambda: (scratch.fill_(1.0), fc2(xs[0])), iters=24)
    rows = [("hot", t_hot), ("rotate", t_rot), ("producer", t_pair - t_fc1), ("flush", t_fill_fc2 - t_fill)]
    for name, us in rows:
        print(json.dumps({"state": name, "M": M, "N": D, "K": F, "fc2_us": round(us, 2),
                          "GBps_algorithmic": round(ab["bytes"] / us / 1e3, 1)}), flush=True)
    print(json.dumps({"fc1_alone_us": round(t_fc1, 2), "fill_320MB_us": round(t_fill, 2)}), flush=True)


if __name__ == "__main__":
    main()
