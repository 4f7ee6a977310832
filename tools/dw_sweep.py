"""Split-K weight-gradient GEMM sweep (GPU box): tile x split x LDS ring depth at the
step's dW shapes (K = B*T' rows), graph-timed including the split-K reduce.
    python tools/dw_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from liteasr_amd import _native as N  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402
from tools.gemm_graph_bench import graph_time, make  # noqa: E402

SHAPES = [("ffn W1 2048x256", 2048, 256, 7968), ("ffn W2 256x2048", 256, 2048, 7968),
          ("Wo 256x256", 256, 256, 7968), ("pw1 512x256", 512, 256, 7968), ("qkv 768x256", 768, 256, 7968)]
TILES = [(0, 0), (64, 64), (64, 128), (128, 64), (128, 128)]


SPLITS = (0, 4, 8, 16)
STAGES = (0,)


def main():
    N.load()
    for name, M, N_, Kd in SHAPES:
        a, b, c, extra = make(M, N_, Kd, "tn", torch.float32, 1, split=1)
        flops = 2.0 * M * N_ * Kd
        rows = []
        for tm, tn in TILES:
            if tm > 2 * M or tn > 2 * N_:
                continue
            N.call("lasr_gemm_force_tile", tm, tn)
            for split in SPLITS:
                for stages in STAGES:
                    N.call("lasr_gemm_force_split", split, stages)
                    plan = K.gemm_plan(a, b, c, **extra)
                    us = graph_time(lambda: K.gemm(a, b, c, **extra))
                    rows.append((us, f"{plan[0]}x{plan[1]}/s{plan[2]}/S{stages or 3}" + ("*" if tm == 0 and split == 0 and stages == 0 else "")))
        N.call("lasr_gemm_force_tile", 0, 0)
        N.call("lasr_gemm_force_split", 0, 0)
        rows.sort()
        default = [r for r in rows if r[1].endswith("*")][0]
        print(f"{name:18s} default {default[1]} {default[0]:6.1f} us | best: " +
              "  ".join(f"{t} {u:6.1f}" for u, t in rows[:6]) + f"  ({flops / rows[0][0] / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
