"""Ring-stage depth sweep of the LDS-DMA GEMM (GPU box): for the step's GEMM shapes, every
tile with 32-deep (ksub 1) and 64-deep (ksub 2) ring stages, graph-timed over rotating cold
operand sets (tools/gemm_graph_bench.py), plus a bit-exactness check of ksub 2 against
ksub 1 (same k order inside every accumulator, so the outputs must be identical).

    python tools/ksub_sweep.py [case-substring ...]

Used to choose gemm_plan's ring depth; not part of the product."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from liteasr_amd import _native as N  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402
from tools.gemm_graph_bench import CASES, graph_time, make  # noqa: E402

TILES = [(0, 0), (64, 64), (128, 64), (64, 128), (128, 128), (128, 256)]
SKIP = ("square4096", "att scores", "conv2", "dW conv2")


def main():
    N.load()
    sel = sys.argv[1:]
    nbuf = 6
    for name, M, N_, Kd, layout, out, batch, kw in CASES:
        if any(s in name for s in SKIP) or (sel and not any(x in name for x in sel)):
            continue
        sets = [make(M, N_, Kd, layout, out, batch, **kw) for _ in range(nbuf)]
        flops = 2.0 * M * N_ * Kd * batch
        res, exact = [], True
        for tm, tn in TILES:
            if tm and (tm > 2 * M + 64 or tn > 2 * N_ + 64):
                continue
            N.call("lasr_gemm_force_tile", tm, tn)
            outs = []
            for ks in (1, 2):
                N.call("lasr_gemm_force_ksub", ks)
                plan = K.gemm_plan(sets[0][0], sets[0][1], sets[0][2], **sets[0][3])
                a, b, c, e = sets[0]
                c.zero_()
                K.gemm(a, b, c, **e)
                torch.cuda.synchronize()
                outs.append(c.clone())
                ctr = [0]

                def run():
                    a_, b_, c_, e_ = sets[ctr[0] % nbuf]
                    ctr[0] += 1
                    K.gemm(a_, b_, c_, **e_)

                us = graph_time(run)
                res.append((f"{plan[0]}x{plan[1]}/s{plan[2]}/k{ks}" + ("*" if tm == 0 else ""), us))
            if not torch.equal(outs[0], outs[1]):
                exact = False
        N.call("lasr_gemm_force_tile", 0, 0)
        N.call("lasr_gemm_force_ksub", 0)
        best = min(res, key=lambda r: r[1])
        cells = "  ".join(f"{t}:{u:6.1f}" for t, u in res)
        print(f"{name:28s} best {best[0]} {best[1]:6.1f} us {flops / best[1] / 1e6:6.1f} TF/s "
              f"exact={exact} | {cells}", flush=True)
        del sets


if __name__ == "__main__":
    main()
