"""GEMM tile sweep at the step's shapes (GPU box), timed without host overhead: each case's
launches are captured into a hipGraph (20 per replay) and the replays timed with events.

    python tools/gemm_graph_bench.py [case-substring ...]

For every case: the planner's tile, then each forced tile (lasr_gemm_force_tile), us per
launch and TFLOP/s.  Used to choose gemm_plan's tiles; not part of the product."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C

import torch

from liteasr_amd import _native as N
from liteasr_amd import kernels as K
from liteasr_amd._native import ACT_GATE, ACT_SWISH

TILES = [(0, 0), (64, 64), (128, 64), (64, 128), (128, 128), (256, 128), (128, 256), (256, 256)]
REPS = 20


def graph_time(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(REPS):
                fn()
    torch.cuda.synchronize()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / (n * REPS) * 1e3


def make(M, N_, Kd, layout, out, batch=1, **kw):
    dev = "cuda"
    bs = (batch,) if batch > 1 else ()
    if layout == "nt":
        a = torch.randn(*bs, M, Kd, device=dev).bfloat16()
        b = torch.randn(*bs, N_, Kd, device=dev).bfloat16().transpose(-1, -2)
    elif layout == "nn":
        a = torch.randn(*bs, M, Kd, device=dev).bfloat16()
        b = torch.randn(*bs, Kd, N_, device=dev).bfloat16()
    else:  # tn
        a = torch.randn(*bs, Kd, M, device=dev).bfloat16().transpose(-1, -2)
        b = torch.randn(*bs, Kd, N_, device=dev).bfloat16()
    c = torch.zeros(*bs, M, N_, device=dev, dtype=out)
    extra = {}
    if kw.get("bias"):
        extra["bias"] = torch.randn(N_, device=dev)
    if kw.get("swish"):
        extra["act"] = ACT_SWISH
        extra["zout"] = torch.empty(M, N_, device=dev, dtype=out)
    if kw.get("aux"):
        extra["aux"], extra["aux_act"] = torch.randn(M, N_, device=dev).bfloat16(), ACT_SWISH
    if kw.get("gate"):  # FFN dX through the stored gate (functional.ffn_backward)
        extra["aux"], extra["aux_act"], extra["alpha"] = torch.rand(M, N_, device=dev).bfloat16(), ACT_GATE, 1.11
    if kw.get("gatez"):  # FFN fc1 forward storing the gate (functional.ffn_forward)
        extra["act"], extra["zout_mode"] = ACT_SWISH, 1
        extra["zout"] = torch.empty(M, N_, device=dev, dtype=out)
    if kw.get("res"):
        extra["res"] = torch.randn(M, N_, device=dev)
    if kw.get("drop"):
        extra["drop_p"], extra["drop_seed"] = 0.1, 7
    if kw.get("split"):
        extra["split_k"] = 0
        extra["beta"] = 1.0
    return a, b, c, extra


CASES = [
    ("square4096", 4096, 4096, 4096, "nt", torch.bfloat16, 1, {}),
    ("fc1 fwd bias+swish+z+drop", 7968, 2048, 256, "nt", torch.bfloat16, 1,
     dict(bias=1, swish=1, drop=1)),
    ("fc1 plain", 7968, 2048, 256, "nt", torch.bfloat16, 1, {}),
    ("fc1 fwd gate (prod)", 7968, 2048, 256, "nt", torch.bfloat16, 1, dict(bias=1, gatez=1, drop=1)),
    ("dX fc2 gate (prod)", 7968, 2048, 256, "nn", torch.bfloat16, 1, dict(gate=1)),
    ("dX fc2 aux+drop (nn)", 7968, 2048, 256, "nn", torch.bfloat16, 1, dict(aux=1, drop=1)),
    ("dX fc2 aux+drop (nt)", 7968, 2048, 256, "nt", torch.bfloat16, 1, dict(aux=1, drop=1)),
    ("dX fc1 (nt K2048)", 7968, 256, 2048, "nt", torch.bfloat16, 1, {}),
    ("dX dd (nt)", 7968, 256, 256, "nt", torch.bfloat16, 1, {}),
    ("dd bias (nt)", 7968, 256, 256, "nt", torch.bfloat16, 1, dict(bias=1)),
    ("dd res f32 (nt)", 7968, 256, 256, "nt", torch.float32, 1, dict(bias=1, res=1)),
    ("dX dd (nn)", 7968, 256, 256, "nn", torch.bfloat16, 1, {}),
    ("qkv (nt)", 7968, 768, 256, "nt", torch.bfloat16, 1, dict(bias=1)),
    ("fc2 fwd res f32 (nt K2048)", 7968, 256, 2048, "nt", torch.float32, 1, dict(bias=1, res=1, drop=1)),
    ("dX fc1 (nn K2048)", 7968, 256, 2048, "nn", torch.bfloat16, 1, {}),
    ("ctc head (nt)", 7968, 4240, 256, "nt", torch.bfloat16, 1, dict(bias=1)),
    ("att scores b128 f32", 249, 249, 64, "nt", torch.float32, 128, {}),
    ("conv2 fwd (nt)", 151392, 256, 2304, "nt", torch.bfloat16, 1, dict(bias=1)),
    ("dW fc1 (tn split)", 2048, 256, 7968, "tn", torch.float32, 1, dict(split=1)),
    ("dW dd (tn split)", 256, 256, 7968, "tn", torch.float32, 1, dict(split=1)),
    ("dW conv2 (tn split)", 256, 2304, 151392, "tn", torch.float32, 1, dict(split=1)),
]


def main():
    lib = N.load()
    sel = [x for x in sys.argv[1:] if x != "--cold"]
    # --cold: rotate over 6 operand/output sets (> the 256 MB MALL at the FFN shapes), as
    # inside a training step where a GEMM's outputs do not stay cache-resident
    nbuf = 6 if "--cold" in sys.argv[1:] else 1
    for name, M, N_, Kd, layout, out, batch, kw in CASES:
        if sel and not any(x in name for x in sel):
            continue
        sets = [make(M, N_, Kd, layout, out, batch, **kw) for _ in range(nbuf)]
        a, b, c, extra = sets[0]
        flops = 2.0 * M * N_ * Kd * batch
        res = []
        for tm, tn in TILES:
            if tm and (tm > 2 * M + 64 or tn > 2 * N_ + 64):
                continue
            N.call("lasr_gemm_force_tile", tm, tn)
            plan = K.gemm_plan(a, b, c, **extra)
            ctr = [0]

            def run():
                a_, b_, c_, e_ = sets[ctr[0] % nbuf]
                ctr[0] += 1
                K.gemm(a_, b_, c_, **e_)

            us = graph_time(run)
            res.append((f"{plan[0]}x{plan[1]}/s{plan[2]}" + ("*" if tm == 0 else ""), us))
        N.call("lasr_gemm_force_tile", 0, 0)
        best = min(r[1] for r in res)
        cells = "  ".join(f"{t}:{u:7.1f}" for t, u in res)
        print(f"{name:28s} best {best:7.1f} us {flops / best / 1e6:7.1f} TF/s | {cells}", flush=True)
        del a, b, c, extra, sets
    _ = lib, C


if __name__ == "__main__":
    main()
