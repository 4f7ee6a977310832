"""Ceiling check: the step's hot GEMM shapes through torch.mm (hipBLASLt on this image) beside
our lasr_gemm with a plain epilogue (same operand layouts, bf16 in, fp32 accumulate), each timed
as a replayed hipGraph of `iters` launches.  One JSON line per shape.
    python tools/blaslt_ref.py"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402


def graph_time(fn, iters=50):
    for _ in range(3):
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
    dev = "cuda"
    gen = torch.Generator(device=dev).manual_seed(1)

    def rnd(*s):
        return torch.randn(*s, device=dev, generator=gen).bfloat16()

    M, D, F = 7968, 256, 2048
    shapes = [
        # name, A (M,K) view, B (K,N) view, out dtype
        ("fc1_dx  M7968 N256 K2048 NN", rnd(M, F), rnd(F, D), torch.bfloat16),
        ("fc2_fwd M7968 N256 K2048 NT", rnd(M, F), rnd(D, F).t(), torch.float32),
        ("fc1_fwd M7968 N2048 K256 NT", rnd(M, D), rnd(F, D).t(), torch.bfloat16),
        ("qkv_fwd M7968 N768 K256 NT", rnd(M, D), rnd(3 * D, D).t(), torch.bfloat16),
        ("o_dx    M7968 N256 K256 NN", rnd(M, D), rnd(D, D), torch.bfloat16),
        ("dW_fc1  M2048 N256 K7968 TN", rnd(M, F).t(), rnd(M, D), torch.float32),
        ("conv2   M151392 N256 K2304 NT", rnd(151392, 2304), rnd(256, 2304).t(), torch.bfloat16),
    ]
    for name, a, b, odt in shapes:
        Mm, Nn = a.shape[0], b.shape[1]
        Kk = a.shape[1]
        c = torch.empty(Mm, Nn, device=dev, dtype=odt)
        ours = graph_time(lambda: K.gemm(a, b, c))
        ref = c.float().clone()
        c2 = torch.empty(Mm, Nn, device=dev, dtype=torch.bfloat16)
        lt = graph_time(lambda: torch.mm(a, b, out=c2))  # bf16 output (fewer bytes than an fp32 one)
        torch.mm(a, b, out=c2)
        err = ((c2.float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * Mm * Nn * Kk
        byts = (Mm * Kk + Kk * Nn) * 2 + Mm * Nn * (4 if odt == torch.float32 else 2)
        print(json.dumps({"shape": name, "ours_us": round(ours, 2), "hipblaslt_us": round(lt, 2),
                          "ours_TFLOPs": round(fl / ours / 1e6, 1), "lt_TFLOPs": round(fl / lt / 1e6, 1),
                          "ours_GBs": round(byts / ours / 1e3, 1), "lt_GBs": round(byts / lt / 1e3, 1),
                          "rel_diff": err}), flush=True)


if __name__ == "__main__":
    main()
