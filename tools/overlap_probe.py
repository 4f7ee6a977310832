"""Probe: how much of a weight-gradient GEMM hides behind the input-gradient GEMM of the
same layer when they run on two streams (both captured in one hipGraph) vs one stream."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd._native import ACT_SWISH  # noqa: E402


def graph_time(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev, bf = "cuda", torch.bfloat16
    M, D, F = 7968, 256, 2048
    ln = torch.randn(M, D, device=dev).to(bf)
    z = torch.randn(M, F, device=dev).to(bf)
    h = torch.randn(M, F, device=dev).to(bf)
    gb = torch.randn(M, D, device=dev).to(bf)
    W1 = (torch.randn(F, D, device=dev) * 0.05).to(bf)
    W2 = (torch.randn(D, F, device=dev) * 0.02).to(bf)
    gW1 = torch.zeros(F, D, device=dev)
    gW2 = torch.zeros(D, F, device=dev)
    gb1 = torch.zeros(F, device=dev)
    gb2 = torch.zeros(D, device=dev)
    dz = torch.empty(M, F, dtype=bf, device=dev)
    dln = torch.empty(M, D, dtype=bf, device=dev)
    side = torch.cuda.Stream()

    def dx_chain():
        K.gemm(gb, W2, dz, aux=z, aux_act=ACT_SWISH, drop_p=0.1, drop_seed=3)
        K.gemm(dz, W1, dln)

    def dw_pair():
        K.gemm(gb.t(), h, gW2, beta=1.0, split_k=0, rowsum=gb2)
        K.gemm(dz.t(), ln, gW1, beta=1.0, split_k=0, rowsum=gb1)

    def seq():
        dx_chain()
        dw_pair()

    def ovl():
        # dW2 needs only gb and h: start it on the side stream before the dX chain
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            K.gemm(gb.t(), h, gW2, beta=1.0, split_k=0, rowsum=gb2)
        K.gemm(gb, W2, dz, aux=z, aux_act=ACT_SWISH, drop_p=0.1, drop_seed=3)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            K.gemm(dz.t(), ln, gW1, beta=1.0, split_k=0, rowsum=gb1)
        K.gemm(dz, W1, dln)
        cur.wait_stream(side)

    for name, fn in [("dx chain alone", dx_chain), ("dw pair alone", dw_pair), ("sequential", seq),
                     ("two streams", ovl)]:
        print(f"{name:16s} {graph_time(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
