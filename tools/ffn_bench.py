"""Fused FFN chains (ffn.hip) vs the two-GEMM path at the step's shape (M 7968, D 256,
F 2048, Swish, dropout 0.1): average launch time with HIP events on the launch stream."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd._native import ACT_SWISH  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main(M=7968, D=256, F=2048, p=0.1):
    dev, bf = "cuda", torch.bfloat16
    ln = torch.randn(M, D, device=dev).to(bf)
    W1 = (torch.randn(F, D, device=dev) * 0.06).to(bf)
    W2 = (torch.randn(D, F, device=dev) * 0.02).to(bf)
    b1 = torch.randn(F, device=dev) * 0.1
    b2 = torch.randn(D, device=dev) * 0.1
    res = torch.randn(M, D, device=dev)
    gb = torch.randn(M, D, device=dev).to(bf)
    z, h = torch.empty(M, F, dtype=bf, device=dev), torch.empty(M, F, dtype=bf, device=dev)
    out = torch.empty(M, D, device=dev)
    dz, dx = torch.empty(M, F, dtype=bf, device=dev), torch.empty(M, D, dtype=bf, device=dev)

    def fwd_fused():
        K.ffn_fwd(ln, W1, b1, W2, b2, ACT_SWISH, p, 1, res, 0.5, p, 2, z, h, out)

    def fwd_two():
        K.linear(ln, W1, h, bias=b1, act=ACT_SWISH, zout=z, drop_p=p, drop_seed=1)
        K.linear(h, W2, out, bias=b2, res=res, res_scale=0.5, drop_p=p, drop_seed=2)

    def bwd_fused():
        K.ffn_bwd_dx(gb, W1, W2, z, ACT_SWISH, p, 1, dz, dx)

    def bwd_two():
        K.gemm(gb, W2, dz, aux=z, aux_act=ACT_SWISH, drop_p=p, drop_seed=1)
        K.gemm(dz, W1, dx)

    r = {k: timeit(f) for k, f in [("fwd_fused", fwd_fused), ("fwd_two_gemm", fwd_two), ("bwd_dx_fused", bwd_fused),
                                   ("bwd_dx_two_gemm", bwd_two)]}
    flops = 2 * 2 * M * D * F
    for k, us in r.items():
        print(f"{k:18s} M={M} D={D} F={F}: {us:8.2f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
    main(D=512)
