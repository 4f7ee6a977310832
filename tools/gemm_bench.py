"""GEMM microbenchmark (GPU box): TFLOP/s of lasr_gemm variants at the step's shapes."""

import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from liteasr_amd import kernels as K
from liteasr_amd._native import ACT_SWISH


TORCH_REF = os.environ.get("GEMM_TORCH_REF", "1") == "1"


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def case(name, M, N, Kd, layout="nt", out=torch.bfloat16, **kw):
    dev = "cuda"
    if layout == "nt":
        a = torch.randn(M, Kd, device=dev).bfloat16()
        b = torch.randn(N, Kd, device=dev).bfloat16().t()
    elif layout == "nn":
        a = torch.randn(M, Kd, device=dev).bfloat16()
        b = torch.randn(Kd, N, device=dev).bfloat16()
    else:  # tn: A = X^T (M-contig), B N-contig
        a = torch.randn(Kd, M, device=dev).bfloat16().t()
        b = torch.randn(Kd, N, device=dev).bfloat16()
    c = torch.empty(M, N, device=dev, dtype=out)
    extra = {}
    if kw.get("bias"):
        extra["bias"] = torch.randn(N, device=dev)
    if kw.get("swish"):
        extra["act"] = ACT_SWISH
        extra["zout"] = torch.empty(M, N, device=dev, dtype=out)
    if kw.get("aux"):
        extra["aux"], extra["aux_act"] = torch.randn(M, N, device=dev).bfloat16(), ACT_SWISH
    if kw.get("res"):
        extra["res"] = torch.randn(M, N, device=dev)
    if kw.get("drop"):
        extra["drop_p"], extra["drop_seed"] = 0.1, 7
    if kw.get("split"):
        extra["split_k"] = kw.get("nsplit", 0)
        extra["beta"] = 1.0
    us = timeit(lambda: K.gemm(a, b, c, **extra))
    tf = 2 * M * N * Kd / us / 1e6
    ref = ""
    if TORCH_REF and not kw.get("split"):
        # hipBLASLt (torch.matmul) on the same operands, plain product, same output dtype
        cc = torch.empty(M, N, device=dev, dtype=out)
        ut = timeit(lambda: torch.matmul(a, b, out=cc) if out == torch.bfloat16 else cc.copy_(a @ b))
        ref = f"   torch {ut:8.1f} us"
    print(f"{name:38s} M={M:6d} N={N:5d} K={Kd:5d} {layout}  {us:8.1f} us  {tf:7.1f} TF/s{ref}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "fc1":
        for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 1):
            case("fc1 plain", 7968, 2048, 256, "nt")
        sys.exit(0)
    case("square 4096 nt f32out", 4096, 4096, 4096, "nt", torch.float32)
    case("square 4096 nt bf16out", 4096, 4096, 4096, "nt")
    case("fc1 plain", 7968, 2048, 256, "nt")
    case("fc1 bias", 7968, 2048, 256, "nt", bias=True)
    case("fc1 bias+swish+z", 7968, 2048, 256, "nt", bias=True, swish=True)
    case("fc1 bias+swish+z+drop", 7968, 2048, 256, "nt", bias=True, swish=True, drop=True)
    case("fc2 (K=2048) f32out", 7968, 256, 2048, "nt", torch.float32)
    case("qkv", 7968, 768, 256, "nt")
    case("ctc head", 7968, 4233, 256, "nt")
    case("dX fc2 (nn)", 7968, 2048, 256, "nn")
    case("dX fc2 + swish-grad aux + drop (nn)", 7968, 2048, 256, "nn", aux=True, drop=True)
    case("fc2 + bias + res + drop f32out", 7968, 256, 2048, "nt", torch.float32, bias=True, res=True, drop=True)
    case("dX fc1 (nn, K=2048)", 7968, 256, 2048, "nn")
    case("dW fc1 (tn split)", 2048, 256, 7968, "tn", torch.float32, split=True)
    for s in (4, 8, 16, 32):
        case(f"dW fc1 (tn split {s})", 2048, 256, 7968, "tn", torch.float32, split=True, nsplit=s)
    case("dW fc2 (tn split)", 256, 2048, 7968, "tn", torch.float32, split=True)
    case("dW conv2 (tn split)", 256, 2304, 151392, "tn", torch.float32, split=True)
    case("conv2 fwd (nt)", 151392, 256, 2304, "nt")
