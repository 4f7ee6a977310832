"""Times lasr_conv1_fwd / lasr_conv1_bwd (subsampling conv1, 1 -> C channels, 3x3 stride 2, bf16
channels-last y1) and prints a hash of the forward output, so that library builds
(LITEASR_HIP_LIB) compare bit for bit.  HBM bytes: y1 written (fwd) / dy1 read (bwd).
Usage: python tools/conv1_bench.py [B T F C]   (default: the small and large configs, C 256 / 512)"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


shapes = [tuple(int(v) for v in sys.argv[1:5])] if len(sys.argv) > 4 else [(32, 1000, 80, 256), (32, 1000, 80, 512)]
for B, T, F, C in shapes:
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B, T, F, device=dev, generator=g)
    w = torch.randn(C, 9, device=dev, generator=g) * 0.3
    b = torch.randn(C, device=dev, generator=g) * 0.1
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    y1 = torch.empty(B, T1, F1, C, dtype=torch.bfloat16, device=dev)
    K.conv1_fwd(x, w, b, y1)
    torch.cuda.synchronize()
    h = hashlib.sha256(y1.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    dy1 = torch.randn(B, T1, F1, C, device=dev, generator=g).bfloat16()
    dw, db = torch.zeros(C, 9, device=dev), torch.zeros(C, device=dev)
    nb = y1.numel() * 2
    tf = timeit(lambda: K.conv1_fwd(x, w, b, y1))
    tb = timeit(lambda: K.conv1_bwd(x, dy1, dw, db))
    print(json.dumps({"shape": [B, T1, F1, C], "conv1_fwd_us": round(tf, 1), "fwd_GBps": round(nb / tf / 1e3, 1),
                      "bwd_us": round(tb, 1), "bwd_GBps": round(nb / tb / 1e3, 1), "hash": h}), flush=True)
