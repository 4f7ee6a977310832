"""Time lasr_conv1_fwd / lasr_conv1_bwd (subsampling conv1, 1 -> C channels, 3x3 stride 2) at
a config's size; HBM bytes: y1 written (fwd) / dy1 read (bwd), bf16 channels-last.
Usage: python tools/conv1_bench.py [B T F C]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from liteasr_amd import kernels as K  # noqa: E402

B, T, Fd, C = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (32, 1000, 80, 256)
T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
dev = "cuda"
x = torch.randn(B, T, Fd, device=dev)
w = torch.randn(C, 9, device=dev) * 0.3
b = torch.randn(C, device=dev) * 0.1
y1 = torch.empty(B, T1, F1, C, device=dev, dtype=torch.bfloat16)
dy1 = torch.randn(B, T1, F1, C, device=dev).bfloat16()
dw = torch.zeros(C, 9, device=dev)
db = torch.zeros(C, device=dev)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


nb = y1.numel() * 2
tf = timeit(lambda: K.conv1_fwd(x, w, b, y1))
tb = timeit(lambda: K.conv1_bwd(x, dy1, dw, db))
print(json.dumps({"shape": [B, T1, F1, C], "fwd_us": round(tf, 1), "fwd_GBps": round(nb / tf / 1e3, 1),
                  "bwd_us": round(tb, 1), "bwd_GBps": round(nb / tb / 1e3, 1)}))
