"""Times lasr_conv1_fwd (the subsampling's first 3x3 stride-2 convolution + ReLU, bf16 output)
at the small / large configs' shapes and prints a hash of its output, so that library builds
(LITEASR_HIP_LIB) compare bit for bit."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
for C in (256, 512):
    B, T, F = 32, 1000, 80
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B, T, F, device=dev, generator=g)
    w = torch.randn(C, 9, device=dev, generator=g) * 0.3
    b = torch.randn(C, device=dev, generator=g) * 0.1
    T1, F1 = (T - 3) // 2 + 1, (F - 3) // 2 + 1
    y1 = torch.empty(B, T1, F1, C, dtype=torch.bfloat16, device=dev)
    K.conv1_fwd(x, w, b, y1)
    torch.cuda.synchronize()
    h = hashlib.sha256(y1.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record(s)
        for _ in range(20):
            K.conv1_fwd(x, w, b, y1)
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
    print(json.dumps({"C": C, "conv1_fwd_us": round(best, 1), "GB_s": round(y1.numel() * 2 / best / 1e3, 1),
                      "hash": h}), flush=True)
