"""Time lasr_conv2_gemm (fwd / dW / dX) at a config's subsampling size and print hashes of
the outputs, so two processes (e.g. two library builds via LITEASR_HIP_LIB) can be compared bit for
bit (forward and data gradient: same k order per output, so equal hashes are expected).
Usage: python tools/conv2_bench.py [B T F C]"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from liteasr_amd import kernels as K  # noqa: E402

B, T, Fd, C = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (32, 1000, 80, 256)
T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
M2 = B * T2 * F2
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(5)
y1 = torch.relu(torch.randn(B, T1, F1, C, device=dev, generator=g)).bfloat16()
w2p = (torch.randn(C, 9 * C, device=dev, generator=g) * 0.02).bfloat16()
b2 = torch.randn(C, device=dev, generator=g) * 0.1
y2 = torch.empty(M2, C, device=dev, dtype=torch.bfloat16)
dy2 = torch.zeros(K.conv2_dy2_rows(M2), C, device=dev, dtype=torch.bfloat16)
dy2[:M2] = torch.randn(M2, C, device=dev, generator=g).bfloat16()
dw = torch.empty(C, 9 * C, device=dev)
db = torch.zeros(C, device=dev)
dy1 = torch.empty_like(y1)
flop = 2.0 * M2 * C * 9 * C


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


def h(t):
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


out = {"lib": os.environ.get("LITEASR_HIP_LIB", "tree"), "shape": [B, T1, F1, C], "gflop": round(flop / 1e9, 1)}
out["fwd_us"] = timeit(lambda: K.conv2_fwd(y1, w2p, b2, y2))
out["dx_us"] = timeit(lambda: K.conv2_dx(dy2, w2p, y1, dy1))


def dwf():
    db.zero_()
    K.conv2_dw(dy2, y1, dw, rowsum=db)


out["dw_us"] = timeit(dwf)
for k in ("fwd", "dx", "dw"):
    out[k + "_tflops"] = round(flop / out[k + "_us"] / 1e6, 1)
    out[k + "_us"] = round(out[k + "_us"], 1)
torch.cuda.synchronize()
out["hash_fwd"], out["hash_dx"] = h(y2), h(dy1)
ref = dw.double()
out["dw_absmax"] = ref.abs().max().item()
print(json.dumps(out), flush=True)
