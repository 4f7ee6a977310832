"""Time lasr_conv2_gemm (fwd / dW / dX) at the small config's subsampling size, and dW
under tile / split / ring-depth variants (lasr_gemm_force_tile / _force_split hooks).
Usage: python tools/conv2_bench.py [B T F C]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from liteasr_amd import _native as N  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402

B, T, Fd, C = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (32, 1000, 80, 256)
T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
M2 = B * T2 * F2
dev = "cuda"
y1 = torch.relu(torch.randn(B, T1, F1, C, device=dev)).bfloat16()
w2p = (torch.randn(C, 9 * C, device=dev) * 0.02).bfloat16()
b2 = torch.zeros(C, device=dev)
y2 = torch.empty(M2, C, device=dev, dtype=torch.bfloat16)
dy2 = torch.zeros(K.conv2_dy2_rows(M2), C, device=dev, dtype=torch.bfloat16)
dy2[:M2] = torch.randn(M2, C, device=dev).bfloat16()
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


out = {"shape": [B, T1, F1, C], "gflop": flop / 1e9}
out["fwd_us"] = timeit(lambda: K.conv2_fwd(y1, w2p, b2, y2))
out["dx_us"] = timeit(lambda: K.conv2_dx(dy2, w2p, y1, dy1))
lib = N.load()
for tile in (128, 256):
    for split in (0, 4, 8, 16, 32):
        for stages in (0, 4):
            if tile == 256 and stages:
                continue
            N.call("lasr_gemm_force_tile", tile if tile == 256 else 0, tile if tile == 256 else 0)
            N.call("lasr_gemm_force_split", split, stages)
            try:
                out[f"dw_t{tile}_s{split}_r{stages}_us"] = timeit(lambda: K.conv2_dw(dy2, y1, dw, rowsum=db))
            except Exception as e:  # noqa: BLE001
                out[f"dw_t{tile}_s{split}_r{stages}_us"] = str(e)[:80]
N.call("lasr_gemm_force_tile", 0, 0)
N.call("lasr_gemm_force_split", 0, 0)
out["dw_us"] = timeit(lambda: K.conv2_dw(dy2, y1, dw, rowsum=db))
for k in list(out):
    if k.endswith("_us") and isinstance(out[k], float):
        out[k] = round(out[k], 1)
print(json.dumps(out, indent=1))
