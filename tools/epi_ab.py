"""FFN fc1 GEMM epilogue timings at config 2's shape (M 7968, N 2048, K 256), each a replayed
hipGraph of 50 launches timed with HIP events: the forward (bias + Swish + stored gate +
dropout, zout_mode 1), the backward dz (x stored gate, dropout scale), and the plain GEMM of the
same shape.  Run once per library (LITEASR_HIP_LIB: e.g. the LASR_EXP ablation builds of
tools/gemm_exp.sh) -> one JSON line per case."""

import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd._native import ACT_GATE, ACT_SWISH  # noqa: E402


def graph_us(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


def main():
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    dev = "cuda"
    M, F, D = 7968, 2048, 256
    ln = torch.randn(M, D, device=dev).bfloat16()
    w1 = (torch.randn(F, D, device=dev) * 0.05).bfloat16()
    w2 = (torch.randn(D, F, device=dev) * 0.05).bfloat16()
    b1 = torch.randn(F, device=dev) * 0.1
    h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    g = torch.empty_like(h)
    gb = torch.randn(M, D, device=dev).bfloat16()
    dz = torch.empty_like(h)
    lib = os.path.basename(os.environ.get("LITEASR_HIP_LIB", "tree"))
    cases = {
        "fc1_fwd": lambda: K.linear(ln, w1, h, bias=b1, act=ACT_SWISH, zout=g, zout_mode=1, drop_p=0.1, drop_seed=11),
        "fc1_dz": lambda: K.gemm(gb, w2, dz, alpha=K.dropout_scale(0.1), aux=g, aux_act=ACT_GATE),
        "fc1_plain": lambda: K.linear(ln, w1, h, bias=b1),
    }
    def hsh(*ts):
        torch.cuda.synchronize()
        m = hashlib.sha256()
        for t in ts:
            m.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
        return m.hexdigest()[:16]

    outs = {"fc1_fwd": (h, g), "fc1_dz": (dz,), "fc1_plain": (h,)}
    for name, fn in cases.items():
        fn()
        hv = hsh(*outs[name])
        print(json.dumps({"lib": lib, "case": name, "us": round(graph_us(fn), 2), "hash": hv}), flush=True)


if __name__ == "__main__":
    main()
