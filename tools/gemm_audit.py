"""Planner audit: every distinct lasr_gemm call of one eager training step (bench.py's model
and batch at --config), replayed alone under each LDS-DMA tile the kernel takes and timed as
a replayed hipGraph (tile_ab.py's graph_time).  One JSON line per call signature: the
planner's tile and time, the best tile and time, and how many times the step issues it.
Grouped (deferred) weight gradients are not audited here (their own sweeps).  Tile shape does
not change any output's summation order (tests/test_fusions_gpu.py, tile_ab.py); outputs are
not compared here.
    python tools/gemm_audit.py [--config small|large|long] [--min-us 5]"""

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402
from tools.tile_ab import graph_time  # noqa: E402

TILES = [(64, 64), (128, 64), (64, 128), (128, 128), (128, 256), (256, 128)]


def sig(a, b, c, kw):
    def t(x):
        return None if x is None else (tuple(x.shape), tuple(x.stride()), str(x.dtype))
    def v_(v):
        if isinstance(v, torch.Tensor):
            return t(v)
        if v is None or isinstance(v, (int, float, bool, str)):
            return v
        return type(v).__name__
    rest = tuple(sorted((k, v_(v)) for k, v in kw.items()))
    return (t(a), t(b), t(c), rest)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="small")
    ap.add_argument("--min-us", type=float, default=4.0)
    args = ap.parse_args()
    cfgd = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig

    net = bench.build(cfgd, "bf16", 0.1, dev)
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=bench.V, smoothing=0.1, ctc_weight=cfgd["w"]))
    batch = bench.synthetic(cfgd, 0, dev)
    calls, order = {}, []
    real = K.gemm

    def rec(a, b, c, **kw):
        if not kw.get("group") and not kw.get("plan_only"):
            s = sig(a, b, c, kw)
            if s not in calls:
                calls[s] = [(a, b, c, dict(kw)), 0]
                order.append(s)
            calls[s][1] += 1
        return real(a, b, c, **kw)

    K.gemm = rec
    try:
        loss = crit(net, *batch)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        K.gemm = real
    print(json.dumps({"config": args.config, "distinct_calls": len(order),
                      "calls": sum(v[1] for v in calls.values())}), flush=True)
    for s in order:
        (a, b, c, kw), n = calls[s]
        kw = {k: v for k, v in kw.items() if k not in ("tile", "ksub")}
        try:
            pm, pn, sp = K.gemm_plan(a, b, c, **kw)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"sig": str(s)[:200], "error": str(e)[:160]}), flush=True)
            continue
        t0 = graph_time(lambda: K.gemm(a, b, c, **kw))
        if t0 < args.min_us:
            continue
        res = {}
        for tl in TILES:
            try:
                res[f"{tl[0]}x{tl[1]}"] = round(graph_time(lambda: K.gemm(a, b, c, tile=tl, **kw)), 2)
            except Exception:  # noqa: BLE001 -- a tile the operands' layout or epilogue does not take
                pass
        best = min(res, key=res.get) if res else None
        M, Kd = a.shape[-2], a.shape[-1]
        Nn = b.shape[-1]
        batch_n = c.numel() // (M * Nn)
        print(json.dumps({"M": M, "N": Nn, "K": Kd, "batch": batch_n, "per_step": n,
                          "akc": a.stride(-1) == 1, "bkc": b.stride(-2) == 1,
                          "epi": sorted(k for k, v in kw.items() if v is not None and v is not False and
                                        k not in ("alpha", "res_scale", "beta", "drop_seed", "split_k") or
                                        (k == "split_k" and v != 1)),
                          "planner": f"{pm}x{pn}" + (f" split {sp}" if sp > 1 else ""), "planner_us": round(t0, 2),
                          "best": best, "best_us": res.get(best), "tiles": res}), flush=True)


if __name__ == "__main__":
    main()
