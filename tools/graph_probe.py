"""Host-bound probe: eager step wall time vs host enqueue time vs a hipGraph replay of
the same step (torch.cuda.graph capture of fwd + loss + bwd + clip + Adam).

    python tools/graph_probe.py [--config small] [--steps 10]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="small")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfgd = bench.CONFIGS[args.config]
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.optims.noam import Noam, NoamConfig

    torch.manual_seed(42)
    model = bench.build(cfgd, "bf16", 0.1, dev)
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=bench.V, smoothing=0.1, ctc_weight=cfgd["w"]))
    opt = Noam(model.parameters(), NoamConfig(model_dim=cfgd["d"]))
    batch = bench.synthetic(cfgd, 0, dev)

    def step():
        loss = crit(model, *batch)
        loss.backward()
        opt.clip_and_step(5.0)
        opt.zero_grad()
        return loss

    out = {}
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    out["eager_ms"] = t_wall / args.steps * 1e3
    out["eager_host_enqueue_ms"] = t_host / args.steps * 1e3

    # graph capture of one whole step on a side stream
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    t0 = time.perf_counter()
    with torch.cuda.graph(g):
        static_loss = step()
    torch.cuda.synchronize()
    out["capture_s"] = time.perf_counter() - t0
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.replay()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    out["graph_ms"] = t_wall / args.steps * 1e3
    out["graph_host_ms"] = t_host / args.steps * 1e3
    out["graph_loss"] = static_loss.item()
    out["opt_state"] = opt.device_state()
    out["utt_per_s_graph"] = cfgd["B"] / (out["graph_ms"] * 1e-3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
