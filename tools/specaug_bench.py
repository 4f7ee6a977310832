"""Time the batched SpecAugment kernels (csrc/specaug.hip) on a config-2 batch
(B 32, T 1000, F 80, reference default cfg) with HIP events, and the reference-style CPU
path (oracle restatement, one utterance at a time) for scale.  GPU box only."""

import json
import random
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from liteasr_amd.utils.transform.spec_augment import SpecAugment  # noqa: E402


def main():
    cfg = types.SimpleNamespace(time_warp=80, freq_mask=27, freq_mask_times=1, time_mask=100,
                                time_mask_times=1, inplace=True, replace_with_zero=False)
    sa = SpecAugment(cfg)
    B, T, F = 32, 1000, 80
    g = torch.Generator().manual_seed(0)
    xlens = torch.randint(int(0.95 * T), T + 1, (B,), generator=g)
    xlens[0] = T
    xs = torch.randn(B, T, F, generator=g).cuda()
    random.seed(0)
    np.random.seed(0)
    plans = [sa.plan_batch(xlens.tolist(), F).cuda() for _ in range(20)]
    xl = xlens.cuda()
    out = torch.empty_like(xs)
    from liteasr_amd import kernels as K

    for p in plans[:3]:
        K.spec_augment(xs, xl, p, out=out)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for p in plans:
        K.spec_augment(xs, xl, p, out=out)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / len(plans)
    # algorithmic bytes: the warp reads x once and writes out once (the masked regions, a
    # few % of the batch, are not counted)
    byts = 2 * B * T * F * 4
    t0 = time.perf_counter()
    from oracle import spec_augment_ref as O

    n = 0
    while time.perf_counter() - t0 < 5.0:
        x = xs[n % B, : int(xlens[n % B])].cpu().numpy()
        O.apply_plan(x, O.draw_plan(x.shape[0], F, cfg))
        n += 1
    cpu_utt_s = n / (time.perf_counter() - t0)
    print(json.dumps({"kernel": "spec_augment(warp+mask)", "batch": [B, T, F], "us_per_batch": round(us, 2),
                      "utt_per_s": round(B / us * 1e6), "GBps_algorithmic": round(byts / us / 1e3, 1),
                      "cpu_oracle_utt_per_s_1core": round(cpu_utt_s, 1)}))


if __name__ == "__main__":
    main()
