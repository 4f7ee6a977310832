"""Paraformer training-step throughput (SURVEY §8 f4 measurement) and the CIF kernels alone.

    python tools/paraformer_bench.py [--steps K --warmup W]

Model: Paraformer on the small encoder (12 x conformer d 256 / 4 heads / ff 2048, 6-layer
parallel decoder, V 4233), bf16, dropout 0.1, Noam; synthetic batch B 32, T 1000, L 40
(SURVEY §8d recipe).  A step = forward (incl. the first no-grad decoder pass, its argmax
copied to the host and the glancing sampler), ParaformerLoss, backward, clip + Noam/Adam.
Eager launches: the host sampling inside the forward (as in the reference) keeps the step
out of a captured graph.  Also times lasr_cif_fwd / lasr_cif_bwd (B 32, T' 249, D 256,
U 40) with HIP events, and the oracle's CPU integrate-and-fire loop (the reference's
algorithm, predictor.py:62-110) on the same sizes for scale."""

import argparse
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    from types import SimpleNamespace

    from liteasr_amd import kernels as K
    from liteasr_amd.criterions.paraformer_loss import ParaformerLoss, ParaformerLossConfig
    from liteasr_amd.models.paraformer import Paraformer, ParaformerConfig
    from liteasr_amd.optims.noam import Noam, NoamConfig
    from liteasr_amd.utils.cfg import resolve_self
    from liteasr_amd.utils.synthetic import synthetic_batch

    dev = torch.device("cuda", 0)
    V, B, T, L = 4233, 32, 1000, 40
    torch.manual_seed(42)
    random.seed(0)
    c = ParaformerConfig(input_dim=80, vocab_size=V, dropout_rate=0.1)
    resolve_self(c)
    c.enc_attn_dropout_rate = 0.0
    model = Paraformer(c).to(dev).train()
    crit = ParaformerLoss(ParaformerLossConfig(vocab_size=V))
    opt = Noam(model.parameters(), NoamConfig(model_dim=256))
    batch = [t.to(dev) for t in synthetic_batch(B, T, L, V, seed=1234)]

    def step():
        loss = crit(model, *batch)
        loss.backward()
        opt.clip_and_step(5.0)
        opt.zero_grad()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    out = {"workload": "Paraformer-small training step (fwd incl. no-grad pass + host glancing sampler, "
                       "ParaformerLoss, bwd, clip + Noam/Adam), eager, bf16",
           "B": B, "T": T, "L": L, "V": V, "ms_per_step": round(el * 1e3, 3),
           "utt_per_s": round(B / el, 2), "final_loss": round(loss.item(), 4)}
    # ---- CIF kernels alone
    Tp, D, U = 249, 256, L
    g = torch.Generator().manual_seed(0)
    z = (torch.randn(B * Tp, 1, generator=g) * 2).to(dev)
    h = torch.randn(B, Tp, D, generator=g).to(dev)
    plen = torch.full((B,), Tp, dtype=torch.int32, device=dev)
    ylen = torch.randint(L // 2, L + 1, (B,), generator=g).int().to(dev)
    M = B * Tp
    f = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
    st = SimpleNamespace(alpha=f(M), acc=f(M), fired=f(M, dt=torch.uint8), row=f(M, dt=torch.int32),
                         sum_alpha=f(B), mae=f(B), out=f(B, U, D))
    gout, gsum, dz, dh = f(B, U, D).normal_(), f(B).normal_(), f(M), f(B, Tp, D)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        K.cif_fwd(z, plen, ylen, h, B, Tp, U, st)
        K.cif_bwd(plen, ylen, h, B, Tp, U, st, gout, gsum, dz, dh)
    n = 50
    ev[0].record()
    for _ in range(n):
        K.cif_fwd(z, plen, ylen, h, B, Tp, U, st)
    ev[1].record()
    for _ in range(n):
        K.cif_bwd(plen, ylen, h, B, Tp, U, st, gout, gsum, dz, dh)
    ev[2].record()
    torch.cuda.synchronize()
    out["cif_fwd_us"] = round(ev[0].elapsed_time(ev[1]) / n * 1e3, 2)
    out["cif_bwd_us"] = round(ev[1].elapsed_time(ev[2]) / n * 1e3, 2)
    # ---- the reference algorithm on the host (oracle restatement, fp32 torch CPU loop)
    from oracle import paraformer_ref as PR

    a = torch.sigmoid(z.view(B, Tp).cpu())
    hc = h.cpu()
    t0 = time.perf_counter()
    PR.cif(a, hc, ylen.cpu().long())
    out["cif_fwd_cpu_reference_loop_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    out["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
