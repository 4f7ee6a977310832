"""Child process of tests/test_switches_gpu.py: one bf16 training step (forward + hybrid loss +
backward) of BASELINE config 2's full model (12 / 6 layers, d 256, V 4233) at B 2 x T 1000,
dropout 0.1, from seeded weights and batch; saves the loss, the flat gradient and the BN
running statistics.  The environment of the process selects the A/B switch under test (they
are read once, at import / library load)."""

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_path):
    from bench import CONFIGS, V, build
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.utils.synthetic import synthetic_batch

    torch.manual_seed(42)
    dev = torch.device("cuda", 0)
    cfgd = dict(CONFIGS["small"], B=2)
    model = build(cfgd, "bf16", 0.1, dev)
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=V, smoothing=0.1, ctc_weight=0.3))
    xs, xlens, ys, ylens = (t.to(dev) for t in synthetic_batch(2, 1000, 40, V, seed=7))
    model.store.ensure_grad().zero_()
    loss = crit(model, xs, xlens, ys, ylens)
    loss.backward()
    torch.cuda.synchronize()
    torch.save({"loss": loss.detach().cpu(), "grad": model.store.grad.detach().cpu(),
                "bn": [b.detach().cpu() for b in model.bn_flat_buffers()]}, out_path)
    print("saved", out_path, float(loss), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
