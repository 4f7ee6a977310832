"""Hybrid CTC-attention loss (liteasr/criterions/hybrid_ctc_attn.py), fused HIP kernels.

loss = ctc_weight * CTC(sum)/B + (1 - ctc_weight) * label-smoothed KL(sum)/B, exactly
the reference's reduction; "CTC-only" is ctc_weight = 1.0 (the decoder still runs and
receives zero gradient, as in the reference).
"""

from dataclasses import dataclass, field
from typing import Optional

from ..config import MISSING, LiteasrDataclass
from ..nets.functional import HybridLossFn
from . import LiteasrLoss, register_criterion


@dataclass
class HybridCTCLossConfig(LiteasrDataclass):
    name: Optional[str] = field(default="hybrid_ctc")
    vocab_size: int = field(default=MISSING)
    padding_idx: int = field(default=-1)
    smoothing: float = field(default=0.0)
    normalize_length: bool = field(default=False)
    ctc_weight: float = field(default=0.0)


@register_criterion("hybrid_ctc", dataclass=HybridCTCLossConfig)
class HybridCTCLoss(LiteasrLoss):
    def __init__(self, cfg: HybridCTCLossConfig, task=None):
        super().__init__(cfg)

    @classmethod
    def build_criterion(cls, cfg, task):
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)

    def __call__(self, model, xs, xlens, ys, ylens):
        h_attn, h_ctc = model(xs, xlens, ys, ylens)
        prep = model.last_prep
        return HybridLossFn.apply(h_attn, h_ctc, prep, float(self.cfg.ctc_weight),
                                  float(self.cfg.smoothing), int(self.cfg.padding_idx))
