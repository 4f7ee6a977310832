"""Paraformer loss (liteasr/criterions/paraformer_loss.py:21-56): gamma * cross-entropy
(ignore -1, mean over targets) + L1(sum_alpha, ylens) (mean), on the fused kernels."""

from dataclasses import dataclass, field
from typing import Optional

from ..config import MISSING, LiteasrDataclass
from ..nets.functional import ParaformerLossFn
from . import LiteasrLoss, register_criterion


@dataclass
class ParaformerLossConfig(LiteasrDataclass):
    name: Optional[str] = field(default="paraformer_loss")
    vocab_size: int = field(default=MISSING)
    gamma: float = field(default=1.0)


@register_criterion("paraformer_loss", dataclass=ParaformerLossConfig)
class ParaformerLoss(LiteasrLoss):
    def __init__(self, cfg: ParaformerLossConfig, task=None):
        super().__init__(cfg)

    @classmethod
    def build_criterion(cls, cfg, task):
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)

    def __call__(self, model, xs, xlens, ys, ylens):
        hs_attn, sum_alpha = model(xs, xlens, ys, ylens)
        tgt = model.get_target(ys, ylens)
        B, L, V = hs_attn.shape
        return ParaformerLossFn.apply(hs_attn.reshape(B * L, V), sum_alpha, tgt.to(hs_attn.device),
                                      ylens.to(hs_attn.device), model.last_count, float(self.cfg.gamma),
                                      model.last_glance.cif)
