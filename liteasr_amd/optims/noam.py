"""Noam schedule (liteasr/optims/noam.py): lr = factor * d^-0.5 * min(s^-0.5, s * w^-1.5),
evaluated on the device from the count of *taken* steps."""

from dataclasses import dataclass, field
from typing import Optional

from . import register_optimzer
from .adam import Adam, AdamConfig


@dataclass
class NoamConfig(AdamConfig):
    name: Optional[str] = field(default="noam")
    beta2: float = field(default=0.98)
    eps: float = field(default=1e-9)
    model_dim: int = field(default=256)
    factor: float = field(default=1.0)
    warmup: int = field(default=25000)


@register_optimzer("noam", dataclass=NoamConfig)
class Noam(Adam):
    def __init__(self, params, cfg: NoamConfig, task=None):
        super().__init__(params, cfg, task)
        self.model_dim = cfg.model_dim
        self.factor = cfg.factor
        self.warmup = cfg.warmup
        for g in self.param_groups:
            g.update(model_dim=self.model_dim, factor=self.factor, warmup=self.warmup)

    def _lr_args(self):
        return 1, 0.0, float(self.factor), float(self.model_dim), float(self.warmup)

    def rate(self, step=None):
        s = self.fused.read()["step"] if step is None else step
        s = max(s, 1)
        return self.factor * self.model_dim ** (-0.5) * min(s ** (-0.5), s * self.warmup ** (-1.5))

    @classmethod
    def build_optimizer(cls, params, cfg, task=None):
        return cls(params, cfg, task)
