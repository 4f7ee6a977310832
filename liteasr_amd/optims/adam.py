"""Adam (liteasr/optims/adam.py) on the fused flat kernel."""

from dataclasses import dataclass, field
from typing import Optional

from .. import kernels as K
from ..config import LiteasrDataclass
from . import LiteasrOptimizer, register_optimzer
from .fused_adam import FlatAdamState, find_store


@dataclass
class AdamConfig(LiteasrDataclass):
    name: Optional[str] = field(default="adam")
    lr: float = field(default=1e-3)
    beta1: float = field(default=0.9)
    beta2: float = field(default=0.999)
    eps: float = field(default=1e-8)
    weight_decay: float = field(default=0.0)
    amsgrad: bool = field(default=False)


class _Groups:
    """param_groups look-alike (one group) so reference-style code keeps working."""

    def __init__(self, params, cfg):
        self.groups = [dict(params=list(params), lr=cfg.lr, betas=(cfg.beta1, cfg.beta2), eps=cfg.eps,
                            weight_decay=cfg.weight_decay, amsgrad=cfg.amsgrad)]


@register_optimzer("adam", dataclass=AdamConfig)
class Adam(LiteasrOptimizer):
    lr_mode = 0

    def __init__(self, params, cfg: AdamConfig, task=None):
        super().__init__(cfg)
        if cfg.amsgrad:
            raise NotImplementedError("amsgrad is not on the U2 hot path")
        params = list(params)
        self.store = find_store(params)
        self._groups = _Groups(params, cfg)
        self.fused = FlatAdamState(self.store)
        self.max_norm = float("inf")  # step() alone does not clip

    @property
    def optimizer(self):
        return self

    @property
    def param_groups(self):
        return self._groups.groups

    def _lr_args(self):
        g = self.param_groups[0]
        return 0, float(g["lr"]), 1.0, 1.0, 1.0

    def clip_and_step(self, max_norm: float):
        """clip_grad_norm_(max_norm) + NaN-skip + Adam step, fused, no host sync."""
        mode, lr, factor, dim, warm = self._lr_args()
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        self.fused.step(float(max_norm), mode, lr, factor, dim, warm, b1, b2, g["eps"], g["weight_decay"])

    def step(self):
        """torch.optim.Adam.step: no clipping (max_norm = +inf; a NaN norm still skips)."""
        self.clip_and_step(self.max_norm)

    def zero_grad(self):
        grad = self.store.ensure_grad()
        K.fill(grad, 0.0)

    def device_state(self):
        """{step, lr, grad_norm, skipped, clip_coef} of the last step (host sync)."""
        return self.fused.read()

    @classmethod
    def build_optimizer(cls, params, cfg, task=None):
        return cls(params, cfg, task)
