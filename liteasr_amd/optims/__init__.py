"""Optimizer registry and interface (liteasr/optims/__init__.py:11-88).

``register_optimzer`` keeps the reference's spelling (it is part of the plugin API).
"""

import importlib
import os

from ..config import LiteasrDataclass
from ..utils.cfg import merge_into

OPTIMIZER_REGISTRY = {}
OPTIMIZER_DATACLASS_REGISTRY = {}
OPTIMIZER_CLASS_NAMES = set()


class LiteasrOptimizer(object):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg

    def build_optimizer(cls, params, cfg, task):
        raise NotImplementedError

    @property
    def optimizer(self):
        return self._optimizer

    @property
    def params(self):
        for param_group in self.param_groups:
            for p in param_group["params"]:
                yield p

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def step(self):
        self.optimizer.step()

    def zero_grad(self):
        self.optimizer.zero_grad()

    def __repr__(self):
        s = self.__class__.__name__ + " ("
        for i, group in enumerate(self.param_groups):
            s += f"\nParameter Group {i}\n"
            for key in sorted(group.keys()):
                if key != "params":
                    s += f"    {key}: {group[key]}\n"
        return s + ")"


def build_optimizer(params, cfg, task) -> LiteasrOptimizer:
    name = cfg.get("name") if isinstance(cfg, dict) else getattr(cfg, "name", None)
    optim = OPTIMIZER_REGISTRY[name]
    merged = merge_into(OPTIMIZER_DATACLASS_REGISTRY[name](), cfg)
    return optim.build_optimizer(params, merged, task)


def register_optimzer(name, dataclass=None):
    def register_optimizer_cls(cls):
        OPTIMIZER_REGISTRY[name] = cls
        OPTIMIZER_CLASS_NAMES.add(cls.__name__)
        if dataclass is not None:
            assert issubclass(dataclass, LiteasrDataclass)
            OPTIMIZER_DATACLASS_REGISTRY[name] = dataclass
        return cls

    return register_optimizer_cls


register_optimizer = register_optimzer

_dir = os.path.dirname(__file__)
for _f in sorted(os.listdir(_dir)):
    if not _f.startswith(("_", ".")) and _f.endswith(".py"):
        importlib.import_module(__name__ + "." + _f[:-3])
