"""Criterion registry and interface (liteasr/criterions/__init__.py:11-56)."""

import importlib
import os

from ..config import LiteasrDataclass
from ..utils.cfg import merge_into

CRITERION_REGISTRY = {}
CRITERION_DATACLASS_REGISTRY = {}
CRITERION_CLASS_NAMES = set()


class LiteasrLoss(object):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg

    def build_criterion(self, cfg, task):
        raise NotImplementedError

    def __call__(self, *input, **kwargs):
        return self._loss(*input, **kwargs)


def build_criterion(cfg, task) -> LiteasrLoss:
    name = cfg.get("name") if isinstance(cfg, dict) else getattr(cfg, "name", None)
    criterion = CRITERION_REGISTRY[name]
    merged = merge_into(CRITERION_DATACLASS_REGISTRY[name](), cfg)
    return criterion.build_criterion(merged, task)


def register_criterion(name, dataclass=None):
    def register_criterion_cls(cls):
        CRITERION_REGISTRY[name] = cls
        CRITERION_CLASS_NAMES.add(cls.__name__)
        if dataclass is not None:
            assert issubclass(dataclass, LiteasrDataclass)
            CRITERION_DATACLASS_REGISTRY[name] = dataclass
        return cls

    return register_criterion_cls


_dir = os.path.dirname(__file__)
for _f in sorted(os.listdir(_dir)):
    if not _f.startswith(("_", ".")) and _f.endswith(".py"):
        importlib.import_module(__name__ + "." + _f[:-3])
