"""Task registry and interface (liteasr/tasks/__init__.py:21-105)."""

import importlib
import os

from .. import criterions, models, optims
from ..config import LiteasrDataclass

TASK_DATACLASS_REGISTRY = {}
TASK_REGISTRY = {}
TASK_CLASS_NAMES = set()


class LiteasrTask(object):
    def __init__(self, cfg):
        self.cfg = cfg
        self.datasets = dict()

    def load_dataset(self, split, data_dir, dataset_cfg, postprocess_cfg, memory_save):
        raise NotImplementedError

    def dataset(self, split: str):
        return self.datasets[split]

    def inference(self, x, model):
        raise NotImplementedError

    def save_model(self, model_name: str, model):
        raise NotImplementedError

    def build_model(self, cfg):
        return models.build_model(cfg, self)

    def build_optimizer(self, params, cfg):
        return optims.build_optimizer(params, cfg, self)

    def build_criterion(self, cfg):
        return criterions.build_criterion(cfg, self)

    def __repr__(self):
        s = self.__class__.__name__ + " ("
        for k in sorted(self.__dict__):
            s += f"\n  {k}: {self.__dict__[k]}"
        return s + "\n)"


def setup_task(cfg) -> LiteasrTask:
    name = cfg.get("name") if isinstance(cfg, dict) else getattr(cfg, "name", None)
    return TASK_REGISTRY[name](cfg)


def register_task(name, dataclass=None):
    def register_task_cls(cls):
        TASK_REGISTRY[name] = cls
        TASK_CLASS_NAMES.add(cls.__name__)
        if dataclass is not None:
            assert issubclass(dataclass, LiteasrDataclass)
            TASK_DATACLASS_REGISTRY[name] = dataclass
        return cls

    return register_task_cls


_dir = os.path.dirname(__file__)
for _f in sorted(os.listdir(_dir)):
    if not _f.startswith(("_", ".")) and _f.endswith(".py"):
        importlib.import_module(__name__ + "." + _f[:-3])
