"""Model registry and interface (liteasr/models/__init__.py:13-86)."""

import importlib
import os

import torch
import torch.nn as nn

from ..config import LiteasrDataclass
from ..utils.cfg import merge_into

MODEL_REGISTRY = {}
MODEL_DATACLASS_REGISTRY = {}


class LiteasrModel(nn.Module):
    def __init__(self):
        super().__init__()

    def build_model(cls, cfg, task):
        raise NotImplementedError

    def inference(self, x):
        raise NotImplementedError

    def save(self, model_path):
        torch.save(self.state_dict(), model_path)

    def get_pred_len(self, xlens):
        raise NotImplementedError

    def get_target(self, ys, ylens):
        raise NotImplementedError

    def get_target_len(self, ylens):
        raise NotImplementedError

    def no_sync(self):
        raise NotImplementedError


def build_model(cfg, task) -> LiteasrModel:
    """Merge the registered dataclass defaults with ``cfg``, build, and copy the
    task-filled fields (input_dim, vocab_size) back into ``cfg`` (models/__init__.py:53-69)."""
    model_name = getattr(cfg, "name", None) if not isinstance(cfg, dict) else cfg.get("name")
    model = MODEL_REGISTRY[model_name]
    dc = MODEL_DATACLASS_REGISTRY[model_name]
    merged = merge_into(dc(), cfg)
    built = model.build_model(merged, task)
    merge_into(cfg, merged, assign_back=True)
    return built


def register_model(name, dataclass=None):
    def register_model_cls(cls):
        MODEL_REGISTRY[name] = cls
        if dataclass is not None:
            assert issubclass(dataclass, LiteasrDataclass)
            MODEL_DATACLASS_REGISTRY[name] = dataclass
        return cls

    return register_model_cls


_dir = os.path.dirname(__file__)
for _f in sorted(os.listdir(_dir)):
    if not _f.startswith(("_", ".")) and _f.endswith(".py"):
        importlib.import_module(__name__ + "." + _f[:-3])
