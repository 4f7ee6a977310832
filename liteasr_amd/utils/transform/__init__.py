"""Feature post-processing registry (liteasr/utils/transform/__init__.py:10-46)."""

import importlib
import os

TRANS_REGISTRY = {}


def register_transformation(name):
    def register_transformation_cls(cls):
        TRANS_REGISTRY[name] = cls
        return cls

    return register_transformation_cls


_dir = os.path.dirname(__file__)
for _f in sorted(os.listdir(_dir)):
    if not _f.startswith(("_", ".")) and _f.endswith(".py"):
        importlib.import_module(__name__ + "." + _f[:-3])


class PostProcess(object):
    def __init__(self, cfg):
        self.workflow = []
        for name in cfg.workflow:
            if name not in TRANS_REGISTRY:
                raise NotImplementedError(f"transformation '{name}' is not available in liteasr_amd")
            self.workflow.append(TRANS_REGISTRY[name](getattr(cfg, name)))

    def __call__(self, x):
        for t in self.workflow:
            x = t(x)
        return x

    def __len__(self):
        return len(self.workflow)
