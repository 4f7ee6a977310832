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

    @property
    def device_capable(self):
        """True when the whole workflow runs as plan-on-host + one batched device call."""
        return len(self.workflow) == 1 and getattr(self.workflow[0], "device_capable", False)

    def plan_batch(self, lengths, feat_dim):
        return self.workflow[0].plan_batch(lengths, feat_dim)

    def apply_batch(self, xs, xlens, plan):
        return self.workflow[0].apply_batch(xs, xlens, plan)
