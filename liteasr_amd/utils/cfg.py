"""Small helpers standing in for OmegaConf.merge / struct configs (no omegaconf here)."""

import dataclasses
import re
from enum import Enum

_INTERP = re.compile(r"^\$\{([\w.]+)\}$")


def _items(obj):
    if obj is None:
        return []
    if isinstance(obj, dict):
        return list(obj.items())
    if dataclasses.is_dataclass(obj):
        return [(f.name, getattr(obj, f.name)) for f in dataclasses.fields(obj)]
    return list(vars(obj).items())


def merge_into(dst, src, assign_back=False):
    """dst.<k> = src[k] for every key of src (dataclass/dict/namespace); with
    assign_back, copy every field of src(=merged) back into dst instead."""
    if assign_back:
        for k, v in _items(src):
            if isinstance(dst, dict):
                dst[k] = v
            else:
                try:
                    setattr(dst, k, v)
                except AttributeError:
                    pass
        return dst
    for k, v in _items(src):
        if k.startswith("_"):
            continue
        if isinstance(dst, dict):
            dst[k] = v
        else:
            setattr(dst, k, v)
    resolve_self(dst)
    return dst


def get(cfg, key, default=None):
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def resolve_self(cfg, scopes=("model", "criterion", "optimizer", "task")):
    """Resolve "${<scope>.field}" strings that refer to fields of cfg itself."""
    for _ in range(8):
        changed = False
        for k, v in _items(cfg):
            if isinstance(v, str):
                m = _INTERP.match(v)
                if m:
                    parts = m.group(1).split(".")
                    if len(parts) == 2 and parts[0] in scopes:
                        nv = get(cfg, parts[1])
                        if nv is not None and nv != v:
                            if isinstance(cfg, dict):
                                cfg[k] = nv
                            else:
                                setattr(cfg, k, nv)
                            changed = True
        if not changed:
            break
    return cfg


def enum_value(v):
    return v.value if isinstance(v, Enum) else v
