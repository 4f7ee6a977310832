"""Hydra-1.1-compatible config composition for the LiteASR CLI surface (no hydra/omegaconf here).

What the reference's ``@hydra.main(config_path="config", config_name="config")`` entry
(liteasr/train.py:21-43) relies on, and what this module implements:

* a primary config ``<config_dir>/<config_name>.yaml`` with a ``defaults`` list:
  ``liteasr_config`` (the structured schema registered by ``config_init``), one
  ``<group>: <option>`` entry per config group (``task``, ``model``, ``criterion``,
  ``optimizer``; ``???`` = must be chosen on the command line) and ``_self_`` (where the
  file's own keys merge; appended when absent, Hydra 1.1's rule);
* group options resolved as ``<config_dir>/<group>/<option>.yaml`` (a user preset, which
  may itself start with ``defaults: [<option>]`` to extend another option of its group)
  or, failing that, the dataclass registered under that name (``@register_model("U2",
  dataclass=U2Config)`` stores ``U2`` in group ``model``, liteasr/models/__init__.py:72-86);
* command-line overrides: ``group=option`` (re-select a group option), ``a.b.c=value``
  (set an existing key), ``+a.b=value`` (add a key), ``~a.b`` (delete);
* ``${a.b.c}`` interpolation against the composed root (a whole-string reference keeps the
  referenced value's type; embedded references are string-formatted), the ``hydra.*``
  run-time keys (``hydra.job.name``, ``hydra.run.dir``, ``hydra.runtime.cwd``) and the
  ``${now:<strftime>}`` resolver; ``???`` marks mandatory values
  (``missing_keys`` lists what is still unset).

The result is a ``Node``: a dict with attribute access (``cfg.model.enc_dim``), the shape of
an OmegaConf DictConfig as the reference's code reads it.
"""

from __future__ import annotations

import copy
import dataclasses
import datetime
import os
import re
from enum import Enum
from typing import Any, Dict, Iterable, List, Optional, Tuple

import yaml

from . import MISSING, LiteasrConfig

GROUPS = ("task", "model", "criterion", "optimizer")
PRESET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "presets")


class ConfigError(ValueError):
    pass


class Node(dict):
    """dict with attribute access, recursively (DictConfig-style reads and writes)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def __deepcopy__(self, memo):
        return Node({k: copy.deepcopy(v, memo) for k, v in self.items()})

    @staticmethod
    def wrap(obj):
        if isinstance(obj, dict):
            return Node({k: Node.wrap(v) for k, v in obj.items()})
        if isinstance(obj, list):
            return [Node.wrap(v) for v in obj]
        return obj

    def to_container(self):
        def un(o):
            if isinstance(o, dict):
                return {k: un(v) for k, v in o.items()}
            if isinstance(o, list):
                return [un(v) for v in o]
            return o

        return un(self)

    def to_yaml(self) -> str:
        return yaml.safe_dump(self.to_container(), sort_keys=False, default_flow_style=False)


# ------------------------------------------------------------------ schemas ---
def dataclass_node(obj) -> Dict[str, Any]:
    """A (registered) dataclass instance as a plain nested dict; enums by value name."""

    def conv(v):
        if dataclasses.is_dataclass(v):
            return {f.name: conv(getattr(v, f.name)) for f in dataclasses.fields(v)}
        if isinstance(v, Enum):
            return v.name
        if isinstance(v, (list, tuple)):
            return [conv(x) for x in v]
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items()}
        return v

    return conv(obj)


def _registries():
    from .. import criterions, models, optims, tasks

    return {"task": tasks.TASK_DATACLASS_REGISTRY, "model": models.MODEL_DATACLASS_REGISTRY,
            "criterion": criterions.CRITERION_DATACLASS_REGISTRY,
            "optimizer": optims.OPTIMIZER_DATACLASS_REGISTRY}


def _registered_node(group: str, option: str) -> Optional[Dict[str, Any]]:
    dc = _registries()[group].get(option)
    if dc is None:
        return None
    node = dataclass_node(dc())
    node["name"] = option  # ConfigStore node._name (models/__init__.py:79-80)
    return node


# -------------------------------------------------------------------- merge ---
def merge(dst: Dict[str, Any], src: Dict[str, Any]) -> Dict[str, Any]:
    """Recursive OmegaConf.merge-like update: dicts merge key by key, anything else
    (lists included) replaces."""
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _load_yaml(path: str) -> Dict[str, Any]:
    with open(path) as fh:
        data = yaml.safe_load(fh) or {}
    if not isinstance(data, dict):
        raise ConfigError(f"{path}: top level must be a mapping")
    return data


def _defaults_entries(defaults) -> List[Tuple[Optional[str], str]]:
    """[(group or None, name)] from a Hydra defaults list."""
    out = []
    for d in defaults or []:
        if isinstance(d, str):
            out.append((None, d))
        elif isinstance(d, dict) and len(d) == 1:
            (g, o), = d.items()
            out.append((str(g), o))
        else:
            raise ConfigError(f"unsupported defaults entry {d!r}")
    return out


def _load_group_option(config_dir: Optional[str], group: str, option: str, seen=()) -> Dict[str, Any]:
    if option == MISSING or option is None:
        raise ConfigError(f"You must specify '{group}', e.g. {group}=<option>")
    if (group, option) in seen:
        raise ConfigError(f"cyclic defaults: {group}/{option}")
    path = os.path.join(config_dir, group, f"{option}.yaml") if config_dir else None
    if path and os.path.exists(path):
        data = _load_yaml(path)
        entries = _defaults_entries(data.pop("defaults", []))
        node: Dict[str, Any] = {}
        self_done = False
        for g, name in entries:
            if g is None and name == "_self_":
                merge(node, data)
                self_done = True
            else:  # inside a group file, a bare name is another option of the same group
                merge(node, _load_group_option(config_dir, g or group, name, seen + ((group, option),)))
        if not self_done:
            merge(node, data)
        return node
    reg = _registered_node(group, option)
    if reg is None:
        where = f"{config_dir}/{group}/{option}.yaml" if config_dir else f"{group}/{option}"
        avail = sorted(_registries()[group])
        raise ConfigError(f"Could not find '{where}' nor a registered {group} '{option}' (registered: {avail})")
    return reg


# ---------------------------------------------------------------- overrides ---
def _parse_value(text: str):
    try:
        return yaml.safe_load(text) if text != "" else ""
    except yaml.YAMLError:
        return text


def _split_overrides(overrides: Iterable[str]):
    groups, sets = {}, []
    for o in overrides:
        o = o.strip()
        if not o:
            continue
        if o.startswith("~"):
            sets.append(("del", o[1:].split("=", 1)[0], None))
            continue
        if "=" not in o:
            raise ConfigError(f"override '{o}' is not key=value")
        key, val = o.split("=", 1)
        add = key.startswith("+")
        key = key.lstrip("+")
        if key in GROUPS and not add:
            groups[key] = val
        else:
            sets.append(("add" if add else "set", key, _parse_value(val)))
    return groups, sets


def _apply_set(root: Dict[str, Any], op: str, key: str, value):
    parts = key.split(".")
    cur = root
    for p in parts[:-1]:
        if not isinstance(cur.get(p), dict):
            if op == "add":
                cur[p] = {}
            else:
                raise ConfigError(f"Could not override '{key}': '{p}' is not a config node")
        cur = cur[p]
    leaf = parts[-1]
    if op == "del":
        cur.pop(leaf, None)
    elif op == "set" and leaf not in cur:
        raise ConfigError(f"Could not override '{key}': key not in the config (use +{key}=...)")
    else:
        cur[leaf] = value


# ------------------------------------------------------------ interpolation ---
_REF = re.compile(r"\$\{([^${}]+)\}")


def _lookup(root, path: str):
    cur = root
    for p in path.split("."):
        if isinstance(cur, str):  # an interpolated node on the way: follow it
            m = _REF.fullmatch(cur)
            if not m:
                raise KeyError(path)
            cur = _resolver(m.group(1), root)
        if isinstance(cur, dict) and p in cur:
            cur = cur[p]
        elif isinstance(cur, list) and p.isdigit() and int(p) < len(cur):
            cur = cur[int(p)]
        else:
            raise KeyError(path)
    return cur


_NOW = []  # the job's start time: every ${now:} of one compose() sees the same instant


def _resolver(expr: str, root):
    if expr.startswith("now:"):
        return (_NOW[-1] if _NOW else datetime.datetime.now()).strftime(expr[4:])
    if expr.startswith("hydra:"):
        return _lookup(root, "hydra." + expr[6:])
    return _lookup(root, expr)


def resolve(root: Dict[str, Any]) -> Dict[str, Any]:
    """Resolve ``${...}`` in place until nothing changes (chains allowed, cycles rejected)."""

    def res(v, depth=0):
        if depth > 32:
            raise ConfigError("interpolation cycle")
        if isinstance(v, dict):
            for k in list(v):
                v[k] = res(v[k], depth)
            return v
        if isinstance(v, list):
            return [res(x, depth) for x in v]
        if not isinstance(v, str) or "${" not in v:
            return v
        m = _REF.fullmatch(v)
        try:
            if m:
                out = copy.deepcopy(_resolver(m.group(1), root))
                return res(out, depth + 1)
            return res(_REF.sub(lambda mm: str(res(_resolver(mm.group(1), root), depth + 1)), v), depth + 1)
        except KeyError as e:
            raise ConfigError(f"interpolation {v!r}: key {e.args[0]!r} not found") from None

    return res(root)


def missing_keys(cfg, prefix="") -> List[str]:
    out = []
    for k, v in cfg.items():
        if isinstance(v, dict):
            out += missing_keys(v, f"{prefix}{k}.")
        elif v == MISSING:
            out.append(prefix + k)
    return out


# ------------------------------------------------------------------ compose ---
def _hydra_node(job_name: str):
    """Hydra 1.1's defaults for the keys the reference reads: job name, run dir, launch cwd
    and job_logging (console + ``<job name>.log`` in the run dir, root at INFO)."""
    return {"job": {"name": job_name}, "run": {"dir": "outputs/${now:%Y-%m-%d}/${now:%H-%M-%S}"},
            "runtime": {"cwd": os.getcwd()},
            "job_logging": {"version": 1,
                            "formatters": {"simple": {"format": "[%(asctime)s][%(name)s][%(levelname)s] - %(message)s"}},
                            "handlers": {"console": {"class": "logging.StreamHandler", "formatter": "simple",
                                                     "stream": "ext://sys.stdout"},
                                         "file": {"class": "logging.FileHandler", "formatter": "simple",
                                                  "filename": "${hydra.job.name}.log"}},
                            "root": {"level": "INFO", "handlers": ["console", "file"]},
                            "disable_existing_loggers": False}}


def compose(config_dir: Optional[str] = None, config_name: str = "config", overrides: Iterable[str] = (),
            job_name: str = "train") -> Node:
    """Compose the config the reference's CLI would see (see the module docstring)."""
    config_dir = config_dir or PRESET_DIR
    primary_path = os.path.join(config_dir, f"{config_name}.yaml")
    primary = _load_yaml(primary_path) if os.path.exists(primary_path) else {
        "defaults": ["liteasr_config"] + [{g: MISSING} for g in GROUPS] + ["_self_"]}
    entries = _defaults_entries(primary.pop("defaults", ["liteasr_config", "_self_"]))
    if (None, "_self_") not in entries:
        entries.append((None, "_self_"))
    group_ovr, sets = _split_overrides(overrides)
    listed = {g for g, _ in entries if g}
    for g in group_ovr:  # a group chosen on the command line but absent from the defaults
        if g not in listed:
            entries.insert(len(entries) - 1, (g, group_ovr[g]))
    root: Dict[str, Any] = {"hydra": _hydra_node(job_name)}
    for g, name in entries:
        if g is None:
            if name == "liteasr_config":
                merge(root, dataclass_node(LiteasrConfig()))
            elif name == "_self_":
                merge(root, primary)
            else:
                raise ConfigError(f"unknown defaults entry '{name}'")
        else:
            root[g] = merge(root.get(g) if isinstance(root.get(g), dict) else {},
                            _load_group_option(config_dir, g, group_ovr.get(g, name)))
    for op, key, val in sets:
        _apply_set(root, op, key, val)
    # the reference's main injects these before resolving (liteasr/train.py:25-30); the
    # schema interpolates run_cfg.dir (InferenceConfig.avg_policy)
    root.setdefault("job_logging_cfg", copy.deepcopy(root["hydra"]["job_logging"]))
    root.setdefault("run_cfg", copy.deepcopy(root["hydra"]["run"]))
    _NOW.append(datetime.datetime.now())
    try:
        resolve(root)
    finally:
        _NOW.pop()
    return Node.wrap(root)


def save_run_config(cfg: Node, run_dir: str, overrides: Iterable[str] = ()):
    """Hydra's ``<run dir>/.hydra/{config,overrides}.yaml`` (the composed job config
    without the ``hydra`` node, and the command-line overrides)."""
    d = os.path.join(run_dir, ".hydra")
    os.makedirs(d, exist_ok=True)
    job = {k: v for k, v in cfg.to_container().items() if k != "hydra"}
    with open(os.path.join(d, "config.yaml"), "w") as fh:
        yaml.safe_dump(job, fh, sort_keys=False)
    with open(os.path.join(d, "overrides.yaml"), "w") as fh:
        yaml.safe_dump(list(overrides), fh)
