"""Structured config schema (liteasr/config/__init__.py:12-102), plain dataclasses.

Hydra / OmegaConf are not available in this environment; ``liteasr_amd.config.compose``
implements the subset of Hydra composition LiteASR's CLI uses (defaults lists,
``group=option`` overrides, dotted overrides, ``${...}`` interpolation, ``???``).
"""

from dataclasses import dataclass, field
from typing import Any, List, Optional

MISSING = "???"


def II(s: str) -> str:
    return "${" + s + "}"


@dataclass
class LiteasrDataclass(object):
    name: Optional[str] = None


@dataclass
class _TriggerConfig(LiteasrDataclass):
    interval: int = field(default=1)
    unit: str = field(default="epoch")


@dataclass
class CommonConfig(LiteasrDataclass):
    seed: int = field(default=1)
    trigger: List[_TriggerConfig] = field(default_factory=lambda: [])
    memory_save: bool = field(default=False)


@dataclass
class DatasetConfig(LiteasrDataclass):
    batch_count: str = field(default="seq")
    batch_size: Optional[int] = field(default=None)
    min_batch_size: Optional[int] = field(default=None)
    max_len_in: Optional[int] = field(default=None)
    max_len_out: Optional[int] = field(default=None)
    max_frame_in: Optional[int] = field(default=None)
    max_frame_out: Optional[int] = field(default=None)
    max_frame_inout: Optional[int] = field(default=None)


@dataclass
class _SpecAugmentConfig(object):
    time_warp: int = field(default=80)
    freq_mask: int = field(default=27)
    freq_mask_times: int = field(default=1)
    time_mask: int = field(default=100)
    time_mask_times: int = field(default=1)
    inplace: bool = field(default=True)
    replace_with_zero: bool = field(default=False)


@dataclass
class PostProcessConfig(LiteasrDataclass):
    spec_aug: _SpecAugmentConfig = field(default_factory=_SpecAugmentConfig)
    workflow: List[str] = field(default_factory=lambda: ["spec_aug"])


@dataclass
class DistributedConfig(LiteasrDataclass):
    world_size: int = field(default=1)
    world_piece_size: List[int] = field(default_factory=lambda: [II("distributed.world_size")])
    machine_rank: int = field(default=0)
    rank: int = field(default=0)
    backend: str = field(default="NCCL")
    init_method: Optional[str] = field(default=None)
    device_id: int = field(default=0)
    num_workers: int = field(default=4)


@dataclass
class OptimizationConfig(LiteasrDataclass):
    max_epoch: int = field(default=-1)
    max_iter: int = field(default=-1)
    accum_grad: int = field(default=1)
    clip_grad_norm: float = field(default=0.0)


@dataclass
class InferenceConfig(LiteasrDataclass):
    ckpt_path: str = II("task.save_dir")
    ckpt_name: Optional[int] = field(default=MISSING)
    model_avg: bool = field(default=False)
    avg_num: int = field(default=1)
    avg_policy: Optional[str] = field(default=II("run_cfg.dir") + "/train.log")
    thread_num: int = field(default=32)


@dataclass
class LiteasrConfig(LiteasrDataclass):
    common: CommonConfig = field(default_factory=CommonConfig)
    dataset: DatasetConfig = field(default_factory=DatasetConfig)
    postprocess: PostProcessConfig = field(default_factory=PostProcessConfig)
    distributed: DistributedConfig = field(default_factory=DistributedConfig)
    optimization: OptimizationConfig = field(default_factory=OptimizationConfig)
    inference: InferenceConfig = field(default_factory=InferenceConfig)
    task: Any = None
    model: Any = None
    criterion: Any = None
    optimizer: Any = None
