"""Process-group helpers and the launcher (liteasr/distributed/utils.py:17-139).

One process per GPU, RCCL (``backend: NCCL`` in the config is RCCL on ROCm) over xGMI.
``call_func`` runs the job in-process for one GPU and spawns ``world_piece_size[machine_rank]``
ranks otherwise, each pinned to its local GPU; rank r of machine m is
``sum(world_piece_size[:m]) + r``, as in the reference.  Same names and return conventions
(``get_rank`` / ``get_world_size`` answer -1 outside a process group).
"""

import logging
import logging.config
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

logger = logging.getLogger(__name__)


def _c(cfg, key, default=None):
    return cfg.get(key, default) if isinstance(cfg, dict) else getattr(cfg, key, default)


def get_rank():
    return dist.get_rank() if dist.is_initialized() else -1


def get_world_size():
    return dist.get_world_size() if dist.is_initialized() else -1


def is_master():
    return not dist.is_initialized() or dist.get_rank() == 0


def _machine_base(cfg):
    pieces = list(_c(cfg, "world_piece_size") or [_c(cfg, "world_size", 1)])
    return sum(int(p) for p in pieces[: int(_c(cfg, "machine_rank", 0))]), pieces


def is_subworld_master(cfg):
    """True on the first rank of this machine (the process that loads first under memory_save)."""
    if not dist.is_initialized():
        return True
    return dist.get_rank() == _machine_base(cfg)[0]


def barrier():
    if dist.is_initialized():
        dist.barrier()


def check_distributed_config(cfg):
    n = torch.cuda.device_count()
    if cfg.world_size > n:
        logger.warning(f"world_size changed from {cfg.world_size} -> {n}")
        cfg.world_size = n


def infer_init_method(cfg):
    """A free local TCP port when no init_method is configured (127.0.0.1: the host name
    may not resolve inside containers)."""
    if _c(cfg, "init_method") is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            cfg.init_method = "tcp://127.0.0.1:{}".format(s.getsockname()[1])


def distributed_init(cfg):
    d = cfg.distributed
    logger.info("distributed init (rank {}) at {}".format(d.rank, d.init_method))
    backend = str(d.backend).lower()
    dist.init_process_group(backend=backend, init_method=d.init_method, world_size=int(d.world_size),
                            rank=int(d.rank))
    logger.info("initialized host {} as rank {}".format(socket.gethostname(), d.rank))
    if torch.cuda.is_available() and backend == "nccl":  # bring the RCCL communicator up now
        dist.all_reduce(torch.zeros(1, device="cuda"))
    d.rank = dist.get_rank()
    if d.rank != 0:  # only rank 0 talks
        sys.stdout = open(os.devnull, "w")
        logging.getLogger().setLevel(logging.WARNING)


def switch_logger_level():
    if get_rank() > 0:
        logging.getLogger().setLevel(logging.WARNING - logging.getLogger().level)


def distributed_func(local_rank, func, cfg):
    """Body of one spawned rank: logging, device, process group, ``func(cfg)``, teardown."""
    if _c(cfg, "job_logging_cfg"):
        logging.config.dictConfig(_to_plain(cfg.job_logging_cfg))
    d = cfg.distributed
    d.device_id = local_rank
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    d.rank = _machine_base(d)[0] + local_rank
    distributed_init(cfg)
    try:
        func(cfg)
    finally:
        dist.destroy_process_group()


def call_func(func, cfg):
    """Run ``func(cfg)`` on one GPU, or on ``world_piece_size[machine_rank]`` local ranks."""
    if not torch.cuda.is_available():
        logger.warning("no GPU is visible: nothing to run (the training path is HIP-only)")
        return
    d = cfg.distributed
    if torch.cuda.device_count() == 1 or int(d.world_size) == 1:
        logger.info("using only one single GPU, not apply DDP training")
        return func(cfg)
    infer_init_method(d)
    nprocs = int(_machine_base(d)[1][int(_c(d, "machine_rank", 0))])
    mp.spawn(fn=distributed_func, args=(func, cfg), nprocs=nprocs, join=True)


def _to_plain(node):
    if isinstance(node, dict):
        return {k: _to_plain(v) for k, v in node.items()}
    if isinstance(node, list):
        return [_to_plain(v) for v in node]
    return node
