"""Training CLI (liteasr/train.py:21-105): ``python -m liteasr_amd.train task=... model=... ...``.

The reference's ``@hydra.main`` entry, without Hydra: ``compose`` builds the job config from
the schema, the preset (or ``--config-dir``) yaml tree and the command-line overrides;
then, as Hydra 1.1 does by default, the run directory ``hydra.run.dir`` is created, the
composed config and overrides are written to ``<run dir>/.hydra/``, the process moves into
the run directory (relative paths such as ``task.save_dir`` land there) and logging is
configured from ``hydra.job_logging`` (console + ``train.log``).  ``main`` then injects
``job_logging_cfg`` / ``run_cfg`` (train.py:25-30) and hands the plain job config to
``call_func`` (one GPU in-process, otherwise one spawned rank per GPU over RCCL).

``train`` follows train.py:46-101 step by step: seed, task, datasets (the memory_save
ordering included), model on the GPU, optimizer, criterion, ``Trainer.run``.
"""

import argparse
import logging
import logging.config
import os
import sys

import torch

from . import tasks
from .config.compose import ConfigError, Node, compose, missing_keys, save_run_config
from .distributed import utils as dist_util
from .trainer import Trainer

logger = logging.getLogger("liteasr_amd.train")


def build_trainer(cfg) -> Trainer:
    """train.py:46-100 up to the Trainer (tests drive ``run`` themselves)."""
    torch.manual_seed(int(cfg.common.seed))
    logger.info("set random seed as {}".format(cfg.common.seed))
    device = torch.device("cuda")

    task = tasks.setup_task(cfg.task)
    logger.info("setting {} task...".format(task.__class__.__name__))

    logger.info("1. load data...")
    data_cfg = cfg.dataset, cfg.postprocess
    if not cfg.common.memory_save:
        task.load_dataset("train", task.cfg.train, *data_cfg, False)
        task.load_dataset("valid", task.cfg.valid, *data_cfg, False)
    else:  # machine masters load one after another, then the rest of each machine at once
        assert dist_util.get_world_size() > 1, "memory_save needs a multi-rank job"
        for r in range(dist_util.get_world_size()):
            if dist_util.get_rank() == r and dist_util.is_subworld_master(cfg.distributed):
                task.load_dataset("train", task.cfg.train, *data_cfg, True)
            dist_util.barrier()
        if not dist_util.is_subworld_master(cfg.distributed):
            task.load_dataset("train", task.cfg.train, *data_cfg, True)
        task.load_dataset("valid", task.cfg.valid, *data_cfg, False)

    model = task.build_model(cfg.model).to(device=device)
    logger.info("2. build model    : {}".format(model.__class__.__name__))
    logger.debug("model structure:\n{}".format(model))
    optim = task.build_optimizer(model.parameters(), cfg.optimizer)
    logger.info("3. build optimizer: {}".format(optim.__class__.__name__))
    criter = task.build_criterion(cfg.criterion)
    logger.info("4. build criterion: {}".format(criter.__class__.__name__))
    if isinstance(cfg, Node):
        logger.debug("model training config:\n  " + cfg.to_yaml().replace("\n", "\n  "))
    return Trainer(cfg, task, model, criter, optim)


def train(cfg):
    build_trainer(cfg).run()


def parse_args(argv=None):
    p = argparse.ArgumentParser(prog="liteasr_amd.train", description=__doc__.splitlines()[0])
    p.add_argument("--config-dir", "-cd", default=None, help="directory with <config-name>.yaml and group dirs")
    p.add_argument("--config-name", "-cn", default="config")
    p.add_argument("--cfg", choices=["job", "hydra", "all"], default=None,
                   help="print the composed config and exit (Hydra's --cfg)")
    p.add_argument("overrides", nargs="*", help="group=option, a.b=value, +a.b=value, ~a.b")
    return p.parse_args(argv)


def prepare(argv=None, job_name="train"):
    """Compose + the Hydra run-dir side effects; returns (job config, run dir)."""
    args = parse_args(argv)
    cfg = compose(args.config_dir, args.config_name, args.overrides, job_name=job_name)
    if args.cfg:
        shown = cfg if args.cfg == "all" else (Node.wrap({"hydra": cfg.hydra}) if args.cfg == "hydra" else
                                               Node.wrap({k: v for k, v in cfg.items() if k != "hydra"}))
        sys.stdout.write(shown.to_yaml())
        return None, None
    unset = [k for k in missing_keys(cfg) if k.split(".")[0] in ("task", "dataset", "optimization", "common")]
    if unset:
        raise ConfigError("missing mandatory value(s): " + ", ".join(unset))
    run_dir = os.path.abspath(os.path.join(cfg.hydra.runtime.cwd, str(cfg.hydra.run.dir)))
    os.makedirs(run_dir, exist_ok=True)
    save_run_config(cfg, run_dir, args.overrides)
    if cfg.hydra.get("job", {}).get("chdir", True):
        os.chdir(run_dir)
    logging.config.dictConfig(cfg.hydra.job_logging.to_container())
    job = Node.wrap({k: v for k, v in cfg.items() if k != "hydra"})
    return job, run_dir


def main(argv=None):
    cfg, _ = prepare(argv)
    if cfg is not None:
        dist_util.call_func(train, cfg)


def cli_main():
    main()


if __name__ == "__main__":
    cli_main()
