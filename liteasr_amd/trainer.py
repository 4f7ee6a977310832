"""Training loop (liteasr/trainer.py:28-227), on the fused HIP step.

Per batch (``run``, reference :130-172): epoch events -> stop check -> batch to the device
(pinned + non_blocking) -> forward/loss/backward under ``no_sync`` on accumulation
micro-steps -> every ``accum_grad`` batches: clip_grad_norm_(clip) + NaN-skip + optimizer
step, iteration events, zero_grad.  The clip, the NaN test and the Adam/Noam update run in
one fused device pass (liteasr_amd/optims/fused_adam.py); the loop then reads the
skipped/taken flag back (one small device->host read per optimizer step, the same host
synchronisation the reference makes with ``math.isnan(grad_norm)``).
"""

import logging
from contextlib import nullcontext

import torch
import torch.distributed as dist
from torch.utils.data.dataloader import DataLoader
from torch.utils.data.distributed import DistributedSampler

from .utils.data_loader import EpochDataLoader
from .utils.trigger import EventManager, Trigger

logger = logging.getLogger(__name__)


def to_device(obj, device):
    if torch.is_tensor(obj):
        return obj.to(device, non_blocking=obj.is_pinned())
    if isinstance(obj, (tuple, list)):
        return tuple(to_device(o, device) for o in obj)
    return obj


def is_master():
    return not dist.is_initialized() or dist.get_rank() == 0


class Trainer(object):
    def __init__(self, cfg, task, model, criterion, optimizer, device=None):
        self.cfg = cfg
        self.task = task
        self._model = model
        self._wrapped_model = None
        self.criterion = criterion
        self.optimizer = optimizer
        self.iter = 0
        train_set, valid_set = task.dataset("train"), task.dataset("valid")
        if dist.is_initialized():
            tr_s, va_s = DistributedSampler(train_set), DistributedSampler(valid_set)
        else:
            tr_s = va_s = None
        self._train_post = getattr(train_set, "postprocess", None)
        pin = torch.cuda.is_available()
        self.train_iter = EpochDataLoader(dataset=train_set, batch_size=1, shuffle=tr_s is None, sampler=tr_s,
                                          num_workers=cfg.distributed.num_workers, collate_fn=train_set.collator,
                                          pin_memory=pin)
        self.valid_iter = DataLoader(dataset=valid_set, batch_size=1, shuffle=va_s is None, sampler=va_s,
                                     collate_fn=valid_set.collator, pin_memory=pin)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self._add_events()
        self.loss = 0
        self.skipped = 0

    @property
    def model(self):
        if self._wrapped_model is None:
            if dist.is_initialized():
                from .distributed.ddp import DistributedDataParallel

                self._wrapped_model = DistributedDataParallel(self._model)
            else:
                self._wrapped_model = self._model
        return self._wrapped_model

    @property
    def epoch(self):
        return self.train_iter.epoch

    @property
    def max_epoch(self):
        return self.cfg.optimization.max_epoch if self.cfg.optimization.max_epoch > 0 else "inf"

    @property
    def max_iter(self):
        return self.cfg.optimization.max_iter if self.cfg.optimization.max_iter > 0 else "inf"

    def _add_events(self):
        self.event_manager = EventManager()
        for t in self.cfg.common.trigger:
            name = t["name"] if isinstance(t, dict) else t.name
            interval = t["interval"] if isinstance(t, dict) else t.interval
            unit = t["unit"] if isinstance(t, dict) else t.unit
            if hasattr(self, name):
                self.event_manager.add_event(Trigger(interval, unit)(getattr(self, name)))

    def stop(self):
        o = self.cfg.optimization
        return (o.max_epoch >= 0 and self.epoch >= o.max_epoch) or (o.max_iter >= 0 and self.iter >= o.max_iter)

    def _optimizer_step(self):
        """clip + NaN check + step, fused on the device; True if the step was taken."""
        opt = self.optimizer
        clip = float(self.cfg.optimization.clip_grad_norm)
        if hasattr(opt, "clip_and_step"):
            opt.clip_and_step(clip)
            return not opt.device_state()["skipped"]
        norm = torch.nn.utils.clip_grad_norm_(self.model.parameters(), clip)
        if torch.isnan(norm):
            return False
        opt.step()
        return True

    def run(self):
        accum = self.cfg.optimization.accum_grad
        for i, batch in enumerate(self.train_iter, start=1):
            self.event_manager.trigger_epoch_events(self)
            if self.stop():
                break
            batch = to_device(batch, self.device)
            if len(batch) == 5:  # device-side postprocess (SpecAugment plan from the collator)
                xs, xlens, ys, ylens, plan = batch
                xs = self._train_post.apply_batch(xs, xlens, plan)
                batch = (xs, xlens, ys, ylens)
            if dist.is_initialized() and i % accum != 0:
                ctx = self.model.no_sync
            else:
                ctx = nullcontext
            with ctx():
                loss = self.criterion(self.model, *batch)
                self.loss += loss.detach() / accum
                loss.backward()
            if i % accum == 0:
                if self._optimizer_step():
                    self.iter += 1
                    self.event_manager.trigger_iteration_events(self)
                else:
                    self.skipped += 1
                    if is_master():
                        logger.warning("iteration {} is skipped since gradient is NaN".format(self.iter + 1))
                self.optimizer.zero_grad()
                self.loss = 0

    def report_loss(self):
        loss = self.loss if torch.is_tensor(self.loss) else torch.tensor(float(self.loss), device=self.device)
        if dist.is_initialized():
            dist.reduce(loss, dst=0)
            loss = loss / dist.get_world_size()
        logger.info("{} / {} iters, {} / {} epochs - current loss: {:.2f}".format(
            self.iter, self.max_iter, self.epoch, self.max_epoch, float(loss)))

    def valid(self):
        self.model.eval()
        with torch.no_grad():
            losses = []
            for bat in self.valid_iter:
                bat = to_device(bat, self.device)
                loss = self.criterion(self.model, *bat)
                if dist.is_initialized():
                    dist.reduce(loss, dst=0)
                    loss = loss / dist.get_world_size()
                losses.append(float(loss))
            reduced = sum(losses) / max(len(losses), 1)
            logger.info("{} / {} iters, {} / {} epochs - valid loss: {:.2f}".format(
                self.iter, self.max_iter, self.epoch, self.max_epoch, reduced))
        self.model.train()
        return reduced

    def save_model(self):
        if is_master():
            self.task.save_model("model.ep.{}.pt".format(self.epoch), self._model)
