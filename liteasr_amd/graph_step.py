"""hipGraph replay of the fixed-shape training step (the body of liteasr/trainer.py:140-171
with accum_grad = 1): forward + hybrid loss + backward + clip_grad_norm + NaN-skip +
Noam/Adam + zero_grad.

Every kernel of the step is a stream-ordered lasr_* launch with no host synchronisation
(dropout draws from a device step counter, the optimizer keeps its step/lr/norm on the
device), so the whole step captures into one graph and a replay costs one host call
instead of ~1.5k kernel launches.

Data parallel (``DistributedDataParallel`` of liteasr_amd.distributed.ddp): the step is
captured as two graphs around the gradient exchange, which stays eager -- the BatchNorm
buffer broadcast from rank 0 (DDP's broadcast_buffers), then graph 1 (forward + loss +
backward, reducer hooks off), then the bucketed all-reduce (mean) of the flat grad
buffer over RCCL, then graph 2 (clip + Adam + zero_grad).  No collective is ever
captured.  Inputs are copied into static buffers (``step(batch)``), so any batch of the
captured shapes can be replayed.
"""

from __future__ import annotations

import torch


class GraphedTrainStep:
    def __init__(self, net, criterion, optimizer, example_batch, clip: float = 5.0, warmup: int = 2):
        from .distributed.ddp import DistributedDataParallel

        self.net = net
        self.ddp = net if isinstance(net, DistributedDataParallel) else None
        self.model = net.module if self.ddp is not None else net
        self.crit = criterion
        self.opt = optimizer
        self.clip = float(clip)
        self.static = [t.clone() for t in example_batch]
        self._capture(warmup)

    # ------------------------------------------------------------------ pieces
    def _fwd_bwd(self):
        loss = self.crit(self.model, *self.static)
        loss.backward()
        return loss

    def _update(self):
        self.opt.clip_and_step(self.clip)
        self.opt.zero_grad()

    def _full(self):
        loss = self._fwd_bwd()
        self._update()
        return loss

    def _capture(self, warmup):
        red = self.ddp.reducer if self.ddp is not None else None
        old = red.enabled if red is not None else None
        if red is not None:
            red.enabled = False  # hooks off: the exchange runs eagerly between the graphs
        try:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):  # grows workspaces / allocator pools
                    self._eager_once()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            self.g1 = torch.cuda.CUDAGraph()
            if self.ddp is None:
                with torch.cuda.graph(self.g1):
                    self.loss = self._full()
                self.g2 = None
            else:
                with torch.cuda.graph(self.g1):
                    self.loss = self._fwd_bwd()
                self.g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g2):
                    self._update()
            torch.cuda.synchronize()
        finally:
            if red is not None:
                red.enabled = old

    def _eager_once(self):
        if self.ddp is not None:
            self.ddp._sync_buffers()
            self._fwd_bwd()
            self.ddp.reducer.allreduce_all()
            self._update()
        else:
            self._full()

    # ---------------------------------------------------------------- replay
    def __call__(self, batch=None):
        if batch is not None:
            for s, b in zip(self.static, batch):
                s.copy_(b, non_blocking=True)
        if self.ddp is None:
            self.g1.replay()
            return self.loss
        if self.ddp.broadcast_buffers:
            self.ddp._sync_buffers()
        self.g1.replay()
        self.ddp.reducer.allreduce_all()
        self.g2.replay()
        return self.loss
