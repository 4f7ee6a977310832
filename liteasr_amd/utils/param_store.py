"""FlatParams: every parameter of a model lives in one flat fp32 buffer.

Why: the optimizer (clip + Adam) is one fused kernel over the flat buffers, the DDP
gradient all-reduce runs over contiguous buckets of the flat grad buffer, and the
GEMM kernels read a flat low-precision *working copy* that the Adam kernel refreshes
in the same pass.  Parameters stay ordinary ``nn.Parameter`` objects (views into the
buffer), so ``state_dict`` keys/shapes are exactly the reference's and any torch code
that touches ``model.parameters()`` keeps working.

Layout rules: each group of names in ``groups`` is laid out contiguously in the given
order (e.g. linear_q/k/v weights -> one [3d, d] matrix for the fused QKV GEMM); every
group / standalone parameter starts at a multiple of ALIGN elements.
"""

from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.nn as nn

ALIGN = 64


class FlatParams:
    def __init__(self, module: nn.Module, groups: Sequence[Sequence[str]], work_dtype):
        named = dict(module.named_parameters())
        self.names: List[str] = list(named)
        self.work_dtype = work_dtype
        # Registration order, with each group placed at its first member: every module's
        # parameters stay one contiguous range (DDP buckets are flat-buffer slices).
        group_of = {}
        for g in groups:
            for n in g:
                assert n in named, f"unknown parameter {n}"
                assert n not in group_of, f"parameter {n} in two groups"
                group_of[n] = list(g)
        placed = set()
        blocks: List[List[str]] = []
        for n in self.names:
            if n in placed:
                continue
            blk = group_of.get(n, [n])
            blocks.append(blk)
            placed.update(blk)
        self.offsets: Dict[str, int] = {}
        self.shapes: Dict[str, torch.Size] = {}
        off = 0
        for blk in blocks:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            for n in blk:
                self.offsets[n] = off
                self.shapes[n] = named[n].shape
                off += named[n].numel()
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        dev = next(iter(named.values())).device
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for n, p in named.items():
                self.view(n).copy_(p.detach().float())
        self.params = named
        self._rebind()
        self.grad = None
        self.work = None
        self._work_version = -1
        self.generation = 0  # bumped whenever flat / grad / work storage is reallocated

    # ------------------------------------------------------------------ views
    def _slice(self, buf, name):
        o = self.offsets[name]
        shp = self.shapes[name]
        return buf[o: o + shp.numel()].view(shp)

    def view(self, name):
        return self._slice(self.flat, name)

    def group_view(self, names: Sequence[str], buf=None, rows_of=None):
        """Contiguous view spanning ``names`` (laid out back to back)."""
        buf = self.flat if buf is None else buf
        o = self.offsets[names[0]]
        n = 0
        for nm in names:
            assert self.offsets[nm] == o + n, f"{names} are not contiguous"
            n += self.shapes[nm].numel()
        v = buf[o: o + n]
        if rows_of is not None:  # stack 2-D weights along rows
            v = v.view(-1, rows_of)
        return v

    def _rebind(self):
        for n, p in self.params.items():
            p.data = self._slice(self.flat, n)
            p._lasr_store = self

    # ----------------------------------------------------------------- grads
    def _grad_buf(self):
        if self.grad is None or self.grad.device != self.flat.device:
            self.grad = torch.zeros_like(self.flat)
            self.generation += 1
        return self.grad

    def ensure_grad(self):
        """Allocate the flat grad buffer and (re)bind every ``p.grad`` as a view of it.
        O(#params): call once per step (model forward / optimizer), not per view."""
        g = self._grad_buf()
        base = g.data_ptr()
        for n, p in self.params.items():
            pg = p.grad
            if pg is None or pg.data_ptr() != base + 4 * self.offsets[n]:
                p.grad = self._slice(g, n)
        return g

    def grad_view(self, name):
        return self._slice(self._grad_buf(), name)

    def grad_group(self, names, rows_of=None):
        return self.group_view(names, self._grad_buf(), rows_of)

    # --------------------------------------------------------- working copy
    def working(self):
        """Low-precision copy of the flat buffer used as GEMM operands."""
        if self.work_dtype == torch.float32:
            return self.flat
        if self.work is None or self.work.device != self.flat.device:
            self.work = torch.empty(self.numel, dtype=self.work_dtype, device=self.flat.device)
            self._work_version = -1
            self.generation += 1
        if self._work_version != self.flat._version:
            from .. import kernels

            kernels.cast(self.flat, self.work)
            self._work_version = self.flat._version
        return self.work

    def mark_work_synced(self):
        """Called after a kernel refreshed ``work`` together with ``flat``."""
        self._work_version = self.flat._version

    def work_view(self, name):
        return self._slice(self.working(), name)

    def work_group(self, names, rows_of=None):
        return self.group_view(names, self.working(), rows_of)

    # ------------------------------------------------------------- movement
    def apply(self, fn):
        self.flat = fn(self.flat)
        if self.grad is not None:
            self.grad = fn(self.grad)
        self.work = None
        self._work_version = -1
        self.generation += 1
        self._rebind()
