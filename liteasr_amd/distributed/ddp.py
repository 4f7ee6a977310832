"""Data parallelism for FlatParams models: bucketed gradient all-reduce over RCCL,
overlapped with the backward pass.

Replaces torch DistributedDataParallel as used by the reference (liteasr/trainer.py:76-88,
DDP defaults: 25 MiB buckets, broadcast_buffers=True).  Because every parameter lives
in one flat fp32 buffer laid out module by module, a bucket is simply a contiguous slice
of the flat grad buffer: no bucket copies, no per-parameter hooks.  The fused backward
nodes call ``module.on_grads_ready()`` after writing a module's weight gradients; the
reducer launches ``all_reduce`` (RCCL, async, its own stream) on a bucket as soon as all
modules inside it are done, in backward order (ctc/decoder -> encoder layers 11..0 ->
subsampling), so communication overlaps the remaining backward compute.

Semantics kept from torch DDP: initial parameter + buffer broadcast from rank 0;
gradient *average*; BatchNorm running stats re-broadcast from rank 0 at every forward
(the constant positional-encoding tables are skipped -- identical on every rank);
``no_sync()`` skips the all-reduce for gradient accumulation (trainer.py:142-147).

``comm="native"`` routes the buckets through libliteasr_comm.so (``lasr_reducer_*``,
include/liteasr_comm.h: its own RCCL communicator and HIP stream) instead of
``torch.distributed.all_reduce``; bucket order and finalize points are the same.
"""

from __future__ import annotations

from contextlib import contextmanager
from typing import List

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import kernels as K

from ..nets.modules import _Bound

BUCKET_BYTES = 25 * 1024 * 1024


class _Unit:
    def __init__(self, name, lo, hi):
        self.name, self.lo, self.hi = name, lo, hi


class FlatReducer:
    def __init__(self, model, process_group=None, bucket_bytes=BUCKET_BYTES, comm="torch"):
        assert comm in ("torch", "native"), comm
        self.model = model
        self.store = model.store
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.enabled = True
        units = self._units()
        # buckets in backward order: group consecutive units until >= bucket_bytes; a bucket
        # is one contiguous slice of the flat buffer, so a unit that does not touch the
        # bucket's current range (the Paraformer's heads sit after its decoder in memory
        # but complete before the encoder) starts a new bucket
        self.buckets: List[List[_Unit]] = []
        breaks = model.reducer_bucket_breaks() if hasattr(model, "reducer_bucket_breaks") else set()
        cur, size = [], 0
        for u in units:
            if cur and (u.name in breaks or not (u.lo == max(v.hi for v in cur) or u.hi == min(v.lo for v in cur))):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(u)
            size += (u.hi - u.lo) * 4
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.unit_bucket = {}
        for bi, b in enumerate(self.buckets):
            for u in b:
                self.unit_bucket[u.name] = bi
        # record mode (liteasr_amd.graph_step capture): buckets that become complete are
        # appended here instead of being launched; the graphed step launches them eagerly
        # between the replayed backward segments
        self.record = None
        self.native = None
        if comm == "native":
            from .native_reducer import NativeReducer, unique_id

            uid = unique_id(process_group)
            spans = [(min(u.lo for u in b), max(u.hi for u in b)) for b in self.buckets]
            self.native = NativeReducer(self.store.grad, spans, uid, self.world, dist.get_rank(process_group))
            # multi-rank behaviour of the second communicator is checked once, at the first
            # step with world > 1 (``_verify_native``): the pre-reduction gradient is kept
            self._verify = self.world > 1
            self._pre = None
        self._reset()
        for mod in model.modules():
            if isinstance(mod, _Bound):
                mod._ready_hook = self._on_ready
        model.encoder._after_norm_hook = self._on_ready
        model._unit_hook = self._on_ready  # units that are not _Bound modules (model.unit_ready)

    def _units(self):
        """Hook units (module prefix -> flat range) in the order backward completes them;
        the model names them (``reducer_units``: U2's CTC head / decoder / encoder, the
        Paraformer's decoder / embedding / predictor / encoder)."""
        st = self.store
        units, covered = [], set()
        for name in self.model.reducer_units():
            names = [n for n in st.names if n == name or n.startswith(name + ".")]
            assert names, name
            lo = min(st.offsets[n] for n in names)
            hi = max(st.offsets[n] + st.shapes[n].numel() for n in names)
            units.append(_Unit(name, lo, hi))
            covered.update(names)
        missing = [n for n in st.names if n not in covered]
        assert not missing, f"parameters outside any reducer unit: {missing[:5]}"
        # extend ranges so buckets tile the buffer contiguously (alignment gaps included)
        units_sorted = sorted(units, key=lambda u: u.lo)
        for a, b in zip(units_sorted, units_sorted[1:]):
            assert a.hi <= b.lo, "units overlap"
            a.hi = b.lo
        units_sorted[0].lo = 0
        units_sorted[-1].hi = st.numel
        return units

    def native_spans(self):
        """(lo, hi) element range of every bucket, in launch order."""
        return [(min(u.lo for u in b), max(u.hi for u in b)) for b in self.buckets]

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.works = []
        self.next_bucket = 0
        self.active = False
        if self.native is not None:  # a backward abandoned part-way leaves C-side marks too
            self.native.reset()

    def _native_bound(self):
        """The C reducer averages the buffer it was given at creation; a device move of the
        model (ParamStore.apply) or a re-allocated gradient replaces ``store.grad``, so rebind
        it (between steps) instead of silently averaging the old buffer."""
        g = self.store.grad
        if self.native.grad_ptr() != g.data_ptr():
            if self.native.launched():  # buckets of this step already went out from the old buffer
                raise RuntimeError("FlatReducer: the flat gradient buffer was replaced inside a step")
            if not g.is_cuda or g.device.index != self.native.device:
                raise RuntimeError(f"FlatReducer: the model's gradient moved to {g.device} but the native reducer "
                                   f"(its RCCL communicator and stream) lives on cuda:{self.native.device}; "
                                   "rebuild the DistributedDataParallel wrapper after a device move")
            self.native.rebind(g)

    def close(self):
        """Free the native reducer (its RCCL communicator and HIP stream) now, not at GC."""
        if self.native is not None:
            self.native.close()
            self.native = None

    def _on_ready(self, mod):
        if not self.enabled:
            return
        name = mod if isinstance(mod, str) else mod._pfx
        if name not in self.unit_bucket:
            return
        if not self.active and self.record is None:
            self.active = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        bi = self.unit_bucket[name]
        self.ready[bi] += 1
        # launch buckets strictly in order (every rank issues the same collective sequence)
        while self.next_bucket < len(self.buckets) and self.ready[self.next_bucket] == len(self.buckets[self.next_bucket]):
            if self.record is not None:
                self.record.append(self.next_bucket)
            else:
                self._launch(self.next_bucket)
            self.next_bucket += 1

    def unit_names(self):
        """Hook-unit names bucket by bucket, each bucket in backward-completion order."""
        return [[u.name for u in b] for b in self.buckets]

    def launch(self, bi):
        """Start bucket ``bi``'s async all-reduce now (graphed step, between segments)."""
        self._launch(bi)
        self.next_bucket = max(self.next_bucket, bi + 1)

    def wait(self):
        """Wait for every launched bucket (the current stream waits on RCCL's stream) and
        launch any bucket that never fired; called before the optimizer step."""
        self._finalize()

    def _slice(self, b):
        lo = min(u.lo for u in b)
        hi = max(u.hi for u in b)
        return self.store.grad[lo:hi]

    def _launch(self, bi):
        if self.native is not None:  # C-ABI reducer: in-order launch on its own stream
            if bi == 0 or self.native.launched() == 0:
                self._native_bound()
            if self._verify:
                if self._pre is None:
                    self._pre = {}
                lo, hi = self.native_spans()[bi]
                self._pre[bi] = self.store.grad[lo:hi].clone()
            self.native.mark(bi)
            return
        g = self._slice(self.buckets[bi])
        if self.world == 1:  # the average over one rank is the identity: no collective, no RCCL kernel
            return
        if g.is_cuda and dist.get_backend(self.pg) == "nccl":
            w = dist.all_reduce(g, op=dist.ReduceOp.AVG, group=self.pg, async_op=True)
        else:  # gloo (CPU plumbing tests): SUM then scale
            w = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        self.works.append((w, g))

    def allreduce_all(self):
        """Average the whole flat grad buffer now, bucket by bucket (used between the two
        graphs of liteasr_amd.graph_step: the exchange is never captured)."""
        self._reset()
        for bi in range(len(self.buckets)):
            self._launch(bi)
        self.next_bucket = len(self.buckets)
        self._finalize()

    def _finalize(self):
        for bi in range(self.next_bucket, len(self.buckets)):  # units that never fired
            self._launch(bi)
        if self.native is not None:
            self._native_bound()
            self.native.finalize()
            if self._verify and self._pre is not None:
                self._verify_native()
        for w, g in self.works:
            w.wait()
            if not (g.is_cuda and dist.get_backend(self.pg) == "nccl"):
                g.div_(self.world)
        self._reset()


    def _verify_native(self):
        """Once, at the first step with world > 1: every bucket the C reducer averaged must equal
        a torch.distributed average of the same pre-reduction gradient.  The two communicators
        may sum in different orders, so each element's bar is the fp32 summation bound of its
        inputs, 4·world·2^-23 · (Σ_ranks |g|) / world, not a fraction of the averaged result
        (which can be near zero where the ranks' gradients cancel)."""
        self._verify = False
        pre, self._pre = self._pre, None
        for bi, (lo, hi) in enumerate(self.native_spans()):
            ref = pre[bi]
            mag = ref.abs()
            dist.all_reduce(ref, op=dist.ReduceOp.SUM, group=self.pg)
            dist.all_reduce(mag, op=dist.ReduceOp.SUM, group=self.pg)
            ref.div_(self.world)
            tol = mag.mul_(4.0 * 2.0 ** -23).add_(1e-30)  # (4·world·eps) · Σ|g| / world
            got = self.store.grad[lo:hi]
            bad = (got - ref).abs() > tol
            if bool(bad.any()):
                i = int(bad.nonzero()[0, 0])
                raise RuntimeError(f"native reducer: bucket {bi} element {i} is {got[i].item():.9g}, "
                                   f"torch.distributed's average {ref[i].item():.9g} (bound {tol[i].item():.3g})")


class DistributedDataParallel(nn.Module):
    """torch-DDP-shaped wrapper (``.module``, ``no_sync()``) around a FlatParams model."""

    def __init__(self, module, process_group=None, broadcast_buffers=True, bucket_cap_mb=25, comm="torch", **_):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.broadcast_buffers = broadcast_buffers
        st = module.store
        st.ensure_grad()
        dist.broadcast(st.flat, 0, group=process_group)
        if hasattr(module, "bn_flat_buffers"):  # U2: BN statistics live in two flat buffers
            self._bn_buffers = module.bn_flat_buffers()
        else:
            self._bn_buffers = [b for n, b in module.named_buffers() if not n.endswith(".pe") and not n.startswith("_")]
        self._world = dist.get_world_size(process_group)
        self._sync_buffers()
        st._work_version = -1  # weights changed under the working copy
        self.reducer = FlatReducer(module, process_group, int(bucket_cap_mb * 1024 * 1024), comm=comm)

    def _sync_buffers(self):
        if not self._bn_buffers or self._world == 1:  # rank 0 to itself: nothing to do
            return
        coalesced = getattr(dist, "_broadcast_coalesced", None)
        if coalesced is not None and self._bn_buffers[0].is_cuda:
            pg = self.process_group if self.process_group is not None else dist.group.WORLD
            coalesced(pg, self._bn_buffers, 1 << 20, 0)
        else:
            for b in self._bn_buffers:
                dist.broadcast(b, 0, group=self.process_group)

    def close(self):
        """Release the reducer's native resources (comm="native") before interpreter teardown."""
        self.reducer.close()

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)

    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.module.training:
            self._sync_buffers()
        return self.module(*args, **kwargs)

    @contextmanager
    def no_sync(self):
        old = self.reducer.enabled
        self.reducer.enabled = False
        try:
            yield
        finally:
            self.reducer.enabled = old
