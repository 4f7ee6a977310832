"""hipGraph replay of the fixed-shape training step (the body of liteasr/trainer.py:140-171
with accum_grad = 1): forward + hybrid loss + backward + clip_grad_norm + NaN-skip +
Noam/Adam + zero_grad.

Every kernel of the step is a stream-ordered lasr_* launch with no host synchronisation
(dropout draws from a device step counter, the optimizer keeps its step/lr/norm on the
device), so the whole step captures into one graph and a replay costs one host call
instead of ~1.5k kernel launches.

Data parallel (``DistributedDataParallel`` of liteasr_amd.distributed.ddp): no collective
is ever captured, yet the bucketed gradient all-reduce still overlaps the backward, as the
reference's DDP hooks make it do (liteasr/trainer.py:76-88).  The backward is split into
segments at the points where a gradient bucket becomes complete (``U2.segmented`` cuts
the encoder's autograd graph there; the reducer's readiness bookkeeping, in record mode,
says which buckets complete in which segment).  Each segment is its own graph, all
sharing one memory pool and replayed in capture order:

    BN buffer broadcast (rank 0, eager)
    graph 0: forward + loss + backward down to the first cut  -> all_reduce(bucket 0..)
    graph 1: next backward segment                            -> all_reduce(bucket ..)
    ...                                                          (RCCL runs on its own
    graph S: last backward segment                               stream while the next
    wait for every bucket                                        segment computes)
    update graph: clip + Adam + zero_grad

Inputs are copied into static buffers (``step(batch)``), so any batch of the captured
shapes can be replayed.  Construction runs ``warmup`` eager steps on the example batch
(to size workspaces and allocator pools) and then restores the parameters, optimizer
moments/state, BN buffers and dropout counter, so building a GraphedTrainStep does not
advance training.
"""

from __future__ import annotations

import torch

from . import kernels as K

# Capture mode: only this thread is barred from capture-unsafe HIP calls.  The RCCL
# process group's watchdog thread polls the events of earlier (finished) collectives
# with hipEventQuery, which the default "global" mode turns into a capture error.
_MODE = "thread_local"


def _new_graph():
    """A graph whose template is kept after capture (``node_counts`` reads it); instantiated
    explicitly right after its capture (``_done``)."""
    try:
        return torch.cuda.CUDAGraph(keep_graph=True)
    except TypeError:  # an older torch: no template to count
        return torch.cuda.CUDAGraph()


def _done(g):
    if hasattr(g, "instantiate"):
        try:
            g.instantiate()
        except RuntimeError:  # already instantiated (keep_graph unsupported)
            pass
    return g


_HIP_NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset"}


def node_counts(graphs):
    """Kernel / memcpy / memset / other node counts of captured graphs (hipGraphGetNodes on
    the kept templates): the launches one replay issues.  None when no template was kept."""
    import ctypes

    try:
        lib = ctypes.CDLL("libamdhip64.so")
        handles = [g.raw_cuda_graph() for g in graphs]
    except (OSError, RuntimeError, AttributeError):
        return None
    out = {"kernel": 0, "memcpy": 0, "memset": 0, "other": 0}
    for h in handles:
        n = ctypes.c_size_t(0)
        if lib.hipGraphGetNodes(ctypes.c_void_p(h), None, ctypes.byref(n)) != 0:
            return None
        nodes = (ctypes.c_void_p * n.value)()
        lib.hipGraphGetNodes(ctypes.c_void_p(h), nodes, ctypes.byref(n))
        for nd in nodes:
            t = ctypes.c_int(-1)
            lib.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
            out[_HIP_NODE_TYPES.get(t.value, "other")] += 1
    return out


class GraphedTrainStep:
    def __init__(self, net, criterion, optimizer, example_batch, clip: float = 5.0, warmup: int = 2,
                 overlap: bool = True, restore: bool = True):
        from .distributed.ddp import DistributedDataParallel

        self.net = net
        self.ddp = net if isinstance(net, DistributedDataParallel) else None
        self.model = net.module if self.ddp is not None else net
        self.crit = criterion
        self.opt = optimizer
        self.clip = float(clip)
        self.static = [t.clone() for t in example_batch]
        self.overlap = bool(overlap) and self.ddp is not None
        self.cuts = self._cut_points() if self.overlap else []
        if not self.cuts:  # one bucket, complete only at the end: nothing to overlap
            self.overlap = False
        snap = self._snapshot() if restore else None
        self._capture(warmup)
        if snap is not None:
            self._restore(snap)

    # ------------------------------------------------------------ schedule
    def _cut_points(self):
        """Encoder positions j (cut before layer j; n = before the heads; -1 = between the
        subsampling's output projection and its convolutions) right after whose backward some
        gradient bucket is complete.  Units finish in the order: ctc, decoder,
        encoder.after_norm (all in the heads node, position n), encoder layer n-1 ... 0
        (layer i at position i), encoder.embed.out (position -1), encoder.embed.conv (end of
        the backward)."""
        n = len(self.model.encoder.enc_layers)
        cuts = set()
        for names in self.ddp.reducer.unit_names():
            last = names[-1]
            if last in ("ctc", "decoder", "encoder.after_norm"):
                cuts.add(n)
            elif last.startswith("encoder.enc_layers."):
                cuts.add(int(last.rsplit(".", 1)[1]))
            elif last == "encoder.embed.out":  # inside the subsampling node (EmbedOutFn | EmbedConvFn)
                cuts.add(-1)
        return sorted(cuts)

    # ------------------------------------------------------------ pieces
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

    def _segments(self):
        """Callables of the segmented fwd/bwd, run in order; the first returns the loss."""
        state = {}

        def complete():
            # every gradient of the piece is reduced by its end (the buckets it completes are
            # all-reduced next): no encoder layer's reductions may still be queued
            if K.held_reductions():
                raise RuntimeError("graph_step: parameter-gradient reductions still queued at a segment end")

        def first():
            with self.model.segmented(self.cuts) as pairs:
                loss = self.crit(self.model, *self.static)
            state["chain"] = sorted(pairs, key=lambda p: p[0], reverse=True)
            top = state["chain"][0][2]
            (state["g"],) = torch.autograd.grad(loss, [top])
            complete()
            state["k"] = 0
            return loss

        def middle():
            k = state["k"]
            _, x, _ = state["chain"][k]
            nxt = state["chain"][k + 1][2]
            (state["g"],) = torch.autograd.grad(x, [nxt], grad_outputs=state["g"])
            complete()
            state["k"] = k + 1

        def last():
            _, x, _ = state["chain"][state["k"]]
            torch.autograd.backward(x, state["g"])
            complete()
            state.clear()

        return [first] + [middle] * (len(self.cuts) - 1) + [last]

    # ------------------------------------------------------------ capture
    def _capture(self, warmup):
        red = self.ddp.reducer if self.ddp is not None else None
        old = red.enabled if red is not None else None
        if red is not None and not self.overlap:
            red.enabled = False  # hooks off: the exchange runs eagerly between two graphs
        try:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):  # grows workspaces / allocator pools
                    self._eager_once()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            if self.ddp is None:
                self.g1 = _new_graph()
                with torch.cuda.graph(self.g1, capture_error_mode=_MODE):
                    self.loss = self._full()
                _done(self.g1)
                self.segs, self.after, self.gupd = None, None, None
            elif not self.overlap:
                self.g1 = _new_graph()
                with torch.cuda.graph(self.g1, capture_error_mode=_MODE):
                    self.loss = self._fwd_bwd()
                _done(self.g1)
                self.gupd = _new_graph()
                with torch.cuda.graph(self.gupd, capture_error_mode=_MODE):
                    self._update()
                _done(self.gupd)
                self.segs, self.after = None, None
            else:
                self.segs, self.after = [], []
                red._reset()
                red.record = []
                try:
                    pool = None
                    for i, fn in enumerate(self._segments()):
                        g = _new_graph()
                        with torch.cuda.graph(g, pool=pool, capture_error_mode=_MODE):
                            out = fn()
                        _done(g)
                        if i == 0:
                            self.loss = out
                            pool = g.pool()
                        self.segs.append(g)
                        self.after.append(list(red.record))
                        red.record.clear()
                finally:
                    red.record = None
                    red._reset()
                launched = [b for a in self.after for b in a]
                assert launched == list(range(len(red.buckets))), launched
                self.gupd = _new_graph()
                with torch.cuda.graph(self.gupd, pool=pool, capture_error_mode=_MODE):
                    self._update()
                _done(self.gupd)
            torch.cuda.synchronize()
            # the graphs address this scratch buffer: keep it alive even if a later eager
            # call grows the workspace (kernels._Workspace replaces, never resizes)
            self._ws = dict(K.WS.buf)
        finally:
            if red is not None:
                red.enabled = old

    def _eager_once(self):
        if self.ddp is None:
            self._full()
            return
        self.ddp._sync_buffers()
        if not self.overlap:
            self._fwd_bwd()
            self.ddp.reducer.allreduce_all()
        else:  # the segmented path with its between-segment launches, eagerly
            red = self.ddp.reducer
            red._reset()
            red.record = []
            try:
                for fn in self._segments():
                    fn()
                    for bi in red.record:
                        red.launch(bi)
                    red.record.clear()
            finally:
                red.record = None
            red.wait()
        self._update()

    # ------------------------------------------------------------ state
    def _state_tensors(self):
        st = self.model.store
        ts = [st.flat]
        if st.work is not None and st.work is not st.flat:
            ts.append(st.work)
        fused = getattr(self.opt, "fused", None)
        if fused is not None:
            ts += [fused.m, fused.v, fused.state]
        ts += [b for b in self.model.buffers()]
        return ts

    def _snapshot(self):
        torch.cuda.synchronize()
        self.model.store.working()  # materialise the working copy so it is captured too
        return [(t, t.clone()) for t in self._state_tensors()]

    def _restore(self, snap):
        with torch.no_grad():
            for t, c in snap:
                t.copy_(c)
        self.model.store.mark_work_synced()  # flat and its working copy restored together
        torch.cuda.synchronize()

    # ------------------------------------------------------------ replay
    def __call__(self, batch=None):
        if batch is not None:
            for s, b in zip(self.static, batch):
                s.copy_(b, non_blocking=True)
        if self.ddp is None:
            self.g1.replay()
            return self.loss
        if self.ddp.broadcast_buffers:
            self.ddp._sync_buffers()
        red = self.ddp.reducer
        if self.segs is None:
            self.g1.replay()
            red.allreduce_all()
        else:
            red._reset()
            ev = self._events
            if ev is not None:
                ev[0].record()
            for k, (g, buckets) in enumerate(zip(self.segs, self.after)):
                g.replay()
                if ev is not None:
                    ev[k + 1].record()
                for bi in buckets:
                    red.launch(bi)
            red.wait()
            if ev is not None:
                ev[-1].record()
        self.gupd.replay()
        return self.loss

    # ------------------------------------------------------------ timing
    _events = None

    def graph_nodes(self):
        """Launches per replayed step: node counts of every graph the step replays."""
        gs = [self.g1] if self.segs is None else list(self.segs)
        if self.gupd is not None:
            gs.append(self.gupd)
        return node_counts(gs)

    def enable_timing(self):
        """Record HIP events between the replayed segments (eager, outside the graphs) so
        ``overlap_report`` can tell how much backward compute follows each bucket's
        all-reduce launch and how much communication stays exposed after the backward."""
        if self.segs is not None:
            self._events = [torch.cuda.Event(enable_timing=True) for _ in range(len(self.segs) + 2)]

    def overlap_report(self):
        """Of the last timed replay (call after synchronising): per segment ms, the buckets
        launched after it, the backward ms still to run after each launch, and the exposed
        communication (end of the last segment -> every bucket reduced)."""
        ev = self._events
        if ev is None:
            return None
        seg = [ev[k].elapsed_time(ev[k + 1]) for k in range(len(self.segs))]
        bwd_after = []
        for k, buckets in enumerate(self.after):
            rest = sum(seg[k + 1:])
            bwd_after += [round(rest, 3)] * len(buckets)
        return {"segment_ms": [round(x, 3) for x in seg], "buckets_after_segment": self.after,
                "backward_ms_after_bucket_launch": bwd_after,
                "exposed_comm_ms": round(ev[-2].elapsed_time(ev[-1]), 3)}
