"""Host-side logic that needs no GPU: the attention mask re-layout (kernels._fwd_mask) and the
FlatReducer's once-per-run check of the native reducer (ddp.FlatReducer._verify_native),
driven over gloo world 2 with a stand-in for the C reducer."""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("sl", [(1, 8, 2, 21), (0, 7, 0, 19), (2, 9, 3, 22)])
def test_fwd_mask_views_the_callers_storage(sl):
    """a sliced (non-contiguous, unaligned) query mask is re-laid out from the
    caller's own storage at (msb, msq) -- not from a contiguous copy the strides do not
    describe.  The returned view equals the mask and has 16-B aligned rows."""
    from liteasr_amd import kernels as K

    g = torch.Generator().manual_seed(sl[0] * 7 + sl[2])
    full = torch.randint(0, 2, (3, 10, 24), dtype=torch.uint8, generator=g)
    m = full[:, sl[0]:sl[1], sl[2]:sl[3]]
    B, Tq, Tk = 3, sl[1] - sl[0], sl[3] - sl[2]
    v, msb, msq = K._fwd_mask(m, m.stride(0), m.stride(1), B, Tq, Tk)
    assert torch.equal(v, m)
    assert msq % 16 == 0 and msb % 16 == 0 and v.data_ptr() % 16 == 0
    assert v.stride() == (msb, msq, 1)
    # the kernels' addressing: element (b, i, j) at data_ptr + b*msb + i*msq + j
    flat = torch.as_strided(v, (v.untyped_storage().nbytes() - v.storage_offset(),), (1,), v.storage_offset())
    for b, i, j in ((0, 0, 0), (B - 1, Tq - 1, Tk - 1), (1, Tq // 2, Tk // 3)):
        assert flat[b * msb + i * msq + j] == m[b, i, j]


class _StubNative:
    """The C reducer's contract (ddp.FlatReducer drives it) over gloo: marked buckets are
    averaged in place at finalize; ``corrupt`` perturbs one element of bucket 0 afterwards."""

    corrupt = 0.0

    def __init__(self, grad, spans, uid, world, rank):
        self.grad, self.spans, self.world = grad, spans, world
        self.device = None
        self.marked = []

    def grad_ptr(self):
        return self.grad.data_ptr()

    def launched(self):
        return len(self.marked)

    def mark(self, bi):
        self.marked.append(bi)

    def reset(self):
        self.marked = []

    def finalize(self):
        for bi in range(len(self.spans)):
            lo, hi = self.spans[bi]
            g = self.grad[lo:hi]
            dist.all_reduce(g, op=dist.ReduceOp.SUM)
            g.div_(self.world)
        if _StubNative.corrupt:
            lo, _ = self.spans[0]
            self.grad[lo] += _StubNative.corrupt
        self.marked = []

    def close(self):
        pass


def _verify_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import liteasr_amd.distributed.native_reducer as NR
        from liteasr_amd.distributed.ddp import FlatReducer
        from test_ddp_cpu import _FakeBackward, _tiny

        NR.NativeReducer = _StubNative
        NR.unique_id = lambda pg=None: b""
        torch.manual_seed(5)
        model = _tiny()
        model.store.ensure_grad().zero_()
        red = FlatReducer(model, bucket_bytes=2048, comm="native")
        assert red._verify
        out = {}
        x = torch.ones(3, requires_grad=True)
        # step 1: rank-dependent gradients ((rank + 1) x unit index), checked against gloo's
        # average of the same pre-reduction buffer
        _FakeBackward.apply(x, model, rank).sum().backward()
        out["verified_once"] = not red._verify
        out["grad"] = model.store.grad.clone().numpy()
        # step 2: no second check (once per run)
        model.store.grad.zero_()
        _StubNative.corrupt = 1.0
        _FakeBackward.apply(x, model, rank).sum().backward()
        out["second_step_unchecked"] = True
        # a fresh reducer whose average is wrong by one element is caught
        model.store.grad.zero_()
        red2 = FlatReducer(model, bucket_bytes=2048, comm="native")
        try:
            _FakeBackward.apply(x, model, rank).sum().backward()
            out["caught"] = None
        except RuntimeError as e:
            out["caught"] = str(e)
        red2._reset()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_verify_native_runs_and_catches_a_wrong_average():
    """_verify_native runs at the first multi-rank step (stand-in C reducer,
    gloo world 2), passes on a correct average, and raises on one wrong element."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert out[r]["verified_once"] and out[r]["second_step_unchecked"]
        assert out[r]["caught"] is not None and "bucket 0" in out[r]["caught"], out[r]["caught"]
    assert (out[0]["grad"] == out[1]["grad"]).all()


def test_held_reductions_queue_order(monkeypatch):
    """kernels.deferred_reductions(hold=True): a held block's reductions and on_done wait for
    the next non-holding block, which launches them first (block order) and then runs every
    callback in block order; an exception inside a held block flushes instead of holding."""
    from liteasr_amd import kernels as K

    launched, events = [], []
    monkeypatch.setattr(K, "_flush_node_end", lambda segs: launched.append([s[0] for s in segs]))
    monkeypatch.setattr(K, "_DEFER", K._Deferred())
    for name, hold in (("L3", True), ("L2", True), ("L1", False)):
        with K.deferred_reductions(hold=hold, on_done=lambda n=name: events.append((n, len(launched)))):
            K._defer(name + "a", 1, 4, None)
            K._defer(name + "b", 1, 4, None)
        if hold:
            assert launched == [] and events == []
            assert K.held_reductions() > 0
    assert launched == [["L3a", "L3b", "L2a", "L2b", "L1a", "L1b"]]
    assert events == [("L3", 1), ("L2", 1), ("L1", 1)]
    assert K.held_reductions() == 0

    with pytest.raises(ValueError):
        with K.deferred_reductions(hold=True, on_done=lambda: events.append(("E", len(launched)))):
            K._defer("E", 1, 4, None)
            raise ValueError
    assert launched[-1] == ["E"] and events[-1] == ("E", 2) and K.held_reductions() == 0
