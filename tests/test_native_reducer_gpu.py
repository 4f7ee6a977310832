"""Native bucketed reducer (libliteasr_comm.so, include/liteasr_comm.h) on the GPU.

World 1 only: RCCL cannot place two ranks on the one device of the test box, and the
average over one rank is the identity, so every check is bit-exact.  The N>1 bucket logic
(order, averaging, no_sync) is the same FlatReducer covered by the gloo tests
(tests/test_ddp_cpu.py); this file covers the C-ABI's stream ordering, in-order launch and
error behaviour, and that a DDP step through it equals the torch.distributed path.
Reference mechanism: torch DDP at liteasr/trainer.py:76-88."""

import os
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    """A world-1 gloo group for the unique-id broadcast; destroyed only if this fixture made it
    (the suite passes in any order next to other modules' groups)."""
    import torch.distributed as dist

    made = False
    if not dist.is_initialized():
        port = random.randint(20000, 40000)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        made = True
    yield dist
    if made and dist.is_initialized():
        dist.destroy_process_group()


def test_reducer_in_order_launch_and_identity(pg):
    from liteasr_amd.distributed.native_reducer import NativeReducer, unique_id

    torch.cuda.set_device(0)
    g = torch.randn(10000, device="cuda")
    ref = g.clone()
    uid = unique_id()
    # world 1 issues nothing by default; with single-rank collectives on, every bucket is a real
    # 1-rank ncclAllReduce on the reducer's stream (the path world > 1 takes)
    for forced in (False, True):
        g.copy_(ref)
        r = NativeReducer(g, [(0, 3000), (3000, 7000), (7000, 10000)], uid if not forced else unique_id(), 1, 0)
        try:
            r.set_single_rank_collectives(forced)
            _in_order(r, g, ref.clone())
        finally:
            r.close()


def test_reducer_rebind_refuses_other_device_memory(pg):
    """rebind accepts only device memory of the reducer's own device (its
    communicator, stream and events stay there); host memory is refused by the Python check and
    by the C side itself; a flag change inside a step is refused."""
    import ctypes

    from liteasr_amd.distributed.native_reducer import NativeReducer, load, unique_id

    g = torch.zeros(4096, device="cuda")
    r = NativeReducer(g, [(0, 4096)], unique_id(), 1, 0)
    try:
        host = torch.zeros(4096)
        with pytest.raises(RuntimeError, match="needs a new DistributedDataParallel"):
            r.rebind(host)
        rc = load().lasr_reducer_rebind(r._h, ctypes.c_void_p(host.data_ptr()), 4096)
        assert rc != 0 and b"not device memory" in load().lasr_comm_last_error()
        assert r.grad_ptr() == g.data_ptr()
        r.mark(0)
        with pytest.raises(RuntimeError, match="inside a step"):
            r.set_single_rank_collectives(True)
        r.finalize()
    finally:
        r.close()


def _in_order(r, g, ref):
    for step in range(2):
        r.mark(2)
        assert r.launched() == 0  # bucket 0 not ready: nothing may launch out of order
        r.mark(0)
        assert r.launched() == 1
        r.mark(1)
        assert r.launched() == 3
        with pytest.raises(RuntimeError, match="marked twice"):
            r.mark(1)
        r.finalize()
        torch.cuda.synchronize()
        assert torch.equal(g, ref)
        assert r.launched() == 0
    # a bucket never marked is launched by finalize, on the consumer stream's order
    g.mul_(2.0)
    r.mark(0)
    r.finalize()
    torch.cuda.synchronize()
    assert torch.equal(g, ref * 2.0)
    with pytest.raises(RuntimeError, match="out of range"):
        r.mark(3)
    # an abandoned step (buckets marked, backward stopped) is cleared by reset: the next
    # step marks from scratch without "marked twice" / out-of-order errors
    r.mark(0)
    r.mark(1)
    r.reset()
    assert r.launched() == 0
    for b in (0, 1, 2):
        r.mark(b)
    r.finalize()
    torch.cuda.synchronize()
    # rebind to a new buffer of the same size; a different size is refused
    g2 = torch.randn_like(g)
    r.rebind(g2)
    assert r.grad_ptr() == g2.data_ptr()
    with pytest.raises(RuntimeError, match="numel"):
        r.rebind(torch.zeros(5, device="cuda"))


def test_reducer_rejects_bad_buckets(pg):
    from liteasr_amd.distributed.native_reducer import NativeReducer, unique_id

    g = torch.zeros(100, device="cuda")
    uid = unique_id()
    with pytest.raises(RuntimeError, match="overlap"):
        NativeReducer(g, [(0, 60), (50, 100)], uid, 1, 0)
    with pytest.raises(RuntimeError, match="outside"):
        NativeReducer(g, [(0, 101)], uid, 1, 0)


def test_reducer_keeps_caller_device_and_follows_buffer_swap(pg):
    """the reducer must not change the caller's current device, and a flat gradient
    buffer replaced after wrapping (a device move re-allocates it) is rebound, not silently
    left behind; a FlatReducer reset mid-step clears the C-side marks too."""
    from liteasr_amd.distributed.ddp import DistributedDataParallel
    from oracle import u2_oracle as O
    from test_model_gpu import _graph_setup

    torch.cuda.set_device(0)
    m, c, o = _graph_setup(0.0)
    net = DistributedDataParallel(m, bucket_cap_mb=0.05, comm="native")
    try:
        red = net.reducer
        assert torch.cuda.current_device() == 0
        b = [t.cuda() for t in O.synthetic_batch(2, 100, 5, 30, seed=81)]
        # partial step: mark two buckets then abandon it
        red._launch(0)
        red.next_bucket = 1
        red._reset()
        assert red.native.launched() == 0
        # replace the gradient buffer under the reducer (what ParamStore.apply does on a move)
        old = m.store.grad.data_ptr()
        m.store.grad = m.store.grad.clone()
        m.store.generation += 1
        assert m.store.grad.data_ptr() != old
        l = c(net, *b)
        l.backward()
        torch.cuda.synchronize()
        assert red.native.grad_ptr() == m.store.grad.data_ptr()
    finally:
        net.close()


def test_ddp_step_native_equals_torch(pg):
    """Eager and segmented-graph DDP steps with comm='native' (several buckets) give the
    same losses and parameters, bit for bit, as the torch.distributed reducer."""
    from liteasr_amd.distributed.ddp import DistributedDataParallel
    from liteasr_amd.graph_step import GraphedTrainStep
    from oracle import u2_oracle as O
    from test_model_gpu import _graph_setup

    torch.cuda.set_device(0)
    out = {}
    for comm in ("torch", "native"):
        for mode in ("eager", "graph"):
            m, c, o = _graph_setup(0.0)
            net = DistributedDataParallel(m, bucket_cap_mb=0.05, comm=comm)
            assert len(net.reducer.buckets) >= 3
            bs = [[t.cuda() for t in O.synthetic_batch(2, 100, 5, 30, seed=80 + i)] for i in range(3)]
            if mode == "eager":
                losses = []
                for b in bs:
                    l = c(net, *b)
                    l.backward()
                    o.clip_and_step(5.0)
                    o.zero_grad()
                    losses.append(l.item())
            else:
                gs = GraphedTrainStep(net, c, o, bs[0], clip=5.0, warmup=1, overlap=True)
                losses = [gs(b).item() for b in bs]
            torch.cuda.synchronize()
            out[comm, mode] = (losses, m.store.flat.clone())
            net.close()
    for mode in ("eager", "graph"):
        lt, ft = out["torch", mode]
        ln, fn = out["native", mode]
        assert lt == ln, (mode, lt, ln)
        assert torch.equal(ft, fn), mode
