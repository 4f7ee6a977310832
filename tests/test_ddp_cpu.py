"""Multi-process (gloo, world_size 2 and 4, CPU) tests of the FlatParams DDP reducer: initial
broadcast, bucket launch order driven by the backward-node hooks, gradient averaging,
no_sync(), and BN-buffer re-broadcast.  The HIP kernels are not involved: a stand-in
autograd node writes rank-dependent gradients into the flat grad buffer and fires the
same ``on_grads_ready`` hooks, in the same order, as the fused backward nodes."""

import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _tiny():
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    c = U2Config(input_dim=40, vocab_size=20, enc_dim=32, enc_ff_dim=64, enc_attn_heads=4, enc_layers=3,
                 dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=2)
    resolve_self(c)
    return U2(c)


class _FakeBackward(torch.autograd.Function):
    """Writes grad = (rank+1) * unit_index into each unit's flat range, firing hooks in
    the fused backward's order (ctc, decoder, encoder.after_norm, layers N-1..0, the
    subsampling's output projection, its convolutions)."""

    @staticmethod
    def forward(ctx, x, model, rank):
        ctx.model, ctx.rank = model, rank
        return x * 1.0

    @staticmethod
    def backward(ctx, g):
        m, r = ctx.model, ctx.rank
        st = m.store
        grad = st.ensure_grad()
        emb = m.encoder.embed
        order = [m.ctc, m.decoder, "encoder.after_norm"] + list(reversed(list(m.encoder.enc_layers))) + \
            [(emb, u) for u in emb.UNITS]
        for i, mod in enumerate(order):
            pfx = mod if isinstance(mod, str) else mod[0]._n(mod[1]) if isinstance(mod, tuple) else mod._pfx
            for n in st.names:
                if n == pfx or n.startswith(pfx + "."):
                    o, k = st.offsets[n], st.shapes[n].numel()
                    grad[o:o + k] += (r + 1) * (i + 1)
            if isinstance(mod, str):
                m.encoder.after_norm_ready()
            elif isinstance(mod, tuple):
                mod[0].unit_ready(mod[1])
            else:
                mod.on_grads_ready()
        return g, None, None


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from liteasr_amd.distributed.ddp import DistributedDataParallel

        torch.manual_seed(100 + rank)  # different init per rank -> broadcast must fix it
        model = _tiny()
        bn = model.encoder.enc_layers[0].conv.norm.running_mean
        bn.fill_(float(rank + 7))
        ddp = DistributedDataParallel(model, bucket_cap_mb=0.05)
        res = {"nbuckets": len(ddp.reducer.buckets)}
        flat0 = model.store.flat.clone()
        res["bn_after_init"] = float(bn[0])
        x = torch.ones(3, requires_grad=True)
        # step 1: synced
        model.store.ensure_grad().zero_()
        _FakeBackward.apply(x, model, rank).sum().backward()
        res["grad_sync"] = model.store.grad.clone()
        # step 2: no_sync accumulates locally
        model.store.grad.zero_()
        with ddp.no_sync():
            _FakeBackward.apply(x, model, rank).sum().backward()
        res["grad_nosync"] = model.store.grad.clone()
        # step 3: record mode (graphed step capture): completed buckets are listed in
        # backward order instead of launched; launched afterwards they average as usual
        red = ddp.reducer
        model.store.grad.zero_()
        red._reset()
        red.record = []
        _FakeBackward.apply(x, model, rank).sum().backward()
        res["record"] = list(red.record)
        res["grad_unreduced"] = model.store.grad.clone()
        for bi in red.record:
            red.launch(bi)
        red.record = None
        red.wait()
        res["grad_record"] = model.store.grad.clone()
        # graphed-step cut points: every bucket but the last ends at an encoder position
        from liteasr_amd.graph_step import GraphedTrainStep

        gs = GraphedTrainStep.__new__(GraphedTrainStep)
        gs.model, gs.ddp = model, ddp
        res["cuts"] = gs._cut_points()
        res["bucket_units"] = red.unit_names()
        res["flat"] = flat0
        # forward-time buffer broadcast (BN running stats from rank 0)
        bn.fill_(float(rank + 20))
        ddp._sync_buffers()
        res["bn_after_sync"] = float(bn[0])
        # by value: a torch tensor through the queue is a shared-memory handle that dies with
        # this process, which may exit before the parent unpickles it
        q.put((rank, {k: (v.numpy().copy() if isinstance(v, torch.Tensor) else v) for k, v in res.items()}))
    finally:
        dist.destroy_process_group()


def _run_world(world):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: {k: (torch.from_numpy(v) if hasattr(v, "dtype") and hasattr(v, "shape") else v) for k, v in d.items()}
           for r, d in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_flat_ddp_gloo_world4():
    """The same reducer at world 4 (the N > 1 path rehearsed on more ranks than the GPU tests
    can use): rank-0 broadcast, the bucket mean over four ranks, rank-local no_sync, record
    mode and the BN re-broadcast hold on every rank."""
    world = 4
    out = _run_world(world)
    a = out[0]
    mean = sum(r + 1 for r in range(world)) / world  # 2.5: exact in fp32
    for r in range(world):
        o = out[r]
        assert o["nbuckets"] == a["nbuckets"] > 2
        assert torch.equal(o["flat"], a["flat"])
        assert o["bn_after_init"] == 7.0 and o["bn_after_sync"] == 20.0
        assert torch.equal(o["grad_sync"], a["grad_sync"])
        assert torch.equal(o["grad_nosync"], (r + 1) * a["grad_nosync"])
        assert torch.equal(o["grad_unreduced"], (r + 1) * a["grad_unreduced"])
        assert torch.equal(o["grad_record"], a["grad_sync"])
        assert o["record"] == list(range(a["nbuckets"]))
        assert o["cuts"] == a["cuts"]
    # averaged: mean_r((r + 1) * i) = 2.5 * i, i.e. 2.5 times the rank-0 local gradient
    assert torch.equal(a["grad_sync"], mean * a["grad_nosync"])


def test_flat_ddp_gloo_world2():
    out = _run_world(2)
    a, b = out[0], out[1]
    assert a["nbuckets"] > 2  # several buckets -> ordered launches were exercised
    assert torch.equal(a["flat"], b["flat"])  # rank-0 parameters broadcast
    assert a["bn_after_init"] == b["bn_after_init"] == 7.0
    # averaged: ((0+1)*i + (1+1)*i) / 2 = 1.5 * i on every rank
    assert torch.equal(a["grad_sync"], b["grad_sync"])
    st = _tiny().store  # same layout on every rank
    g = a["grad_sync"]
    nz = g[g != 0]
    assert len(nz) > 0
    vals = torch.unique(nz)
    assert torch.allclose(vals / 1.5, torch.round(vals / 1.5)), vals
    # no_sync: rank-local values ((r+1) * i)
    assert torch.equal(b["grad_nosync"], 2 * a["grad_nosync"])
    assert a["bn_after_sync"] == b["bn_after_sync"] == 20.0
    # record mode: every bucket recorded once, in order, nothing reduced until launched
    assert a["record"] == list(range(a["nbuckets"]))
    assert torch.equal(b["grad_unreduced"], 2 * a["grad_unreduced"])
    assert torch.equal(a["grad_record"], a["grad_sync"]) and torch.equal(b["grad_record"], a["grad_sync"])
    # cut points: one per bucket whose last unit completes before the subsampling convolutions'
    # backward
    n_layers = 3
    ends = [u[-1] for u in a["bucket_units"]]
    expect = set()
    for e in ends:
        if e in ("ctc", "decoder", "encoder.after_norm"):
            expect.add(n_layers)
        elif e.startswith("encoder.enc_layers."):
            expect.add(int(e.rsplit(".", 1)[1]))
        elif e == "encoder.embed.out":
            expect.add(-1)  # inside the subsampling: its convolutions' backward is the last segment
    assert a["cuts"] == sorted(expect) and len(a["cuts"]) >= 2 and -1 in a["cuts"], (a["cuts"], ends)
    assert ends[-2:] == ["encoder.embed.out", "encoder.embed.conv"], ends
    del st


def _spawn_target(rank, world, port, argv):
    """Stand-in for bench.py's per-rank main: the env bench.spawn_ranks sets, checked
    through a real gloo rendezvous on 127.0.0.1."""
    assert os.environ.get("RANK") is None  # the parent's env is clean; the child sets it
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    ok = dist.get_world_size() == world and t.item() == world * (world + 1) / 2 and argv == ["--x", "1"]
    dist.destroy_process_group()
    sys.exit(0 if ok else 3)


def test_bench_spawns_one_process_per_rank():
    """bench.py --gpus N (no launcher): N spawned ranks rendezvous as one world of N
    (liteasr/distributed/utils.py:119-139 call_func -> mp.spawn)."""
    import bench

    assert bench.spawn_ranks(3, argv=["--x", "1"], target=_spawn_target) == 0


def _tiny_paraformer():
    from liteasr_amd.models.paraformer import Paraformer, ParaformerConfig
    from liteasr_amd.utils.cfg import resolve_self

    c = ParaformerConfig(input_dim=40, vocab_size=20, enc_dim=32, enc_ff_dim=64, enc_attn_heads=4, enc_layers=2,
                         dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=2)
    resolve_self(c)
    return Paraformer(c)


def _fire_units(model, rank):
    """Stand-in backward: every reducer unit gets (rank+1)*(i+1) and fires its hook the way
    the fused nodes do (_Bound.on_grads_ready, encoder.after_norm_ready, model.unit_ready)."""
    from liteasr_amd.nets.modules import _Bound

    st = model.store
    grad = st.ensure_grad()
    mods = {m._pfx: m for m in model.modules() if isinstance(m, _Bound)}
    for i, name in enumerate(model.reducer_units()):
        for n in st.names:
            if n == name or n.startswith(name + "."):
                o, k = st.offsets[n], st.shapes[n].numel()
                grad[o:o + k] += (rank + 1) * (i + 1)
        if name == "encoder.after_norm":
            model.encoder.after_norm_ready()
        elif name in mods:
            mods[name].on_grads_ready()
        else:
            model.unit_ready(name)


def _tiny_transducer():
    from liteasr_amd.models.transducer import Transducer, TransducerConfig
    from liteasr_amd.utils.cfg import resolve_self

    c = TransducerConfig(input_dim=40, vocab_size=20, enc_dim=64, enc_ff_dim=128, enc_attn_heads=4, enc_layers=2,
                         activation="swish", enc_arch="conformer", dec_dim=16, dec_units=48, dec_layers=2,
                         joint_dim=24)
    resolve_self(c)
    return Transducer(c)


def _paraformer_worker(rank, world, port, q, make=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from liteasr_amd.distributed.ddp import DistributedDataParallel

        torch.manual_seed(200 + rank)
        model = (make or _tiny_paraformer)()
        ddp = DistributedDataParallel(model, bucket_cap_mb=0.02)
        red = ddp.reducer
        model.store.ensure_grad().zero_()
        red._reset()
        red.record = []
        _fire_units(model, rank)
        rec = list(red.record)
        for bi in red.record:
            red.launch(bi)
        red.record = None
        red.wait()
        q.put((rank, {"units": model.reducer_units(), "nbuckets": len(red.buckets), "record": rec,
                      "grad": model.store.grad.numpy().copy(), "flat": model.store.flat.numpy().copy()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("which", ["paraformer", "transducer"])
def test_flat_ddp_other_heads_gloo_world2(which):
    """DDP over the Paraformer (predictor, target embedding, no CTC head) and the
    Transducer (joint projections, LSTM prediction network): every parameter sits in a
    reducer unit, every unit's hook completes its bucket, gradients average over the two
    ranks."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    make = _tiny_paraformer if which == "paraformer" else _tiny_transducer
    procs = [ctx.Process(target=_paraformer_worker, args=(r, 2, port, q, make)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = out[0], out[1]
    heads = {"paraformer": ["decoder", "embed", "predictor"], "transducer": ["lin_jnt", "lin_dec", "decoder", "lin_enc"]}
    assert a["units"][:len(heads[which]) + 1] == heads[which] + ["encoder.after_norm"]
    assert a["nbuckets"] >= 2 and a["record"] == list(range(a["nbuckets"]))
    assert (a["flat"] == b["flat"]).all()
    g = torch.from_numpy(a["grad"])
    assert torch.equal(g, torch.from_numpy(b["grad"]))
    nz = g[g != 0]
    assert nz.numel() == g.numel() - int((g == 0).sum())
    assert torch.allclose(nz / 1.5, torch.round(nz / 1.5))  # ((0+1) i + (1+1) i) / 2


def _spans_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bench import CONFIGS, build
        from liteasr_amd.distributed.ddp import FlatReducer

        out = {}
        for name, model in (("tiny", _tiny()), ("small", build(CONFIGS["small"], "bf16", 0.1, "cpu"))):
            red = FlatReducer(model, bucket_bytes=25 * 1024 * 1024 if name == "small" else 2048)
            out[name] = (red.native_spans(), [[u.name for u in b] for b in red.buckets], model.store.numel,
                         [str(red._slice(b).data_ptr() - model.store.grad.data_ptr() if model.store.grad is not None
                              else "") for b in red.buckets])
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_native_spans_tile_flat_buffer_in_bucket_order():
    """The (lo, hi) spans the native reducer is given (FlatReducer.native_spans) are exactly the
    buckets' flat slices, in launch order, and tile [0, numel) with no gap or overlap; the
    launch order is backward-completion order (heads first, subsampling last).  For the small
    config the last bucket -- the one only the final backward segment precedes -- is the
    subsampling alone (7.35 MB of 184.8 MB)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    p = ctx.Process(target=_spans_worker, args=(0, 1, port, q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    for name, (spans, units, numel, _) in out.items():
        cover = sorted(spans)
        assert cover[0][0] == 0 and cover[-1][1] == numel, name
        for (a0, a1), (b0, b1) in zip(cover, cover[1:]):
            assert a1 == b0, (name, a1, b0)
        # launch order walks the flat buffer from the heads' end downwards (encoder layers are
        # laid out 0..n-1, and backward completes n-1..0)
        assert units[0][0] == "ctc" and units[-1][-1] == "encoder.embed.conv", (name, units)
    spans, units, numel, _ = out["small"]
    # the subsampling's output projection and its convolutions are buckets of their own: the
    # projection's is launched before the convolutions' backward, only 2.37 MB is left after it
    assert units[-2] == ["encoder.embed.out"] and units[-1] == ["encoder.embed.conv"]
    (lo0, hi0), (lo1, hi1) = spans[-2], spans[-1]
    assert abs((hi0 - lo0) * 4 / 1e6 - 4.98) < 0.05 and abs((hi1 - lo1) * 4 / 1e6 - 2.37) < 0.05
    assert len(spans) == 7
