"""Shared host side of the models whose encoder is the fused Conformer stack
(liteasr/nets/transformer_encoder.py:28-127): flat parameter store, BN running-stat
buffers, bookkeeping kernel, the fused encoder forward, graph segmentation and the
reusable ``encode`` block.  U2 (liteasr/models/u2.py) and Paraformer
(liteasr/models/paraformer.py) build on it."""

from __future__ import annotations

import contextlib
from types import SimpleNamespace

import torch
from torch import Tensor

from .. import kernels as K
from ..nets import functional as FN
from ..nets.modules import _Bound
from ..utils.param_store import FlatParams
from . import LiteasrModel


def _require_hip(model, xs):
    """The fused models run on the HIP device only: there is no CPU path (tools/step_census.py,
    a host-only launch recorder, is the one caller that replaces this check)."""
    if xs.device.type != "cuda":
        raise RuntimeError(f"liteasr_amd.{type(model).__name__} runs on the HIP device only (no CPU path); "
                           "move the model and batch to cuda")


class FusedEncoderModel(LiteasrModel):
    """Subclasses build ``self.encoder`` (TransformerEncoder), ``self.decoder`` (with
    ``dec_layers`` and ``rates``), set ``compute_dtype``, ``chunk_size``, ``sos``/``eos``,
    then call ``_finalize()``."""

    # ------------------------------------------------------------ flat params
    def _finalize(self):
        groups = []
        for name, mod in self.named_modules():
            if isinstance(mod, _Bound):
                mod._pfx = name
        for i, layer in enumerate(self.encoder.enc_layers):
            groups += layer.flat_groups()
            layer.seed = 1000 + 16 * i
        dgroups = getattr(self.decoder, "flat_groups", None)  # Transformer decoders: cross-layer K/V
        for i, layer in enumerate(self.decoder.dec_layers):
            if dgroups is None:
                groups += layer.flat_groups()
            layer.seed = 5000 + 16 * i
        if dgroups is not None:
            groups += dgroups()
        self.store = FlatParams(self, groups, self.compute_dtype)
        for mod in self.modules():
            if isinstance(mod, _Bound):
                mod._store = self.store
        self.register_buffer("_drop_ctr", torch.zeros(1, dtype=torch.int64), persistent=False)
        # the streaming chunk size of the step (int32, device): written by the prep kernel when
        # it draws c (dynamic_chunk), read by it when chunk_from_device is set (see chunk_mode)
        self.register_buffer("_chunk_dev", torch.zeros(1, dtype=torch.int32), persistent=False)
        self.dynamic_chunk = bool(getattr(self, "dynamic_chunk", False))
        self.chunk_max = int(getattr(self, "chunk_max", 25))
        self.chunk_from_device = False
        self._flatten_bn()
        self.last_prep = None
        self._seed_base = 77
        self._seg = None  # active graph-segmentation cuts (see `segmented`)

    def _apply(self, fn, recurse=True):
        """Device/dtype moves act on the flat buffers; parameters stay views."""
        self.store.apply(fn)
        for mod in self.modules():
            for k, b in mod._buffers.items():
                if b is not None:
                    mod._buffers[k] = fn(b)
        self._flatten_bn()
        return self

    def _flatten_bn(self):
        """BatchNorm running statistics as views of two flat buffers (fp32 mean/var, int64
        num_batches_tracked), so the per-forward buffer broadcast of data parallelism
        (DDP broadcast_buffers, liteasr/trainer.py:80-84) is two collectives on
        contiguous memory instead of dozens of small copies + a coalesced broadcast."""
        bns = [m for m in self.modules() if isinstance(m, torch.nn.BatchNorm1d)]
        if not bns:
            self._bn_flat = ()
            return
        f32 = torch.cat([t.detach().reshape(-1).float() for m in bns for t in (m.running_mean, m.running_var)])
        i64 = torch.stack([m.num_batches_tracked.detach().reshape(()) for m in bns])
        off = 0
        for i, m in enumerate(bns):
            C = m.running_mean.numel()
            m._buffers["running_mean"] = f32[off:off + C]
            m._buffers["running_var"] = f32[off + C:off + 2 * C]
            m._buffers["num_batches_tracked"] = i64[i]
            off += 2 * C
        self._bn_flat = (f32, i64)

    def bn_flat_buffers(self):
        """The flat BN running-statistics buffers (see ``_flatten_bn``)."""
        return list(self._bn_flat)

    def flat_parameters(self):
        return self.store

    # ------------------------------------------------------ data-parallel units
    _unit_hook = None

    def reducer_units(self):
        """Parameter-prefix units in the order the fused backward completes them (the
        bucket order of distributed.ddp.FlatReducer): the heads, then the encoder top-down.
        Every name must fire a ready hook (a _Bound module's on_grads_ready, the encoder's
        after_norm_ready, or unit_ready)."""
        enc = self.encoder
        return (self._head_units() + ["encoder.after_norm"] + [l._pfx for l in reversed(list(enc.enc_layers))]
                + [enc.embed._n(u) for u in enc.embed.UNITS])

    def reducer_bucket_breaks(self):
        """Units that always start a new gradient bucket: the subsampling convolutions, so
        the output projection's bucket is launched before their backward and only the
        convolutions' gradients (2.4 MB at d 256) remain to reduce after the last segment."""
        return {self.encoder.embed._n("conv")}

    def _head_units(self):
        return ["ctc", "decoder"]

    def unit_ready(self, name):
        """A reducer unit that is not a _Bound module has its gradients complete."""
        if self._unit_hook is not None:
            self._unit_hook(name)

    # ------------------------------------------------------------- bookkeeping
    def get_pred_len(self, xlens) -> Tensor:
        """liteasr/models/u2.py:319-321."""
        return torch.div(torch.div(xlens - 1, 2, rounding_mode="floor") - 1, 2, rounding_mode="floor")

    def chunk_mode(self):
        """How the encoder's streaming chunk mask is formed this step (lasr_u2_prep_chunk):
        none (key padding only), a fixed ``chunk_size`` > 0, the device scalar ``_chunk_dev``
        (``chunk_from_device``: set it with ``set_chunk`` between graph replays), or a per-step
        draw on the device (``dynamic_chunk``, training mode only: WeNet's distribution, see
        ``dynamic_chunk_size``; in eval mode a dynamic-chunk model uses ``chunk_size``)."""
        if self.dynamic_chunk and self.training:
            return K.CHUNK_SAMPLE
        if self.chunk_from_device:
            return K.CHUNK_DEVICE
        return K.CHUNK_FIXED if self.chunk_size > 0 else K.CHUNK_NONE

    def set_chunk(self, c):
        """Device-scalar chunk size (stream-ordered write; c <= 0 or c >= T' = full context)
        for ``chunk_from_device`` mode: a captured step reads it at every replay."""
        self._chunk_dev.fill_(int(c))

    def last_chunk(self):
        """The chunk size the last prep used in dynamic / device mode (host sync)."""
        return int(self._chunk_dev.item())

    @staticmethod
    def dynamic_chunk_size(seed, ctr, Tsub, cmax=25):
        """Host mirror of the prep kernel's draw (csrc/prep.hip chunk_draw) for step counter
        value ``ctr``: r uniform in [1, T'-1]; r > T'/2 -> full context (returns T'), else
        r mod cmax + 1 (wenet/utils/mask.py add_optional_chunk_mask's distribution)."""
        M32, M64 = 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF

        def mix32(x):
            x &= M32
            x ^= x >> 16
            x = (x * 0x7FEB352D) & M32
            x ^= x >> 15
            x = (x * 0x846CA68B) & M32
            x ^= x >> 16
            return x

        if Tsub <= 1:
            return max(Tsub, 1)
        s = (seed + ctr * 0xD1B54A32D192ED03) & M64
        key = mix32((s & M32) ^ mix32(((s >> 32) + 0x9E3779B9) & M32))
        h = mix32(key ^ 0x5BD1E995)
        r = 1 + h % (Tsub - 1)
        return Tsub if r > Tsub // 2 else r % cmax + 1

    def _prep(self, xs, xlens, ys, ylens):
        dev = xs.device
        B, Tx = xs.shape[0], xs.shape[1]
        L = ys.shape[1]
        Tsub = ((Tx - 1) // 2 - 1) // 2
        i32, u8 = torch.int32, torch.uint8
        # query-dependent masks with 16-B aligned rows (the attention kernels stage their tiles
        # by LDS-DMA): u2_prep writes the padded rows itself (padding columns masked)
        P16 = lambda n: (n + 15) // 16 * 16  # noqa: E731
        out = {
            "ys_in": torch.empty(B, L + 1, dtype=i32, device=dev),
            "tgt": torch.empty(B * (L + 1), dtype=i32, device=dev),
            "tgt_ctc": torch.empty(B, L, dtype=i32, device=dev),
            "dec_mask": torch.empty(B, L + 1, P16(L + 1), dtype=u8, device=dev),
            "enc_mask": torch.empty(B, Tsub, dtype=u8, device=dev),
            "pred_len": torch.empty(B, dtype=i32, device=dev),
            "ylen": torch.empty(B, dtype=i32, device=dev),
        }
        xl = xlens.to(device=dev, dtype=torch.int64)
        yy = ys.to(device=dev, dtype=torch.int64).contiguous()
        yl = ylens.to(device=dev, dtype=torch.int64)
        mode = self.chunk_mode()
        if mode != K.CHUNK_NONE:
            out["chunk_mask"] = torch.empty(B, Tsub, P16(Tsub), dtype=u8, device=dev)
        K.u2_prep(xl, yy, yl, Tx, Tsub, self.sos, self.eos, self.chunk_size, out, chunk_mode=mode,
                  chunk_dev=self._chunk_dev, ctr=self._drop_ctr, chunk_seed=self._seed_base + 11,
                  chunk_max=self.chunk_max)
        chunk = out.pop("chunk_mask")[:, :, :Tsub] if mode != K.CHUNK_NONE else None
        # kernels read the masks through (msb, msq) = the views' strides
        out["dec_mask"] = out["dec_mask"][:, :, :L + 1]
        p = SimpleNamespace(B=B, Tx=Tx, T=Tsub, L=L, chunk_mask=chunk, **out)
        return p

    def _run_encoder(self, xs, xlens, ys, ylens):
        """Bookkeeping (_prep) + Conv2DLayer/PE + conformer layers: the encoder residual
        stream x [B*T', d] fp32 (before after_norm), prep and the kernel env."""
        _require_hip(self, xs)
        prep = self._prep(xs, xlens, ys, ylens)
        self.last_prep = prep
        enc, dec = self.encoder, self.decoder
        tr = self.training
        er, dr = enc.rates, dec.rates
        ctc = getattr(self, "ctc", None)
        B, T, L1 = prep.B, prep.T, prep.L + 1
        env = SimpleNamespace(
            B=B, T=T, L1=L1, H=enc.n_head, adt=self.compute_dtype, training=tr,
            p_drop=er.drop, p_ff=er.ff, p_att=er.att, p_pos=er.pos if tr else 0.0,
            p_ctc=ctc.dropout_rate if ctc is not None else 0.0,  # always on (liteasr/nets/ctc.py:29)
            p_dec=dr.drop, p_dec_ff=dr.ff, p_dec_att=dr.self_att, p_dec_src_att=dr.src_att,
            p_dec_pos=getattr(dr, "pos", 0.0), ys_in=prep.ys_in, dec_mask=prep.dec_mask, mask_k=prep.enc_mask,
            seed=self._seed_base)
        if prep.chunk_mask is not None:
            env.mask, env.msb, env.msq = prep.chunk_mask, prep.chunk_mask.stride(0), prep.chunk_mask.stride(1)
        else:
            env.mask, env.msb, env.msq = prep.enc_mask, T, 0
        K.set_dropout_counter(self._drop_ctr)
        K.counter_add(self._drop_ctr, 1)
        self.store.working()
        if torch.is_grad_enabled():
            self.store.ensure_grad()  # p.grad views of the flat grad buffer (once per step)
        enc.embed.repack(self.compute_dtype)
        d = enc.h_dim
        rel = getattr(enc, "use_rel", True)
        env.abs_pe = None if rel else enc.pe.table(T)  # absolute PE: added to x in the embed node
        x = FN.EmbedFn.apply(xs.float(), enc.embed.out.weight, enc.embed, env, cut=lambda y: self._cut(y, -1))
        pos, pp = None, None
        if rel:  # relative PE: the dropped-out table feeds every layer's positional projection
            pos = torch.empty(T, d, dtype=self.compute_dtype, device=xs.device)
            K.pe_fwd(None, T, T, d, enc.pe.table(T), 1.0, pos, env.p_pos, env.seed + 4)
            pp = FN.pos_projections(pos, [layer.weights().att.Wpos for layer in enc.enc_layers]) \
                if FN.BATCH_POS_PROJ else None
        env.pos_proj = {id(layer): p for layer, p in zip(enc.enc_layers, pp)} if pp else None
        layers = list(enc.enc_layers)
        conformer = getattr(enc, "arch", "conformer") == "conformer"
        env.pre_ln = env.bwd_chain = None
        # layer nodes that launch the queued parameter-gradient reductions (FN.LAYER_RED_HOLD):
        # the lowest layer, and the lowest layer of every backward segment (a cut before layer j)
        seg = self._seg
        env.red_flush = {id(layers[0])} if layers else set()
        if seg is not None:
            env.red_flush |= {id(layers[j]) for j in seg.cuts if 0 <= j < len(layers)}
        for j, layer in enumerate(layers):
            x = self._cut(x, j)
            if not conformer:  # Transformer layers: no final norm to chain the next first norm into
                env.next_ln = None
                x = FN.TransformerLayerFn.apply(x, pos, layer.feed_forward_norm.weight, layer, env)
                continue
            if j + 1 < len(layers):
                wn = layers[j + 1].weights().ln_a
                env.next_ln = (layers[j + 1], wn.g, wn.b)
            else:
                env.next_ln = None
            x = FN.ConformerLayerFn.apply(x, pos, layer.final_norm.weight, layer, env)
        env.next_ln = env.pre_ln = None
        x = self._cut(x, len(enc.enc_layers))
        return x, prep, env

    # ---------------------------------------------------- backward segmentation
    @contextlib.contextmanager
    def segmented(self, cuts):
        """Cut the autograd graph of the encoder residual stream before encoder layer j
        for every j in ``cuts`` (j == enc_layers: between the last layer and the heads;
        j == -1: inside the subsampling, between its convolutions and its output projection).
        Inside the block each forward appends ``(j, x, x_leaf)`` to the yielded list,
        where ``x_leaf = x.detach().requires_grad_()`` is what the rest of the forward
        consumes, so the backward can run as separate pieces (``torch.autograd.grad`` from
        the loss down to the top ``x_leaf``, then from each ``x`` down to the next leaf).
        liteasr_amd.graph_step captures each piece as its own hipGraph so the data-parallel
        gradient buckets can be all-reduced between the pieces, overlapping the rest of
        the backward (the reference gets this overlap from DDP's autograd hooks,
        liteasr/trainer.py:76-88).  Numerics are unchanged: the pieces run the same fused
        backward nodes in the same order."""
        self._seg = SimpleNamespace(cuts=frozenset(int(c) for c in cuts), pairs=[])
        try:
            yield self._seg.pairs
        finally:
            self._seg = None

    def _cut(self, x, j):
        seg = self._seg
        if seg is None or j not in seg.cuts or not x.requires_grad:
            return x
        leaf = x.detach().requires_grad_(True)
        seg.pairs.append((j, x, leaf))
        return leaf

    def encode(self, xs, xlens):
        """`self.encoder(xs, mask=padding_mask(xlens))` (transformer_encoder.py:107-127) as a
        reusable, differentiable block: (h (B, T', d) fp32, key mask (B, T') bool, True =
        padding).  Training-mode dropout / BN batch statistics follow `self.training`;
        gradients reach the flat parameter store through the fused layer backward."""
        B = xs.shape[0]
        ys = torch.full((B, 1), -1, dtype=torch.int64, device=xs.device)
        ylens = torch.zeros(B, dtype=torch.int64, device=xs.device)
        x, prep, env = self._run_encoder(xs, xlens, ys, ylens)
        h = FN.EncoderOutFn.apply(x, self.encoder.after_norm.weight, self, self.compute_dtype)
        return h.view(B, prep.T, -1), prep.enc_mask.bool()

