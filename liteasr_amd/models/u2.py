"""U2: Conformer encoder + Transformer decoder + CTC (liteasr/models/u2.py), HIP path.

Same config schema, registry name, state_dict and call conventions as the reference:
``model(xs, xlens, ys, ylens) -> (h_attn (B, L+1, V), h_ctc (B, T', V))``.  The compute
runs in the fused HIP nodes of liteasr_amd.nets.functional; bookkeeping (masks,
decoder inputs, targets, CTC lengths) is one device kernel (lasr_u2_prep).

Extensions (default off = reference behaviour):
  compute_dtype  "bf16" (default; fp32 masters/accumulation) or "fp32" (parity build)
  chunk_size     > 0 adds triangle_mask(T', stage=chunk_size) to the encoder
                 self-attention mask (the dynamic-chunk config's oracle-by-composition)
"""

from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass, field
from enum import Enum
from types import SimpleNamespace
from typing import Optional, Tuple

import torch
from torch import Tensor

from .. import kernels as K
from ..config import II, MISSING, LiteasrDataclass
from ..nets import functional as FN
from .. import decoding as D
from ..nets.modules import CTC, TransformerDecoder, TransformerEncoder, _Bound
from ..utils.cfg import enum_value
from ..utils.param_store import FlatParams
from . import LiteasrModel, register_model


class EncoderArch(Enum):
    Transformer = "transformer"
    Conformer = "conformer"


class DecoderArch(Enum):
    Transformer = "transformer"


@dataclass
class U2Config(LiteasrDataclass):
    name: Optional[str] = field(default="U2")
    dropout_rate: float = field(default=0.0)
    enc_arch: EncoderArch = field(default=EncoderArch.Conformer)
    use_rel: bool = field(default=True)
    input_dim: int = field(default=MISSING)
    enc_dim: int = field(default=256)
    enc_ff_dim: int = field(default=2048)
    enc_attn_heads: int = field(default=4)
    enc_dropout_rate: float = II("model.dropout_rate")
    enc_pos_dropout_rate: float = II("model.enc_dropout_rate")
    enc_attn_dropout_rate: float = II("model.enc_dropout_rate")
    enc_ff_dropout_rate: float = II("model.enc_dropout_rate")
    enc_layers: int = field(default=12)
    activation: str = field(default="swish")
    dec_arch: DecoderArch = field(default=DecoderArch.Transformer)
    vocab_size: int = field(default=MISSING)
    dec_dim: int = field(default=256)
    dec_ff_dim: int = field(default=2048)
    dec_attn_heads: int = field(default=4)
    dec_dropout_rate: float = II("model.dropout_rate")
    dec_pos_dropout_rate: float = II("model.dec_dropout_rate")
    dec_self_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_src_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_ff_dropout_rate: float = II("model.dec_dropout_rate")
    dec_layers: int = field(default=6)
    # liteasr_amd extensions
    compute_dtype: str = field(default="bf16")
    chunk_size: int = field(default=0)


def _arch(v, enum):
    v = enum_value(v)
    if isinstance(v, str):
        for e in enum:
            if v.lower() in (e.value, e.name.lower()):
                return e.value
    return v


@register_model("U2", dataclass=U2Config)
class U2(LiteasrModel):
    def __init__(self, cfg: U2Config, task=None):
        super().__init__()
        g = lambda k, d=None: getattr(cfg, k, d)  # noqa: E731
        self.encoder = TransformerEncoder(
            use_rel=g("use_rel", True), i_dim=g("input_dim"), h_dim=g("enc_dim"), ff_dim=g("enc_ff_dim"),
            n_head=g("enc_attn_heads"), n_layer=g("enc_layers"), dropout_rate=float(g("enc_dropout_rate")),
            pos_dropout_rate=float(g("enc_pos_dropout_rate")), attn_dropout_rate=float(g("enc_attn_dropout_rate")),
            ff_dropout_rate=float(g("enc_ff_dropout_rate")), activation=g("activation", "swish"),
            arch=_arch(g("enc_arch", "conformer"), EncoderArch))
        self.decoder = TransformerDecoder(
            i_dim=g("vocab_size"), h_dim=g("dec_dim"), ff_dim=g("dec_ff_dim"), n_head=g("dec_attn_heads"),
            n_layer=g("dec_layers"), dropout_rate=float(g("dec_dropout_rate")),
            pos_dropout_rate=float(g("dec_pos_dropout_rate")),
            self_attn_dropout_rate=float(g("dec_self_attn_dropout_rate")),
            src_attn_dropout_rate=float(g("dec_src_attn_dropout_rate")),
            ff_dropout_rate=float(g("dec_ff_dropout_rate")), arch=_arch(g("dec_arch", "transformer"), DecoderArch))
        self.ctc = CTC(i_dim=g("enc_dim"), o_dim=g("vocab_size"), dropout_rate=float(g("dropout_rate", 0.0)))
        self.ignore = -1
        self.blank = 0
        self.sos = g("vocab_size") - 1
        self.eos = g("vocab_size") - 1
        cd = str(g("compute_dtype", "bf16")).lower()
        self.compute_dtype = torch.float32 if cd in ("fp32", "float32", "float") else torch.bfloat16
        self.chunk_size = int(g("chunk_size", 0) or 0)
        self.vocab_size = g("vocab_size")
        self._finalize()

    # ------------------------------------------------------------ flat params
    def _finalize(self):
        groups = []
        for name, mod in self.named_modules():
            if isinstance(mod, _Bound):
                mod._pfx = name
        for i, layer in enumerate(self.encoder.enc_layers):
            groups += layer.flat_groups()
            layer.seed = 1000 + 16 * i
        for i, layer in enumerate(self.decoder.dec_layers):
            groups += layer.flat_groups()
            layer.seed = 5000 + 16 * i
        self.store = FlatParams(self, groups, self.compute_dtype)
        for mod in self.modules():
            if isinstance(mod, _Bound):
                mod._store = self.store
        self.register_buffer("_drop_ctr", torch.zeros(1, dtype=torch.int64), persistent=False)
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

    # ------------------------------------------------------------- bookkeeping
    def get_pred_len(self, xlens) -> Tensor:
        """liteasr/models/u2.py:319-321."""
        return torch.div(torch.div(xlens - 1, 2, rounding_mode="floor") - 1, 2, rounding_mode="floor")

    def get_target(self, ys, ylens) -> Tuple[Tensor, Tensor]:
        """liteasr/models/u2.py:323-333."""
        ignore = torch.full((ys.size(0), 1), self.ignore, dtype=ys.dtype, device=ys.device)
        tgt_attn = torch.cat([ys, ignore], dim=1)
        tgt_attn[torch.arange(len(ylens), device=ys.device), ylens] = self.eos
        return tgt_attn, ys

    def get_target_len(self, ylens) -> Tensor:
        return ylens

    def _prep(self, xs, xlens, ys, ylens):
        dev = xs.device
        B, Tx = xs.shape[0], xs.shape[1]
        L = ys.shape[1]
        Tsub = ((Tx - 1) // 2 - 1) // 2
        i32, u8 = torch.int32, torch.uint8
        out = {
            "ys_in": torch.empty(B, L + 1, dtype=i32, device=dev),
            "tgt": torch.empty(B * (L + 1), dtype=i32, device=dev),
            "tgt_ctc": torch.empty(B, L, dtype=i32, device=dev),
            "dec_mask": torch.empty(B, L + 1, L + 1, dtype=u8, device=dev),
            "enc_mask": torch.empty(B, Tsub, dtype=u8, device=dev),
            "pred_len": torch.empty(B, dtype=i32, device=dev),
            "ylen": torch.empty(B, dtype=i32, device=dev),
        }
        xl = xlens.to(device=dev, dtype=torch.int64)
        yy = ys.to(device=dev, dtype=torch.int64).contiguous()
        yl = ylens.to(device=dev, dtype=torch.int64)
        K.u2_prep(xl, yy, yl, Tx, Tsub, self.sos, self.eos, 0, out)
        chunk = None
        if self.chunk_size > 0:
            tmp = dict(out)
            tmp["enc_mask"] = torch.empty(B, Tsub, Tsub, dtype=u8, device=dev)
            K.u2_prep(xl, yy, yl, Tx, Tsub, self.sos, self.eos, self.chunk_size, tmp)
            chunk = tmp["enc_mask"]
        p = SimpleNamespace(B=B, Tx=Tx, T=Tsub, L=L, chunk_mask=chunk, **out)
        return p

    def _run_encoder(self, xs, xlens, ys, ylens):
        """Bookkeeping (_prep) + Conv2DLayer/PE + conformer layers: the encoder residual
        stream x [B*T', d] fp32 (before after_norm), prep and the kernel env."""
        if xs.device.type != "cuda":
            raise RuntimeError("liteasr_amd.U2 runs on the HIP device only (no CPU path); "
                               "move the model and batch to cuda")
        prep = self._prep(xs, xlens, ys, ylens)
        self.last_prep = prep
        enc, dec = self.encoder, self.decoder
        tr = self.training
        er, dr = enc.rates, dec.rates
        B, T, L1 = prep.B, prep.T, prep.L + 1
        env = SimpleNamespace(
            B=B, T=T, L1=L1, H=enc.n_head, adt=self.compute_dtype, training=tr,
            p_drop=er.drop, p_ff=er.ff, p_att=er.att, p_pos=er.pos if tr else 0.0,
            p_ctc=self.ctc.dropout_rate,  # always on (liteasr/nets/ctc.py:29)
            p_dec=dr.drop, p_dec_ff=dr.ff, p_dec_att=dr.self_att, p_dec_src_att=dr.src_att,
            p_dec_pos=dr.pos, ys_in=prep.ys_in, dec_mask=prep.dec_mask, mask_k=prep.enc_mask,
            seed=self._seed_base)
        if prep.chunk_mask is not None:
            env.mask, env.msb, env.msq = prep.chunk_mask, T * T, T
        else:
            env.mask, env.msb, env.msq = prep.enc_mask, T, 0
        K.set_dropout_counter(self._drop_ctr)
        K.counter_add(self._drop_ctr, 1)
        self.store.working()
        if torch.is_grad_enabled():
            self.store.ensure_grad()  # p.grad views of the flat grad buffer (once per step)
        enc.embed.repack(self.compute_dtype)
        x = FN.EmbedFn.apply(xs.float(), enc.embed.out.weight, enc.embed, env)
        d = enc.h_dim
        pos = torch.empty(T, d, dtype=self.compute_dtype, device=xs.device)
        K.pe_fwd(None, T, T, d, enc.pe.table(T), 1.0, pos, env.p_pos, env.seed + 4)
        for j, layer in enumerate(enc.enc_layers):
            x = self._cut(x, j)
            x = FN.ConformerLayerFn.apply(x, pos, layer.final_norm.weight, layer, env)
        x = self._cut(x, len(enc.enc_layers))
        return x, prep, env

    # ---------------------------------------------------- backward segmentation
    @contextlib.contextmanager
    def segmented(self, cuts):
        """Cut the autograd graph of the encoder residual stream before encoder layer j
        for every j in ``cuts`` (j == enc_layers: between the last layer and the heads).
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

    # ----------------------------------------------------------------- forward
    def forward(self, xs, xlens, ys, ylens):
        x, prep, env = self._run_encoder(xs, xlens, ys, ylens)
        B, T, L1 = prep.B, prep.T, prep.L + 1
        h_attn, h_ctc = FN.HeadsFn.apply(x, self.ctc.ctc_lo.weight, self, env)
        return h_attn.view(B, L1, -1), h_ctc.view(B, T, -1)

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

    # --------------------------------------------------------------- inference
    def _prep_targets(self, ys, ylens, B, Tx):
        """_prep for a decoder-only pass: every one of the Tx frames valid."""
        xs = torch.empty(B, Tx, 0, device=ys.device)  # shape / device only
        xlens = torch.full((B,), Tx, dtype=torch.int64, device=ys.device)
        return self._prep(xs, xlens, ys, ylens)

    @torch.no_grad()
    def inference(self, x):
        """liteasr/models/u2.py:160-161."""
        return self.attention_rescore(x)

    @torch.no_grad()
    def attention(self, x):
        """liteasr/models/u2.py:163-216 (beam 10); returns the best hypothesis incl. sos."""
        return D.attention_beam_search(self, x, beam=10)

    @torch.no_grad()
    def _ctc_prefix_beam_search(self, x):
        """liteasr/models/u2.py:218-263: ([(tokens tuple, score)], h (1, T', d))."""
        hyps, h, T = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return [(tuple(t), sc) for t, sc in hyps], h.view(1, T, -1).clone()

    @torch.no_grad()
    def ctc_prefix_beam_search(self, x):
        """liteasr/models/u2.py:265-267."""
        hyps, _, _ = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return tuple(hyps[0][0])

    @torch.no_grad()
    def attention_rescore(self, x):
        """liteasr/models/u2.py:269-317 (ctc weight 0.5)."""
        hyps, h, T = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return tuple(hyps[D.rescore(self, hyps, h, T, ctc_weight=0.5)][0])

    @classmethod
    def build_model(cls, cfg: U2Config, task=None):
        cfg.input_dim = task.feat_dim
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)
