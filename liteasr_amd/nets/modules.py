"""nn.Module tree of the U2 hot path, mirroring liteasr.nets attribute-for-attribute.

The constructors build the same torch parameter containers (nn.Linear, nn.Conv1d/2d,
nn.BatchNorm1d, nn.LayerNorm, nn.Embedding) in the same order as the reference, so
``torch.manual_seed(s); U2(cfg)`` yields bit-identical initial weights and identical
``state_dict`` keys (checked against the reference by tests/test_oracle_golden.py).
The arithmetic does NOT run through these containers: after construction the top
model moves every parameter into a FlatParams store and the forward/backward run the
fused HIP nodes of ``functional.py``.

Each module knows its state_dict prefix (``_pfx``) and the store (``_store``) and
exposes ``weights()`` (working-copy / fp32 views for the kernels), ``grads()``
(views into the flat fp32 grad buffer) and ``on_grads_ready()`` (DDP bucket hook).
"""

from __future__ import annotations

import math
from types import SimpleNamespace

import torch
import torch.nn as nn


class _Bound(nn.Module):
    """Mixin: access to the owning FlatParams store."""

    _store = None
    _pfx = ""
    _ready_hook = None

    def _n(self, name):
        return f"{self._pfx}.{name}" if self._pfx else name

    def _w(self, name):  # GEMM operand: working (compute-dtype) copy
        return self._store.work_view(self._n(name))

    def _p(self, name):  # fp32 master (biases, norms, small weights read in fp32)
        return self._store.view(self._n(name))

    def _g(self, name):
        return self._store.grad_view(self._n(name))

    def _wg(self, names, rows):  # contiguous group, working copy
        return self._store.work_group([self._n(n) for n in names], rows)

    def _pg(self, names, rows=None):
        return self._store.group_view([self._n(n) for n in names], rows_of=rows)

    def _gg(self, names, rows=None):
        return self._store.grad_group([self._n(n) for n in names], rows)

    def on_grads_ready(self):
        if self._ready_hook is not None:
            self._ready_hook(self)

    def _cached(self, key, fn):
        """View bundles are rebuilt only when the store's buffers were reallocated."""
        gen = self._store.generation
        c = self.__dict__.get("_vcache")
        if c is None or c[0] != gen:
            c = (gen, {})
            self.__dict__["_vcache"] = c
        v = c[1].get(key)
        if v is None:
            v = c[1][key] = fn()
        return v


class LayerNorm(nn.LayerNorm):
    """liteasr/nets/layer_norm.py:8-21 (eps = 1e-12)."""

    def __init__(self, nout: int, dim=-1):
        super().__init__(nout, eps=1e-12)
        self.dim = dim


class Swish(nn.Module):
    """liteasr/nets/swish.py:7-16 (fused into the FFN GEMM epilogue on the HIP path)."""

    def forward(self, x):
        return x * torch.sigmoid(x)


class PositionwiseFeedForward(nn.Module):
    """liteasr/nets/feed_forward.py:4-19."""

    def __init__(self, i_dim, h_units, dropout_rate, activation=None):
        super().__init__()
        self.fc1 = nn.Linear(i_dim, h_units)
        self.fc2 = nn.Linear(h_units, i_dim)
        self.dropout = nn.Dropout(dropout_rate)
        self.activation = activation if activation is not None else nn.ReLU()


class MultiHeadAttention(nn.Module):
    """liteasr/nets/attention.py:8-71."""

    def __init__(self, n_head, i_dim, dropout_rate):
        super().__init__()
        assert i_dim % n_head == 0
        self.d_k = i_dim // n_head
        self.scaling = self.d_k ** -0.5
        self.h = n_head
        self.linear_q = nn.Linear(i_dim, i_dim)
        self.linear_k = nn.Linear(i_dim, i_dim)
        self.linear_v = nn.Linear(i_dim, i_dim)
        self.linear_o = nn.Linear(i_dim, i_dim)
        self.dropout = nn.Dropout(dropout_rate)
        self.softmax = nn.Softmax(dim=-1)


class RelativeMultiHeadAttention(MultiHeadAttention):
    """liteasr/nets/attention.py:74-154 (legacy rel_shift)."""

    def __init__(self, n_head, i_dim, dropout_rate):
        super().__init__(n_head, i_dim, dropout_rate)
        self.linear_pos = nn.Linear(i_dim, i_dim, bias=False)
        self.pos_bias_u = nn.Parameter(torch.Tensor(self.h, self.d_k))
        self.pos_bias_v = nn.Parameter(torch.Tensor(self.h, self.d_k))
        torch.nn.init.xavier_uniform_(self.pos_bias_u)
        torch.nn.init.xavier_uniform_(self.pos_bias_v)


class Convolution(nn.Module):
    """liteasr/nets/conformer_convolution.py:4-57."""

    def __init__(self, channels, kernel_size, bias=True, activation=None):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0
        self.pointwise_conv1 = nn.Conv1d(channels, 2 * channels, 1, 1, 0, bias=bias)
        self.depthwise_conv = nn.Conv1d(channels, channels, kernel_size, 1, (kernel_size - 1) // 2,
                                        groups=channels, bias=bias)
        self.pointwise_conv2 = nn.Conv1d(channels, channels, 1, 1, 0, bias=bias)
        self.norm = nn.BatchNorm1d(num_features=channels)
        self.activation = activation if activation is not None else nn.ReLU()


class PositionalEncoding(nn.Module):
    """liteasr/nets/positional_encoding.py:9-56: sin/cos table registered as ``pe``."""

    def __init__(self, h_dim, dropout_rate, max_len=5000):
        super().__init__()
        if h_dim % 2 != 0:
            raise ValueError(f"Cannot use sin/cos positional encoding with odd dim (got dim={h_dim})")
        self.h_dim = h_dim
        self.scale = math.sqrt(h_dim)
        self.dropout = nn.Dropout(dropout_rate)
        self.max_len = max_len
        self.register_buffer("pe", self.init_pe())

    def init_pe(self):
        pe = torch.zeros(self.max_len, self.h_dim)
        position = torch.arange(0, self.max_len).unsqueeze(1).float()
        div_term = torch.exp(torch.arange(0, self.h_dim, 2).float() * -(math.log(10000.0) / self.h_dim))
        pe[:, 0::2] = torch.sin(position * div_term)
        pe[:, 1::2] = torch.cos(position * div_term)
        return pe.unsqueeze(0)

    def table(self, T):
        """fp32 [>=T, d] table on the model device (extends like extend_pe, :40-47)."""
        if self.pe.size(1) < T:
            self.max_len = T
            self.pe = self.init_pe().to(self.pe.device)
        return self.pe[0]


class RelativePositionalEncoding(PositionalEncoding):
    """liteasr/nets/positional_encoding.py:59-75."""


class Conv2DLayer(_Bound):
    """liteasr/nets/subsampling.py:9-48."""

    def __init__(self, i_dim, o_dim, dropout_rate):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(1, o_dim, 3, 2), nn.ReLU(), nn.Conv2d(o_dim, o_dim, 3, 2),
                                  nn.ReLU())
        f_dim = (i_dim - 3) // 2 + 1
        f_dim = (f_dim - 3) // 2 + 1
        self.f_dim = f_dim
        self.o_dim = o_dim
        self.out = nn.Linear(o_dim * f_dim, o_dim)
        self._repack = None

    def repack(self, work_dtype):
        """Kernel-layout working copies: conv2 [C,(kh,kw,cin)], out [d,(f,c)]."""
        from .. import kernels as K

        C, F2 = self.o_dim, self.f_dim
        dev = self._store.flat.device
        if self._repack is None or self._repack[0].device != dev or self._repack[0].dtype != work_dtype:
            self._repack = (torch.empty(C, 9 * C, dtype=work_dtype, device=dev),
                            torch.empty(C, F2 * C, dtype=work_dtype, device=dev))
        W2p, Woutp = self._repack
        K.permute_last2(self._p("conv.2.weight"), C, C, 9, W2p)
        K.permute_last2(self._p("out.weight"), C, C, F2, Woutp)

    def weights(self):
        C = self.o_dim
        W2p, Woutp = self._repack
        return SimpleNamespace(C=C, d=C, W1=self._p("conv.0.weight").view(C, 9), b1=self._p("conv.0.bias"),
                               W2p=W2p, b2=self._p("conv.2.bias"), Woutp=Woutp,
                               bout=self._p("out.bias"))

    def grads(self):
        C = self.o_dim
        return SimpleNamespace(W1=self._g("conv.0.weight").view(C, 9), b1=self._g("conv.0.bias"),
                               conv2_w=self._g("conv.2.weight"), b2=self._g("conv.2.bias"),
                               out_w=self._g("out.weight"), bout=self._g("out.bias"))

    # two data-parallel reducer units (models/_fused.py reducer_units): the output projection's
    # gradients complete before the convolutions' backward runs (nets/functional.py EmbedOutFn)
    UNITS = ("out", "conv")

    def conv_anchor(self):
        """The parameter EmbedConvFn takes as its autograd anchor."""
        return self.conv[0].weight

    def unit_ready(self, part):
        """Gradients of ``<prefix>.<part>`` (``out`` / ``conv``) are complete."""
        if self._ready_hook is not None:
            self._ready_hook(self._n(part))


class _LayerCommon(_Bound):
    def _ln(self, name, grad=False):
        f = self._g if grad else self._p
        return SimpleNamespace(g=f(name + ".weight"), b=f(name + ".bias"))

    def _ffn(self, name, grad=False):
        if grad:
            return SimpleNamespace(W1=self._g(name + ".fc1.weight"), b1=self._g(name + ".fc1.bias"),
                                   W2=self._g(name + ".fc2.weight"), b2=self._g(name + ".fc2.bias"))
        return SimpleNamespace(W1=self._w(name + ".fc1.weight"), b1=self._p(name + ".fc1.bias"),
                               W2=self._w(name + ".fc2.weight"), b2=self._p(name + ".fc2.bias"))


QKV_W = ("linear_q.weight", "linear_k.weight", "linear_v.weight")
QKV_B = ("linear_q.bias", "linear_k.bias", "linear_v.bias")
KV_W = ("linear_k.weight", "linear_v.weight")
KV_B = ("linear_k.bias", "linear_v.bias")


def _act_code(activation):
    """The encoder activation module -> the kernels' epilogue code (Swish or ReLU)."""
    from .._native import ACT_RELU, ACT_SWISH

    return ACT_SWISH if isinstance(activation, Swish) else ACT_RELU


def _att_weights(layer, grad):
    """Self-attention operand views of an encoder layer: the fused q/k/v projection, the
    output projection and, for the relative-position attention (attention.py:74-154), the
    positional projection and the two position biases (rel False: None)."""
    d = layer.size
    a = "self_attn."
    rel = layer.rel
    if grad:
        return SimpleNamespace(Wqkv=layer._gg([a + n for n in QKV_W], d), bqkv=layer._gg([a + n for n in QKV_B]),
                               Wpos=layer._g(a + "linear_pos.weight") if rel else None,
                               u=layer._g(a + "pos_bias_u").view(-1) if rel else None,
                               v=layer._g(a + "pos_bias_v").view(-1) if rel else None,
                               Wo=layer._g(a + "linear_o.weight"), bo=layer._g(a + "linear_o.bias"))
    return SimpleNamespace(Wqkv=layer._wg([a + n for n in QKV_W], d), bqkv=layer._pg([a + n for n in QKV_B]),
                           Wpos=layer._w(a + "linear_pos.weight") if rel else None,
                           u=layer._p(a + "pos_bias_u").view(-1) if rel else None,
                           v=layer._p(a + "pos_bias_v").view(-1) if rel else None,
                           Wo=layer._w(a + "linear_o.weight"), bo=layer._p(a + "linear_o.bias"))


def _att_groups(layer):
    a = layer._pfx + ".self_attn."
    g = [[a + n for n in QKV_W], [a + n for n in QKV_B]]
    return g + [[a + "pos_bias_u", a + "pos_bias_v"]] if layer.rel else g


class RelativeEncoderLayer(_LayerCommon):
    """Conformer encoder layer: RelativeEncoderLayer (liteasr/nets/conformer_layer.py:84-147)
    with a RelativeMultiHeadAttention, or EncoderLayer (:10-81, use_rel False) with a plain
    MultiHeadAttention (+ the EncoderLayer base of liteasr/nets/transformer_layer.py:10-27);
    the FFN / conv-module activation is Swish or ReLU (transformer_encoder.py:77-80)."""

    def __init__(self, size, self_attn, feed_forward, feed_forward_macaron, conv, dropout_rate,
                 normalize_before=True, concat_after=False):
        super().__init__()
        assert normalize_before, "only the pre-norm (default) layer is on the hot path"
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.self_attn_norm = LayerNorm(size)
        self.feed_forward_norm = LayerNorm(size)
        self.dropout = nn.Dropout(dropout_rate)
        self.size = size
        self.normalize_before = normalize_before
        self.feed_forward_macaron = feed_forward_macaron
        self.conv = conv
        self.feed_forward_macaron_norm = LayerNorm(size)
        self.conv_norm = LayerNorm(size)
        self.final_norm = LayerNorm(size)
        self.feed_forward_scale = 0.5
        self.seed = 0
        self.rel = isinstance(self_attn, RelativeMultiHeadAttention)
        self.act = _act_code(feed_forward.activation)

    def flat_groups(self):
        return _att_groups(self)

    def weights(self):
        return self._cached("w", self._weights)

    def grads(self):
        return self._cached("g", self._grads)

    def _weights(self):
        d = self.size
        c = "conv."
        bn = self.conv.norm
        return SimpleNamespace(
            ln_a=self._ln("feed_forward_macaron_norm"), ln_b=self._ln("self_attn_norm"),
            ln_c=self._ln("conv_norm"), ln_d=self._ln("feed_forward_norm"), ln_f=self._ln("final_norm"),
            ffm=self._ffn("feed_forward_macaron"), ff=self._ffn("feed_forward"),
            att=_att_weights(self, False), act=self.act,
            conv=SimpleNamespace(act=self.act, Wpw1=self._w(c + "pointwise_conv1.weight").view(2 * d, d),
                                 bpw1=self._p(c + "pointwise_conv1.bias"),
                                 wdw=self._p(c + "depthwise_conv.weight").view(d, -1),
                                 bdw=self._p(c + "depthwise_conv.bias"),
                                 kernel=self.conv.depthwise_conv.kernel_size[0],
                                 Wpw2=self._w(c + "pointwise_conv2.weight").view(d, d),
                                 bpw2=self._p(c + "pointwise_conv2.bias"),
                                 gamma=self._p(c + "norm.weight"), beta=self._p(c + "norm.bias"),
                                 rmean=bn.running_mean, rvar=bn.running_var, nbt=bn.num_batches_tracked))

    def _grads(self):
        d = self.size
        c = "conv."
        return SimpleNamespace(
            ln_a=self._ln("feed_forward_macaron_norm", True), ln_b=self._ln("self_attn_norm", True),
            ln_c=self._ln("conv_norm", True), ln_d=self._ln("feed_forward_norm", True),
            ln_f=self._ln("final_norm", True),
            ffm=self._ffn("feed_forward_macaron", True), ff=self._ffn("feed_forward", True),
            att=_att_weights(self, True),
            conv=SimpleNamespace(Wpw1=self._g(c + "pointwise_conv1.weight").view(2 * d, d),
                                 bpw1=self._g(c + "pointwise_conv1.bias"),
                                 wdw=self._g(c + "depthwise_conv.weight").view(d, -1),
                                 bdw=self._g(c + "depthwise_conv.bias"),
                                 Wpw2=self._g(c + "pointwise_conv2.weight").view(d, d),
                                 bpw2=self._g(c + "pointwise_conv2.bias"),
                                 gamma=self._g(c + "norm.weight"), beta=self._g(c + "norm.bias")))


class TransformerEncoderLayer(_LayerCommon):
    """Transformer encoder layer (enc_arch "transformer"): EncoderLayer / RelativeEncoderLayer
    of liteasr/nets/transformer_layer.py:10-136, pre-norm: x + drop(MHA(LN(x))), then
    x + drop(FFN(LN(x))) with the FFN's default ReLU (feed_forward.py:11)."""

    def __init__(self, size, self_attn, feed_forward, dropout_rate, normalize_before=True, concat_after=False):
        super().__init__()
        assert normalize_before, "only the pre-norm (default) layer is on the hot path"
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.self_attn_norm = LayerNorm(size)
        self.feed_forward_norm = LayerNorm(size)
        self.dropout = nn.Dropout(dropout_rate)
        self.size = size
        self.normalize_before = normalize_before
        self.seed = 0
        self.rel = isinstance(self_attn, RelativeMultiHeadAttention)
        self.act = _act_code(feed_forward.activation)

    def flat_groups(self):
        return _att_groups(self)

    def weights(self):
        return self._cached("w", lambda: SimpleNamespace(
            ln_b=self._ln("self_attn_norm"), ln_d=self._ln("feed_forward_norm"), ff=self._ffn("feed_forward"),
            att=_att_weights(self, False), act=self.act))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(
            ln_b=self._ln("self_attn_norm", True), ln_d=self._ln("feed_forward_norm", True),
            ff=self._ffn("feed_forward", True), att=_att_weights(self, True)))


class DecoderLayer(_LayerCommon):
    """liteasr/nets/transformer_layer.py:139-221 (pre-norm)."""

    def __init__(self, size, self_attn, src_attn, feed_forward, dropout_rate, normalize_before=True,
                 concat_after=False):
        super().__init__()
        assert normalize_before
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.self_attn_norm = LayerNorm(size)
        self.feed_forward_norm = LayerNorm(size)
        self.dropout = nn.Dropout(dropout_rate)
        self.size = size
        self.normalize_before = normalize_before
        self.src_attn = src_attn
        self.src_attn_norm = LayerNorm(size)
        self.seed = 0

    def flat_groups(self, kv=True):
        """kv False: the source attention's key/value weights are grouped by the decoder
        across its layers instead (decoder_kv_groups)."""
        s = self._pfx + ".self_attn."
        c = self._pfx + ".src_attn."
        g = [[s + n for n in QKV_W], [s + n for n in QKV_B]]
        return g + [[c + n for n in KV_W], [c + n for n in KV_B]] if kv else g

    def _w_all(self, grad):
        d = self.size
        wg = (lambda names, rows: self._gg(names, rows)) if grad else (lambda names, rows: self._wg(names, rows))
        pg = (lambda names: self._gg(names)) if grad else (lambda names: self._pg(names))
        w1 = self._g if grad else self._w
        p1 = self._g if grad else self._p
        s, c = "self_attn.", "src_attn."
        return SimpleNamespace(
            ln1=self._ln("self_attn_norm", grad), ln2=self._ln("src_attn_norm", grad),
            ln3=self._ln("feed_forward_norm", grad), ff=self._ffn("feed_forward", grad),
            sa=SimpleNamespace(Wqkv=wg([s + n for n in QKV_W], d), bqkv=pg([s + n for n in QKV_B]),
                               Wo=w1(s + "linear_o.weight"), bo=p1(s + "linear_o.bias")),
            ca=SimpleNamespace(Wq=w1(c + "linear_q.weight"), bq=p1(c + "linear_q.bias"),
                               Wkv=wg([c + n for n in KV_W], d), bkv=pg([c + n for n in KV_B]),
                               Wo=w1(c + "linear_o.weight"), bo=p1(c + "linear_o.bias")))


class TransformerEncoder(_Bound):
    """liteasr/nets/transformer_encoder.py:28-127: Conv2DLayer, the relative (use_rel) or
    absolute positional encoding, n_layer Conformer (arch "conformer", Swish or ReLU) or
    Transformer (arch "transformer") layers with relative or plain self-attention, after_norm.
    Constructed in the reference's order (same seed -> same initial weights)."""

    def __init__(self, use_rel, i_dim, h_dim, ff_dim, n_head, n_layer, dropout_rate, pos_dropout_rate,
                 attn_dropout_rate, ff_dropout_rate, activation, arch):
        super().__init__()
        if arch not in ("conformer", "transformer") or (arch == "conformer" and activation not in ("swish", "relu")):
            raise ValueError(f"encoder arch {arch!r} / activation {activation!r}: the reference builds "
                             "conformer (swish | relu) and transformer")
        self.embed = Conv2DLayer(i_dim, h_dim, dropout_rate)
        self.use_rel = bool(use_rel)
        pe = RelativePositionalEncoding if use_rel else PositionalEncoding
        mha = RelativeMultiHeadAttention if use_rel else MultiHeadAttention
        self.pe = pe(h_dim, dropout_rate=pos_dropout_rate)
        self.arch = arch
        if arch == "transformer":
            self.enc_layers = nn.ModuleList([
                TransformerEncoderLayer(
                    size=h_dim,
                    self_attn=mha(n_head, h_dim, attn_dropout_rate),
                    feed_forward=PositionwiseFeedForward(h_dim, ff_dim, dropout_rate=ff_dropout_rate),
                    dropout_rate=dropout_rate,
                ) for _ in range(n_layer)
            ])
        else:
            act = nn.ReLU() if activation == "relu" else Swish()
            self.enc_layers = nn.ModuleList([
                RelativeEncoderLayer(
                    size=h_dim,
                    self_attn=mha(n_head, h_dim, attn_dropout_rate),
                    feed_forward=PositionwiseFeedForward(h_dim, ff_dim, dropout_rate=ff_dropout_rate, activation=act),
                    feed_forward_macaron=PositionwiseFeedForward(h_dim, ff_dim, dropout_rate=ff_dropout_rate,
                                                                 activation=act),
                    conv=Convolution(h_dim, 15, activation=act),
                    dropout_rate=dropout_rate,
                ) for _ in range(n_layer)
            ])
        self.after_norm = LayerNorm(h_dim)
        self.h_dim, self.n_head = h_dim, n_head
        self.rates = SimpleNamespace(drop=dropout_rate, pos=pos_dropout_rate, att=attn_dropout_rate,
                                     ff=ff_dropout_rate)

    _after_norm_hook = None

    def after_norm_ready(self):
        if self._after_norm_hook is not None:
            self._after_norm_hook("encoder.after_norm")

    def after_norm_weights(self):
        return SimpleNamespace(g=self._p("after_norm.weight"), b=self._p("after_norm.bias"))

    def after_norm_grads(self):
        return SimpleNamespace(g=self._g("after_norm.weight"), b=self._g("after_norm.bias"))


def decoder_kv_groups(dec):
    """Flat-store groups of a decoder: each layer's own, plus ALL layers' source-attention
    linear_k / linear_v weights (and biases) back to back -- one [n_layer * 2d, d] matrix, so
    the memory's keys/values of every layer are ONE GEMM over the encoder output (the memory
    is the same for all layers) and their input gradients one K = n_layer * 2d GEMM
    (nets/functional.py decoder_layers_fwd / _bwd).  Each layer's [2d, d] block stays a
    contiguous view."""
    gs = []
    for layer in dec.dec_layers:
        gs += layer.flat_groups(kv=False)
    pf = [layer._pfx + ".src_attn." for layer in dec.dec_layers]
    return gs + [[p + n for p in pf for n in KV_W], [p + n for p in pf for n in KV_B]]


def decoder_kv_all(dec, grad):
    """The cross-layer source-attention key/value matrix and bias (decoder_kv_groups)."""
    pf = ["dec_layers.%d.src_attn." % i for i in range(len(dec.dec_layers))]
    wn = [p + n for p in pf for n in KV_W]
    bn = [p + n for p in pf for n in KV_B]
    if grad:
        return SimpleNamespace(W=dec._gg(wn, dec.h_dim), b=dec._gg(bn))
    return SimpleNamespace(W=dec._wg(wn, dec.h_dim), b=dec._pg(bn))


class TransformerDecoder(_Bound):
    """liteasr/nets/transformer_decoder.py:13-93."""

    def __init__(self, i_dim, h_dim, ff_dim, n_head, n_layer, dropout_rate, pos_dropout_rate,
                 self_attn_dropout_rate, src_attn_dropout_rate, ff_dropout_rate, arch):
        super().__init__()
        self.embed = nn.Embedding(i_dim, h_dim)
        self.pe = PositionalEncoding(h_dim, dropout_rate=pos_dropout_rate)
        self.dec_layers = nn.ModuleList([
            DecoderLayer(
                size=h_dim,
                self_attn=MultiHeadAttention(n_head=n_head, i_dim=h_dim, dropout_rate=self_attn_dropout_rate),
                src_attn=MultiHeadAttention(n_head=n_head, i_dim=h_dim, dropout_rate=src_attn_dropout_rate),
                feed_forward=PositionwiseFeedForward(i_dim=h_dim, h_units=ff_dim, dropout_rate=ff_dropout_rate),
                dropout_rate=dropout_rate,
            ) for _ in range(n_layer)
        ])
        self.after_norm = LayerNorm(h_dim)
        self.linear_out = nn.Linear(h_dim, i_dim)
        self.h_dim, self.n_head = h_dim, n_head
        self.rates = SimpleNamespace(drop=dropout_rate, pos=pos_dropout_rate, self_att=self_attn_dropout_rate,
                                     src_att=src_attn_dropout_rate, ff=ff_dropout_rate)

    def weights(self):
        return self._cached("w", self._weights)

    def grads(self):
        return self._cached("g", self._grads)

    def flat_groups(self):
        return decoder_kv_groups(self)

    def _weights(self):
        return SimpleNamespace(d=self.h_dim, H=self.n_head, E=self._p("embed.weight"),
                               pe=self.pe.table(1), layers=[l._w_all(False) for l in self.dec_layers],
                               ln_f=SimpleNamespace(g=self._p("after_norm.weight"), b=self._p("after_norm.bias")),
                               Wout=self._w("linear_out.weight"), bout=self._p("linear_out.bias"),
                               kv_all=decoder_kv_all(self, False))

    def _grads(self):
        return SimpleNamespace(E=self._g("embed.weight"), layers=[l._w_all(True) for l in self.dec_layers],
                               ln_f=SimpleNamespace(g=self._g("after_norm.weight"), b=self._g("after_norm.bias")),
                               Wout=self._g("linear_out.weight"), bout=self._g("linear_out.bias"),
                               kv_all=decoder_kv_all(self, True))


class CTC(_Bound):
    """liteasr/nets/ctc.py:7-30 (input dropout is always on, :29)."""

    def __init__(self, i_dim, o_dim, dropout_rate):
        super().__init__()
        self.ctc_lo = nn.Linear(i_dim, o_dim)
        self.dropout_rate = dropout_rate

    def weights(self):
        return self._cached("w", lambda: SimpleNamespace(W=self._w("ctc_lo.weight"), b=self._p("ctc_lo.bias")))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(W=self._g("ctc_lo.weight"), b=self._g("ctc_lo.bias")))


class ParallelDecoder(_Bound):
    """liteasr/nets/paraformer/parallel_decoder.py:10-66: the Transformer decoder layers
    without embedding / positional encoding (the input is the CIF output mixed with target
    embeddings) and without a self-attention mask."""

    def __init__(self, i_dim, h_dim, ff_dim, n_head, n_layer, dropout_rate, self_attn_dropout_rate,
                 src_attn_dropout_rate, ff_dropout_rate):
        super().__init__()
        self.dec_layers = nn.ModuleList([
            DecoderLayer(
                size=h_dim,
                self_attn=MultiHeadAttention(n_head=n_head, i_dim=h_dim, dropout_rate=self_attn_dropout_rate),
                src_attn=MultiHeadAttention(n_head=n_head, i_dim=h_dim, dropout_rate=src_attn_dropout_rate),
                feed_forward=PositionwiseFeedForward(i_dim=h_dim, h_units=ff_dim, dropout_rate=ff_dropout_rate),
                dropout_rate=dropout_rate,
            ) for _ in range(n_layer)
        ])
        self.after_norm = LayerNorm(h_dim)
        self.linear_out = nn.Linear(h_dim, i_dim)
        self.h_dim, self.n_head = h_dim, n_head
        self.rates = SimpleNamespace(drop=dropout_rate, self_att=self_attn_dropout_rate, src_att=src_attn_dropout_rate,
                                     ff=ff_dropout_rate)

    def flat_groups(self):
        return decoder_kv_groups(self)

    def weights(self):
        return self._cached("w", lambda: SimpleNamespace(
            d=self.h_dim, H=self.n_head, layers=[l._w_all(False) for l in self.dec_layers],
            ln_f=SimpleNamespace(g=self._p("after_norm.weight"), b=self._p("after_norm.bias")),
            Wout=self._w("linear_out.weight"), bout=self._p("linear_out.bias"), kv_all=decoder_kv_all(self, False)))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(
            layers=[l._w_all(True) for l in self.dec_layers],
            ln_f=SimpleNamespace(g=self._g("after_norm.weight"), b=self._g("after_norm.bias")),
            Wout=self._g("linear_out.weight"), bout=self._g("linear_out.bias"), kv_all=decoder_kv_all(self, True)))


class Predictor(_Bound):
    """liteasr/nets/paraformer/predictor.py:12-22: Conv1d(d, d, 3, padding 1) -> ReLU ->
    Linear(d, 1) -> Sigmoid, then the CIF scan (csrc/cif.hip)."""

    def __init__(self, size):
        super().__init__()
        self.conv = nn.Conv1d(in_channels=size, out_channels=size, kernel_size=3, padding=1)
        self.relu = nn.ReLU()
        self.lin = nn.Linear(size, 1)
        self.sigmoid = nn.Sigmoid()
        self.size = size

    def weights(self):
        return SimpleNamespace(Wc=self._p("conv.weight"), bc=self._p("conv.bias"), Wl=self._w("lin.weight"),
                               bl=self._p("lin.bias"))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(Wc=self._g("conv.weight"), bc=self._g("conv.bias"),
                                                         Wl=self._g("lin.weight"), bl=self._g("lin.bias")))



class LSTMCell(nn.LSTMCell):
    """torch.nn.LSTMCell parameter container (weight_ih, weight_hh, bias_ih, bias_hh; gate
    order i, f, g, o) of liteasr/nets/rnn_decoder.py:21-24; the arithmetic runs in
    csrc/rnnt.hip (lstm_cell_fwd / bwd) around the host's recurrent GEMMs."""

    seed = 0

    def flat_groups(self):
        return []


class RNNDecoder(_Bound):
    """liteasr/nets/rnn_decoder.py:10-80 (the Transducer's prediction network): Embedding
    (padding_idx 0) -> dropout -> n_layer LSTMCells, dropout after each cell's output."""

    def __init__(self, i_dim, h_dim, h_units, n_layer, dropout_rate):
        super().__init__()
        self.embed = nn.Embedding(i_dim, h_dim, padding_idx=0)
        self.dropout_embed = nn.Dropout(dropout_rate)
        self.dec_layers = nn.ModuleList([LSTMCell(h_dim, h_units)] +
                                        [LSTMCell(h_units, h_units) for _ in range(1, n_layer)])
        self.dropout_dec = nn.ModuleList([nn.Dropout(dropout_rate) for _ in range(n_layer)])
        self.h_dim, self.h_units, self.n_layer = h_dim, h_units, n_layer
        self.rates = SimpleNamespace(drop=dropout_rate, pos=0.0, self_att=0.0, src_att=0.0, ff=0.0)

    def weights(self):
        return self._cached("w", lambda: SimpleNamespace(
            E=self._p("embed.weight"),
            layers=[SimpleNamespace(Wih=self._w(f"dec_layers.{i}.weight_ih"), Whh=self._w(f"dec_layers.{i}.weight_hh"),
                                    bih=self._p(f"dec_layers.{i}.bias_ih"), bhh=self._p(f"dec_layers.{i}.bias_hh"))
                    for i in range(self.n_layer)]))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(
            E=self._g("embed.weight"),
            layers=[SimpleNamespace(Wih=self._g(f"dec_layers.{i}.weight_ih"), Whh=self._g(f"dec_layers.{i}.weight_hh"),
                                    bih=self._g(f"dec_layers.{i}.bias_ih"), bhh=self._g(f"dec_layers.{i}.bias_hh"))
                    for i in range(self.n_layer)]))


class Joint(_Bound):
    """Transducer.joint's projections (liteasr/models/transducer.py:91-95,199-203) as one
    bound view bundle over the top-level lin_enc / lin_dec / lin_jnt parameters."""

    def __init__(self, owner):
        super().__init__()
        object.__setattr__(self, "_owner", owner)  # not a submodule: keys stay top-level

    def weights(self):
        return self._cached("w", lambda: SimpleNamespace(
            We=self._w("lin_enc.weight"), be=self._p("lin_enc.bias"), Wd=self._w("lin_dec.weight"),
            Wj=self._w("lin_jnt.weight"), bj=self._p("lin_jnt.bias")))

    def grads(self):
        return self._cached("g", lambda: SimpleNamespace(
            We=self._g("lin_enc.weight"), be=self._g("lin_enc.bias"), Wd=self._g("lin_dec.weight"),
            Wj=self._g("lin_jnt.weight"), bj=self._g("lin_jnt.bias")))
