"""CPU oracle for the U2 / Conformer + hybrid CTC-attention training step.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / CPU baseline --
never as the thing measured or shipped.  The product path (liteasr_amd/) never
imports it.

This is a from-scratch, functional restatement (plain PyTorch on the CPU, fp32 or
fp64) of the reference's arithmetic on the hot path.  Each function names the
reference file:line it follows (paths relative to /root/reference).  Parameters are
a flat ``{state_dict_key: tensor}`` mapping using the reference's key names, so the
oracle, the reference and liteasr_amd can all be fed the same weights.

Parity pin: tests/test_oracle_golden.py checks this module against golden vectors
produced by importing the reference itself in the build container
(tests/golden/make_golden.py).
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


# ------------------------------------------------------------------ bookkeeping
def padding_mask(lengths: torch.Tensor, width: Optional[int] = None) -> torch.Tensor:
    """True = padding.  liteasr/utils/mask.py:8-27 (width = max(lengths))."""
    w = int(lengths.max()) if width is None else width
    return torch.arange(w)[None, :] >= lengths[:, None]


def triangle_mask(rows: int, cols: int = 0, stage: int = 1, diagonal: int = 1) -> torch.Tensor:
    """liteasr/utils/mask.py:30-90: mask[r, c] = c//stage > r//stage + diagonal - 1."""
    cols = rows if cols == 0 else cols
    r = torch.arange(rows)[:, None] // stage
    c = torch.arange(cols)[None, :] // stage
    return c > r + (diagonal - 1)


def subsampled_len(T: int) -> int:
    """Length after the two 3x3/stride-2 convs: liteasr/nets/subsampling.py:31-36."""
    return ((T - 1) // 2 - 1) // 2


def pred_len(xlens: torch.Tensor) -> torch.Tensor:
    """liteasr/models/u2.py:319-321 (Python floor division)."""
    return torch.div(torch.div(xlens - 1, 2, rounding_mode="floor") - 1, 2, rounding_mode="floor")


def encoder_key_mask(xlens: torch.Tensor, Tmax: int) -> torch.Tensor:
    """(B, T') padding after the "convolution simulation" slicing
    liteasr/nets/transformer_encoder.py:117-120: frame t' is padding iff 4t' >= xlen."""
    m = padding_mask(xlens, Tmax)
    return m[:, :-2:2][:, :-2:2]


def decoder_io(ys: torch.Tensor, ylens: torch.Tensor, sos: int, eos: int, ignore: int = -1):
    """ys_in / decoder self-attention mask / attention targets.
    liteasr/models/u2.py:146-148 (mask), :323-333 (get_target), :339-358 (_preprocess)."""
    B, L = ys.shape
    ys_in = torch.cat([torch.full((B, 1), sos, dtype=ys.dtype), ys.masked_fill(ys == ignore, eos)], 1)
    ys_mask = padding_mask(ylens + 1, L + 1)
    dec_mask = ys_mask[:, None, :] | triangle_mask(L + 1)[None]
    tgt = torch.cat([ys, torch.full((B, 1), ignore, dtype=ys.dtype)], 1)
    tgt[torch.arange(B), ylens] = eos
    return ys_in, dec_mask, tgt


# ----------------------------------------------------------------------- blocks
def layer_norm(x, p: Params, name: str, eps: float = 1e-12):
    """liteasr/nets/layer_norm.py:8-21."""
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


def linear(x, p: Params, name: str, bias: bool = True):
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias") if bias else None)


def sinusoid_table(T: int, d: int, dtype=torch.float32) -> torch.Tensor:
    """pe[t, 2i] = sin(t / 10000^(2i/d)), pe[t, 2i+1] = cos(...)
    (liteasr/nets/positional_encoding.py:29-38, computed in fp32 as the reference)."""
    pos = torch.arange(T, dtype=torch.float32)[:, None]
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe = torch.zeros(T, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.to(dtype)


def subsample(x, p: Params, name: str):
    """Conv2DLayer: liteasr/nets/subsampling.py:42-48 (c-major flatten: index = c*F' + f)."""
    y = F.relu(F.conv2d(x.unsqueeze(1), p[name + ".conv.0.weight"], p[name + ".conv.0.bias"], stride=2))
    y = F.relu(F.conv2d(y, p[name + ".conv.2.weight"], p[name + ".conv.2.bias"], stride=2))
    B, C, T, Fp = y.shape
    return linear(y.transpose(1, 2).reshape(B, T, C * Fp), p, name + ".out")


def rel_shift(bd: torch.Tensor) -> torch.Tensor:
    """Legacy relative shift (liteasr/nets/attention.py:99-118), closed form:
    out[i, j] = bd[i, T-1-i+j] (j <= i); 0 (j == i+1); bd[i+1, j-i-2] (j > i+1)."""
    T = bd.shape[-1]
    i = torch.arange(T)[:, None]
    j = torch.arange(T)[None, :]
    k = (i + 1) * T + j
    r, c = k // (T + 1), k % (T + 1)
    g = bd[..., r.clamp(max=T - 1), (c - 1).clamp(min=0)]
    return torch.where(c == 0, torch.zeros((), dtype=bd.dtype), g)


def attention(q, k, v, mask, p: Params, name: str, H: int, pos=None, drop=0.0, training=True):
    """Multi-head attention.  Plain: liteasr/nets/attention.py:61-71; relative (pos given):
    :120-154.  mask (B,1|Tq,Tk) bool, True = masked, filled with -1e38 (:54)."""
    B, Tq, d = q.shape
    dk = d // H
    Q = linear(q, p, name + ".linear_q").view(B, Tq, H, dk)
    Kt = linear(k, p, name + ".linear_k").view(B, -1, H, dk).transpose(1, 2)
    Vt = linear(v, p, name + ".linear_v").view(B, -1, H, dk).transpose(1, 2)
    if pos is None:
        scores = Q.transpose(1, 2) @ Kt.transpose(-1, -2) / math.sqrt(dk)
    else:
        P = F.linear(pos, p[name + ".linear_pos.weight"]).view(1, -1, H, dk).transpose(1, 2)
        qu = (Q + p[name + ".pos_bias_u"]).transpose(1, 2)
        qv = (Q + p[name + ".pos_bias_v"]).transpose(1, 2)
        scores = (qu @ Kt.transpose(-1, -2) + rel_shift(qv @ P.transpose(-1, -2))) / math.sqrt(dk)
    if mask is not None:
        scores = scores.masked_fill(mask.unsqueeze(1), -1e38)
    attn = F.dropout(torch.softmax(scores, -1), drop, training)
    out = (attn @ Vt).transpose(1, 2).reshape(B, Tq, d)
    return linear(out, p, name + ".linear_o")


def ffn(x, p: Params, name: str, act: str, drop=0.0, training=True, gate=None, pre=None):
    """PositionwiseFeedForward: liteasr/nets/feed_forward.py:18-19, Swish swish.py:14-16.
    Test hook (ReLU only): ``gate`` (0/1, the shape of the pre-activation) replaces the branch
    relu takes, h = u * gate -- a parity test feeds the branch the GPU build took so that a
    pre-activation within rounding of 0 takes the same side on both; ``pre`` collects
    (u, bound): bound = K 2^-23 (|x| |W|^T + |b|), the worst-case error of an fp32 K-term dot
    product (plus bias), per element -- how far from 0 an fp32 build may put u on the other side."""
    h = linear(x, p, name + ".fc1")
    if pre is not None:
        w, b = p[name + ".fc1.weight"], p.get(name + ".fc1.bias")
        mag = F.linear(x.detach().abs(), w.detach().abs(), None if b is None else b.detach().abs())
        pre.append((h.detach(), w.shape[1] * 2.0 ** -23 * mag))
    if gate is not None:
        assert act == "relu"
        h = h * gate.to(h.dtype).view_as(h)
    else:
        h = h * torch.sigmoid(h) if act == "swish" else F.relu(h)
    return linear(F.dropout(h, drop, training), p, name + ".fc2")


def conv_module(x, p: Params, name: str, bn_state: Optional[dict], training=True, act: str = "swish"):
    """Convolution: liteasr/nets/conformer_convolution.py:44-57 (BatchNorm1d train mode:
    batch stats over B*T incl. padding; running stats updated, momentum 0.1, eps 1e-5);
    activation Swish or ReLU (transformer_encoder.py:77-80)."""
    y = x.transpose(1, 2)
    y = F.conv1d(y, p[name + ".pointwise_conv1.weight"], p[name + ".pointwise_conv1.bias"])
    y = F.glu(y, dim=1)
    Kk = p[name + ".depthwise_conv.weight"].shape[-1]
    y = F.conv1d(y, p[name + ".depthwise_conv.weight"], p[name + ".depthwise_conv.bias"],
                 padding=(Kk - 1) // 2, groups=y.shape[1])
    rm = bn_state[name + ".norm.running_mean"] if bn_state is not None else None
    rv = bn_state[name + ".norm.running_var"] if bn_state is not None else None
    y = F.batch_norm(y, rm, rv, p[name + ".norm.weight"], p[name + ".norm.bias"], training, 0.1, 1e-5)
    if bn_state is not None and training:
        bn_state[name + ".norm.num_batches_tracked"] += 1
    y = y * torch.sigmoid(y) if act == "swish" else F.relu(y)
    y = F.conv1d(y, p[name + ".pointwise_conv2.weight"], p[name + ".pointwise_conv2.bias"])
    return y.transpose(1, 2)


def conformer_layer(x, pos, mask, p: Params, name: str, H: int, cfg, bn_state, training=True):
    """Conformer layer (pre-norm, macaron 0.5 scale): RelativeEncoderLayer
    liteasr/nets/conformer_layer.py:130-147 (pos given) or EncoderLayer :68-81 (use_rel
    False: plain attention); FFN and conv-module activation cfg["activation"]."""
    dr, ff_dr, at_dr = cfg["dropout"], cfg["ff_dropout"], cfg["attn_dropout"]
    act = cfg.get("activation", "swish")
    h = layer_norm(x, p, name + ".feed_forward_macaron_norm")
    x = x + 0.5 * F.dropout(ffn(h, p, name + ".feed_forward_macaron", act, ff_dr, training), dr, training)
    h = layer_norm(x, p, name + ".self_attn_norm")
    x = x + F.dropout(attention(h, h, h, mask, p, name + ".self_attn", H, pos, at_dr, training), dr, training)
    h = layer_norm(x, p, name + ".conv_norm")
    x = x + F.dropout(conv_module(h, p, name + ".conv", bn_state, training, act), dr, training)
    h = layer_norm(x, p, name + ".feed_forward_norm")
    x = x + 0.5 * F.dropout(ffn(h, p, name + ".feed_forward", act, ff_dr, training), dr, training)
    return layer_norm(x, p, name + ".final_norm")


def transformer_layer(x, pos, mask, p: Params, name: str, H: int, cfg, training=True):
    """Transformer encoder layer (enc_arch "transformer", pre-norm): EncoderLayer
    liteasr/nets/transformer_layer.py:27-76 / RelativeEncoderLayer :79-136; the FFN keeps its
    default ReLU (feed_forward.py:11, transformer_encoder.py:58-62)."""
    dr, ff_dr, at_dr = cfg["dropout"], cfg["ff_dropout"], cfg["attn_dropout"]
    h = layer_norm(x, p, name + ".self_attn_norm")
    x = x + F.dropout(attention(h, h, h, mask, p, name + ".self_attn", H, pos, at_dr, training), dr, training)
    h = layer_norm(x, p, name + ".feed_forward_norm")
    return x + F.dropout(ffn(h, p, name + ".feed_forward", "relu", ff_dr, training), dr, training)


def encoder(xs, xlens, p: Params, cfg, bn_state=None, training=True, chunk: int = 0):
    """TransformerEncoder: liteasr/nets/transformer_encoder.py:107-127 -- conformer or
    transformer layers (cfg enc_arch), relative PE (use_rel: x * sqrt(d), the table feeds the
    attention, positional_encoding.py:68-75) or absolute PE (x * sqrt(d) + pe, :49-56).
    chunk > 0 adds the chunk mask triangle_mask(T', stage=chunk) (config 4 oracle-by-composition)."""
    d = cfg["enc_dim"]
    x = subsample(xs, p, "encoder.embed")
    B, T, _ = x.shape
    pe = sinusoid_table(T, d, x.dtype)
    if cfg.get("use_rel", True):
        x = F.dropout(x * math.sqrt(d), cfg["pos_dropout"], training)
        pos = F.dropout(pe.unsqueeze(0), cfg["pos_dropout"], training)
    else:
        x = F.dropout(x * math.sqrt(d) + pe.unsqueeze(0), cfg["pos_dropout"], training)
        pos = None
    kmask = encoder_key_mask(xlens, xs.shape[1])  # (B, T')
    mask = kmask[:, None, :]
    if chunk > 0:
        mask = mask | triangle_mask(T, stage=chunk)[None]
    for i in range(cfg["enc_layers"]):
        if cfg.get("enc_arch", "conformer") == "transformer":
            x = transformer_layer(x, pos, mask, p, f"encoder.enc_layers.{i}", cfg["enc_heads"], cfg, training)
        else:
            x = conformer_layer(x, pos, mask, p, f"encoder.enc_layers.{i}", cfg["enc_heads"], cfg, bn_state,
                                training)
    return layer_norm(x, p, "encoder.after_norm"), kmask


def decoder(ys_in, dec_mask, memory, mem_mask, p: Params, cfg, training=True, gates=None, pre=None):
    """TransformerDecoder: liteasr/nets/transformer_decoder.py:70-93, DecoderLayer
    liteasr/nets/transformer_layer.py:179-221 (pre-norm, ReLU FFN).  ``gates`` / ``pre``: the
    per-layer ReLU test hook of ``ffn``."""
    d = cfg["dec_dim"]
    H = cfg["dec_heads"]
    dr = cfg["dec_dropout"]
    y = F.embedding(ys_in, p["decoder.embed.weight"])
    y = F.dropout(y * math.sqrt(d) + sinusoid_table(y.shape[1], d, y.dtype)[None], cfg["dec_pos_dropout"], training)
    mm = mem_mask[:, None, :]
    for i in range(cfg["dec_layers"]):
        n = f"decoder.dec_layers.{i}"
        h = layer_norm(y, p, n + ".self_attn_norm")
        y = y + F.dropout(attention(h, h, h, dec_mask, p, n + ".self_attn", H, None, 0.0, training), dr, training)
        h = layer_norm(y, p, n + ".src_attn_norm")
        y = y + F.dropout(attention(h, memory, memory, mm, p, n + ".src_attn", H, None, 0.0, training), dr, training)
        h = layer_norm(y, p, n + ".feed_forward_norm")
        y = y + F.dropout(ffn(h, p, n + ".feed_forward", "relu", cfg["dec_ff_dropout"], training,
                              gate=None if gates is None else gates[i], pre=pre), dr, training)
    y = layer_norm(y, p, "decoder.after_norm")
    return linear(y, p, "decoder.linear_out")


def u2_forward(xs, xlens, ys, ylens, p: Params, cfg, bn_state=None, training=True, chunk=0, dec_gates=None,
               dec_pre=None):
    """U2.forward: liteasr/models/u2.py:116-159.  Returns (h_attn, h_ctc, h_enc, tgt).
    ``dec_gates`` / ``dec_pre``: the decoder's ReLU test hook (``ffn``)."""
    V = cfg["vocab_size"]
    sos = eos = V - 1
    h_enc, kmask = encoder(xs, xlens, p, cfg, bn_state, training, chunk)
    ys_in, dec_mask, tgt = decoder_io(ys, ylens, sos, eos)
    h_attn = decoder(ys_in, dec_mask, h_enc, kmask, p, cfg, training, dec_gates, dec_pre)
    h_ctc = linear(F.dropout(h_enc, cfg["dropout"], True), p, "ctc.ctc_lo")  # always on (ctc.py:29)
    return h_attn, h_ctc, h_enc, tgt


def hybrid_loss(h_attn, h_ctc, tgt, ys, xlens, ylens, ctc_weight: float, smoothing: float,
                ignore: int = -1):
    """HybridCTCLoss.__call__: liteasr/criterions/hybrid_ctc_attn.py:39-79."""
    B = ys.shape[0]
    V = h_attn.shape[-1]
    t = tgt.reshape(-1)
    ign = t == ignore
    logp = torch.log_softmax(h_attn.reshape(-1, V), 1)
    td = torch.full_like(logp, smoothing / (V - 1))
    td.scatter_(1, t.masked_fill(ign, 0).unsqueeze(1), 1.0 - smoothing)
    kl = F.kl_div(logp, td, reduction="none").masked_fill(ign.unsqueeze(1), 0)
    loss_att = kl.sum() / B
    lp = h_ctc.transpose(0, 1).log_softmax(-1)
    loss_ctc = F.ctc_loss(lp, ys, pred_len(xlens), ylens, blank=0, reduction="sum") / B
    loss = ctc_weight * loss_ctc + (1 - ctc_weight) * loss_att
    return loss, loss_ctc, loss_att


# ------------------------------------------------------------------- train step
def noam_lr(step: int, model_dim: int, factor: float = 1.0, warmup: int = 25000) -> float:
    """liteasr/optims/noam.py:41-46."""
    return factor * model_dim ** (-0.5) * min(step ** (-0.5), step * warmup ** (-1.5))


def train_step(params: Params, buffers: dict, batch, cfg, ctc_weight=0.3, smoothing=0.1,
               clip=5.0, opt_state=None, model_dim=None, chunk=0, training=True, dec_gates=None, dec_pre=None):
    """One reference training iteration (accum_grad=1): liteasr/trainer.py:147-171 with
    torch.optim.Adam(betas=(0.9, 0.98), eps=1e-9) under Noam (noam.py:33-39).
    training=False runs the forward in eval mode (BN running statistics, no dropout but
    the CTC head's always-on one) and still differentiates it.
    Returns (loss, grads, new_params, opt_state, grad_norm)."""
    xs, xlens, ys, ylens = batch
    names = [k for k in params if params[k].is_floating_point()]
    leaf = {k: params[k].detach().clone().requires_grad_() for k in names}
    h_attn, h_ctc, _, tgt = u2_forward(xs, xlens, ys, ylens, leaf, cfg, buffers, training, chunk, dec_gates, dec_pre)
    loss, lc, la = hybrid_loss(h_attn, h_ctc, tgt, ys, xlens, ylens, ctc_weight, smoothing)
    loss.backward()
    grads = {k: (leaf[k].grad if leaf[k].grad is not None else torch.zeros_like(leaf[k])) for k in names}
    gl = [grads[k] for k in names]
    norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in gl]))
    coef = min(clip / (float(norm) + 1e-6), 1.0)
    st = opt_state or {"step": 0, "m": {}, "v": {}}
    new = dict(params)
    if not math.isnan(float(norm)):
        st["step"] += 1
        s = st["step"]
        lr = noam_lr(s, model_dim or cfg["enc_dim"])
        b1, b2, eps = 0.9, 0.98, 1e-9
        for k in names:
            g = grads[k] * coef
            m = st["m"].get(k, torch.zeros_like(g)).lerp(g, 1 - b1)
            v = st["v"].get(k, torch.zeros_like(g)) * b2 + (1 - b2) * g * g
            st["m"][k], st["v"][k] = m, v
            denom = v.sqrt() / math.sqrt(1 - b2 ** s) + eps
            new[k] = params[k] - (lr / (1 - b1 ** s)) * m / denom
    return loss.detach(), grads, new, st, float(norm)


def default_cfg(**kw):
    cfg = dict(enc_dim=256, enc_heads=4, enc_ff=2048, enc_layers=12, dec_dim=256, dec_heads=4,
               dec_ff=2048, dec_layers=6, vocab_size=4233, input_dim=80, dropout=0.0,
               ff_dropout=0.0, attn_dropout=0.0, pos_dropout=0.0, dec_dropout=0.0,
               dec_pos_dropout=0.0, dec_ff_dropout=0.0)
    cfg.update(kw)
    return cfg


def init_params(cfg, seed: int = 42, dtype=torch.float32) -> Params:
    """Random weights with the reference's state_dict key names and shapes (U2 of
    liteasr/models/u2.py:72-114).  Scales keep activations O(1) for parity tests."""
    g = torch.Generator().manual_seed(seed)
    d, ff, V, Fin = cfg["enc_dim"], cfg["enc_ff"], cfg["vocab_size"], cfg["input_dim"]
    H = cfg["enc_heads"]
    p: Params = {}

    def lin(name, o, i, bias=True):
        p[name + ".weight"] = torch.randn(o, i, generator=g) / math.sqrt(i)
        if bias:
            p[name + ".bias"] = torch.randn(o, generator=g) * 0.02

    def ln(name, n):
        p[name + ".weight"] = 1 + 0.1 * torch.randn(n, generator=g)
        p[name + ".bias"] = 0.1 * torch.randn(n, generator=g)

    f1 = (Fin - 3) // 2 + 1
    f2 = (f1 - 3) // 2 + 1
    p["encoder.embed.conv.0.weight"] = torch.randn(d, 1, 3, 3, generator=g) / 3
    p["encoder.embed.conv.0.bias"] = torch.randn(d, generator=g) * 0.02
    p["encoder.embed.conv.2.weight"] = torch.randn(d, d, 3, 3, generator=g) / math.sqrt(9 * d)
    p["encoder.embed.conv.2.bias"] = torch.randn(d, generator=g) * 0.02
    lin("encoder.embed.out", d, d * f2)
    rel = cfg.get("use_rel", True)
    tfm = cfg.get("enc_arch", "conformer") == "transformer"
    for i in range(cfg["enc_layers"]):
        n = f"encoder.enc_layers.{i}"
        if rel:
            p[n + ".self_attn.pos_bias_u"] = torch.randn(H, d // H, generator=g) * 0.1
            p[n + ".self_attn.pos_bias_v"] = torch.randn(H, d // H, generator=g) * 0.1
        for q in ("q", "k", "v", "o"):
            lin(f"{n}.self_attn.linear_{q}", d, d)
        if rel:
            lin(n + ".self_attn.linear_pos", d, d, bias=False)
        if tfm:  # transformer layer: attention, one FFN, two norms
            lin(n + ".feed_forward.fc1", ff, d)
            lin(n + ".feed_forward.fc2", d, ff)
            ln(n + ".self_attn_norm", d)
            ln(n + ".feed_forward_norm", d)
            continue
        for f in ("feed_forward", "feed_forward_macaron"):
            lin(f"{n}.{f}.fc1", ff, d)
            lin(f"{n}.{f}.fc2", d, ff)
        for nn_ in ("self_attn_norm", "feed_forward_norm", "feed_forward_macaron_norm", "conv_norm", "final_norm"):
            ln(f"{n}.{nn_}", d)
        c = n + ".conv"
        p[c + ".pointwise_conv1.weight"] = torch.randn(2 * d, d, 1, generator=g) / math.sqrt(d)
        p[c + ".pointwise_conv1.bias"] = torch.randn(2 * d, generator=g) * 0.02
        p[c + ".depthwise_conv.weight"] = torch.randn(d, 1, 15, generator=g) / math.sqrt(15)
        p[c + ".depthwise_conv.bias"] = torch.randn(d, generator=g) * 0.02
        p[c + ".pointwise_conv2.weight"] = torch.randn(d, d, 1, generator=g) / math.sqrt(d)
        p[c + ".pointwise_conv2.bias"] = torch.randn(d, generator=g) * 0.02
        ln(c + ".norm", d)
    ln("encoder.after_norm", d)
    dd, dff = cfg["dec_dim"], cfg["dec_ff"]
    p["decoder.embed.weight"] = torch.randn(V, dd, generator=g)
    for i in range(cfg["dec_layers"]):
        n = f"decoder.dec_layers.{i}"
        for a in ("self_attn", "src_attn"):
            for q in ("q", "k", "v", "o"):
                lin(f"{n}.{a}.linear_{q}", dd, dd)
        lin(n + ".feed_forward.fc1", dff, dd)
        lin(n + ".feed_forward.fc2", dd, dff)
        for nn_ in ("self_attn_norm", "feed_forward_norm", "src_attn_norm"):
            ln(f"{n}.{nn_}", dd)
    ln("decoder.after_norm", dd)
    lin("decoder.linear_out", V, dd)
    lin("ctc.ctc_lo", V, d)
    return {k: v.to(dtype) for k, v in p.items()}


def init_buffers(cfg) -> dict:
    b = {}
    if cfg.get("enc_arch", "conformer") == "transformer":
        return b  # no convolution module, no BatchNorm
    for i in range(cfg["enc_layers"]):
        n = f"encoder.enc_layers.{i}.conv.norm"
        b[n + ".running_mean"] = torch.zeros(cfg["enc_dim"])
        b[n + ".running_var"] = torch.ones(cfg["enc_dim"])
        b[n + ".num_batches_tracked"] = torch.zeros((), dtype=torch.long)
    return b


def synthetic_batch(B: int, T: int, L: int, V: int, F_: int = 80, seed: int = 0):
    """SURVEY.md §8(d) synthetic inputs: xs ~ N(0,1) zeroed past xlen, xlens ~ U[0.95T, T]
    with xlens[0] = T, ys ~ U{1..V-2} padded with -1, ylens ~ U[L/2, L] with ylens[0] = L."""
    g = torch.Generator().manual_seed(seed)
    xlens = torch.randint(int(0.95 * T), T + 1, (B,), generator=g)
    xlens[0] = T
    xs = torch.randn(B, T, F_, generator=g)
    xs = xs.masked_fill(padding_mask(xlens, T).unsqueeze(-1), 0.0)
    ylens = torch.randint(max(1, L // 2), L + 1, (B,), generator=g)
    ylens[0] = L
    ys = torch.randint(1, V - 1, (B, L), generator=g)
    ys = ys.masked_fill(padding_mask(ylens, L), -1)
    return xs, xlens, ys, ylens
