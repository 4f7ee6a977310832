"""bf16-emulating CPU oracle of the U2 training step (forward + backward).

TEST INFRASTRUCTURE ONLY.  Only tests/ may import this module, as the checker -- never
as the thing measured or shipped.  The product path (liteasr_amd/) never imports it.

The reference runs fp32 end to end; liteasr_amd's default build stores GEMM
operands, saved activations and gradient hand-offs in bf16 and keeps the residual stream,
LayerNorm / BatchNorm / softmax statistics and every accumulation in fp32.  Held against
the fp64 oracle (u2_oracle.py), that build differs by the sum of all its bf16 roundings,
which bounds a parity test at a few 1e-2.  This module is the same arithmetic as
u2_oracle.py (same reference file:line citations, same state_dict keys, same masks and
bookkeeping), evaluated in float64 with bf16 rounding inserted exactly where the HIP path
rounds, so that a kernel bug shows up far above the remaining difference (fp32 vs fp64
accumulation and the rare element whose fp32 value straddles a bf16 rounding boundary):

  R(x)  forward rounds to bf16 (a bf16 tensor in HBM), backward passes the gradient as is;
  G(x)  forward identity, backward rounds the incoming gradient to bf16 (a bf16 gradient
        tensor handed to the next kernel);
  ActGate  Swish / ReLU whose backward multiplies by the STORED bf16 gate act'(u) and
        rounds the product (nets/functional.py ffn_forward / ffn_backward);
  FlashAttn  the fused attention kernels (csrc/attn_flash.hip): 64-key blocks with the
        online softmax, P rounded to bf16 before P.V, ctx rounded; backward recomputes P
        from the forward's row statistics, D = rowsum(dctx * ctx) on the rounded tensors,
        dS rounded before the dQ / dK / dBD products, P rounded before dV.

Where each rounding sits (HIP path, liteasr_amd/nets/functional.py):
  subsampling   y1 = R(relu(conv1)), y2 = R(relu(conv2)), both with G (their data
                gradients are bf16); out linear fp32; gradient of it bf16
  layer norms   bf16 outputs with G (dln of the consuming GEMM is bf16); the final
                LayerNorm of a Conformer layer stays fp32 (residual stream)
  projections   qkv / q / kv / z1 (pw1) / pos-projection R + G; u/v biases R(q + bias)
  residual      out = res + scale * G(branch)   (gb = bf16(scale * dres))
  conv module   y = R(dwconv(GLU(z1))) (BN statistics on the stored value),
                h3 = R(swish(BN(y))) + G, BN / DW gradients fp32
  heads         encoder after_norm R (its gradient accumulates in fp32); logits R + G
This file is checked against the fp64 oracle on the reference goldens
(tests/test_oracle_golden.py::test_bf16_oracle_tracks_fp64) and is the tight bar for the
bf16 build (tests/test_model_gpu.py::test_parity_bf16_emulated*).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import u2_oracle as O


def bf16(x: torch.Tensor) -> torch.Tensor:
    """Round to the nearest bf16 (round-to-nearest-even, as the kernels' f2bf), keep dtype."""
    return x.to(torch.float32).to(torch.bfloat16).to(x.dtype)


class _R(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return bf16(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _G(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return bf16(g)


def R(x):
    return _R.apply(x)


def G(x):
    return _G.apply(x)


def RG(x):
    return G(R(x))


class ActGate(torch.autograd.Function):
    """h = act(u) (rounded by the caller); du = bf16(dh * bf16(act'(u))) -- the fc1 epilogue
    stores the gate act'(u) * keep in bf16 and the dz GEMM multiplies by it (dropout 0).
    `gate` (optional): use this stored gate instead of act'(u) -- a test feeds the kernel's
    own ReLU gate so that a pre-activation within accumulation error of zero (a kink the
    two sides may resolve differently) cannot decide a gradient comparison."""

    @staticmethod
    def forward(ctx, u, act, gate=None):
        ctx.save_for_backward(u)
        ctx.act, ctx.gate = act, gate
        if act == "swish":
            return u * torch.sigmoid(u)
        return F.relu(u)

    @staticmethod
    def backward(ctx, dh):
        (u,) = ctx.saved_tensors
        if ctx.gate is not None:
            gate = ctx.gate.to(u.dtype).view_as(u)
        elif ctx.act == "swish":
            s = torch.sigmoid(u)
            gate = s * (1 + u * (1 - s))
        else:
            gate = (u > 0).to(u.dtype)
        return bf16(dh * bf16(gate)), None, None


def _relshift_index(T):
    """(rows, cols) into bd for every (i, j) of rel_shift's output, and the j == i+1 zeros
    (u2_oracle.rel_shift closed form, liteasr/nets/attention.py:99-118)."""
    i = torch.arange(T)[:, None]
    j = torch.arange(T)[None, :]
    k = (i + 1) * T + j
    r, c = k // (T + 1), k % (T + 1)
    return r.clamp(max=T - 1), (c - 1).clamp(min=0), c == 0


class FlashAttn(torch.autograd.Function):
    """Scaled dot-product attention as csrc/attn_flash.hip computes it (relative-position
    term when p is given: liteasr/nets/attention.py:120-154; plain: :61-71).
    qu, qv (B,H,T,dk), k, v (B,H,Tk,dk), p (H,T,dk) or None, mask bool (B,1|T,Tk) True =
    masked (-1e38, attention.py:54).  Returns ctx (B,H,T,dk), bf16-rounded."""

    BLK = 64

    @staticmethod
    def _scores(qu, qv, k, p, mask, scale):
        s = qu @ k.transpose(-1, -2)
        if p is not None:
            T = s.shape[-1]
            bd = qv @ p.transpose(-1, -2).unsqueeze(0)
            r, c, z = _relshift_index(T)
            bd = torch.where(z, torch.zeros((), dtype=bd.dtype), bd[..., r, c])
            s = s + bd
        s = s * scale
        if mask is not None:
            s = s.masked_fill(mask.unsqueeze(1), -1e38)
        return s

    @staticmethod
    def forward(ctx, qu, qv, k, v, p, mask, scale):
        S = FlashAttn._scores(qu, qv, k, p, mask, scale)
        Tk = S.shape[-1]
        m = torch.full(S.shape[:-1], -math.inf, dtype=S.dtype)
        l = torch.zeros(S.shape[:-1], dtype=S.dtype)
        o = torch.zeros(qu.shape[:-1] + (v.shape[-1],), dtype=S.dtype)
        for j0 in range(0, Tk, FlashAttn.BLK):
            sb = S[..., j0:j0 + FlashAttn.BLK]
            mn = torch.maximum(m, sb.amax(-1))
            al = torch.exp(m - mn)
            pb = torch.exp(sb - mn[..., None])
            l = l * al + pb.sum(-1)
            o = o * al[..., None] + bf16(pb) @ v[..., j0:j0 + FlashAttn.BLK, :]
            m = mn
        ctxo = bf16(o / l[..., None])
        ctx.save_for_backward(qu, qv, k, v, p if p is not None else torch.empty(0), ctxo, m, l)
        ctx.mask, ctx.scale, ctx.has_p = mask, scale, p is not None
        return ctxo

    @staticmethod
    def backward(ctx, dctx):
        qu, qv, k, v, p, ctxo, m, l = ctx.saved_tensors
        p = p if ctx.has_p else None
        scale = ctx.scale
        S = FlashAttn._scores(qu, qv, k, p, ctx.mask, scale)
        P = torch.exp(S - m[..., None]) / l[..., None]
        dP = dctx @ v.transpose(-1, -2)
        D = (dctx * ctxo).sum(-1, keepdim=True)
        dS = torch.where(S > -1e38, P * (dP - D), torch.zeros((), dtype=P.dtype))
        dSb = bf16(dS)
        dqu = bf16(scale * dSb @ k)
        dk = bf16(scale * dSb.transpose(-1, -2) @ qu)
        dv = bf16(bf16(P).transpose(-1, -2) @ dctx)
        dqv = dp = None
        if p is not None:
            T = S.shape[-1]
            r, c, z = _relshift_index(T)
            keep = ~z
            dbd = torch.zeros_like(dSb)
            dbd[..., r[keep], c[keep]] = dSb[..., keep]
            dqv = bf16(scale * dbd @ p.unsqueeze(0))
            dp = bf16(scale * (dbd.transpose(-1, -2) @ qv).sum(0))
        return dqu, dqv, dk, dv, dp, None, None


# ---------------------------------------------------------------------- blocks
def layer_norm(x, p, name, eps=1e-12):
    """liteasr/nets/layer_norm.py:8-21 (statistics in full precision)."""
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


def linear(x, p, name, bias=True):
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias") if bias else None)


def subsample(x, p, name):
    """Conv2DLayer (liteasr/nets/subsampling.py:42-48), EmbedFn's storage: y1, y2 bf16."""
    y = RG(F.relu(F.conv2d(x.unsqueeze(1), p[name + ".conv.0.weight"], p[name + ".conv.0.bias"], stride=2)))
    y = RG(F.relu(F.conv2d(y, p[name + ".conv.2.weight"], p[name + ".conv.2.bias"], stride=2)))
    B, C, T, Fp = y.shape
    return linear(y.transpose(1, 2).reshape(B, T, C * Fp), p, name + ".out")


def ffn(x_ln, p, name, act, gate=None, pre=None):
    """PositionwiseFeedForward (liteasr/nets/feed_forward.py:18-19), swish.py:14-16.  `gate`:
    see ActGate; `pre` (a list) receives the fc1 pre-activation."""
    u = linear(x_ln, p, name + ".fc1")
    if pre is not None:
        pre.append(u.detach())
    h = R(ActGate.apply(u, act, gate))
    return linear(h, p, name + ".fc2")


def mha(x_ln, mem, mask, p, name, H, pos=None):
    """MultiHeadAttention / RelativeMultiHeadAttention (liteasr/nets/attention.py:27-71,
    120-154) on the fused kernels: projections bf16 with bf16 gradients, (q + u), (q + v)
    rounded, FlashAttn, ctx with a bf16 gradient, fp32 output projection."""
    B, Tq, d = x_ln.shape
    dk = d // H
    heads = lambda t: t.reshape(B, -1, H, dk).transpose(1, 2)  # noqa: E731
    q = RG(linear(x_ln, p, name + ".linear_q"))
    src = x_ln if mem is None else mem
    k = RG(linear(src, p, name + ".linear_k"))
    v = RG(linear(src, p, name + ".linear_v"))
    scale = dk ** -0.5
    if pos is not None:
        P = RG(F.linear(pos, p[name + ".linear_pos.weight"])).view(-1, H, dk).transpose(0, 1)
        qu = R(q + p[name + ".pos_bias_u"].reshape(-1))
        qv = R(q + p[name + ".pos_bias_v"].reshape(-1))
        ctx = FlashAttn.apply(heads(qu), heads(qv), heads(k), heads(v), P, mask, scale)
    else:
        qh = heads(q)
        ctx = FlashAttn.apply(qh, qh, heads(k), heads(v), None, mask, scale)
    ctx = G(ctx).transpose(1, 2).reshape(B, Tq, d)
    return linear(ctx, p, name + ".linear_o")


def conv_module(x_ln, p, name, bn_state, training=True):
    """Convolution (liteasr/nets/conformer_convolution.py:44-57) as conv.hip stores it."""
    z1 = RG(F.linear(x_ln, p[name + ".pointwise_conv1.weight"].squeeze(-1), p[name + ".pointwise_conv1.bias"]))
    g = F.glu(z1, dim=-1).transpose(1, 2)
    Kk = p[name + ".depthwise_conv.weight"].shape[-1]
    y = R(F.conv1d(g, p[name + ".depthwise_conv.weight"], p[name + ".depthwise_conv.bias"], padding=(Kk - 1) // 2,
                   groups=g.shape[1]))
    rm = bn_state[name + ".norm.running_mean"] if bn_state is not None else None
    rv = bn_state[name + ".norm.running_var"] if bn_state is not None else None
    y = F.batch_norm(y, rm, rv, p[name + ".norm.weight"], p[name + ".norm.bias"], training, 0.1, 1e-5)
    if bn_state is not None and training:
        bn_state[name + ".norm.num_batches_tracked"] += 1
    h3 = RG(y * torch.sigmoid(y)).transpose(1, 2)
    return F.linear(h3, p[name + ".pointwise_conv2.weight"].squeeze(-1), p[name + ".pointwise_conv2.bias"])


def conformer_layer(x, pos, mask, p, name, H, bn_state, training=True):
    """RelativeEncoderLayer (liteasr/nets/conformer_layer.py:130-147), dropout 0."""
    x = x + 0.5 * G(ffn(RG(layer_norm(x, p, name + ".feed_forward_macaron_norm")), p,
                        name + ".feed_forward_macaron", "swish"))
    x = x + G(mha(RG(layer_norm(x, p, name + ".self_attn_norm")), None, mask, p, name + ".self_attn", H, pos))
    x = x + G(conv_module(RG(layer_norm(x, p, name + ".conv_norm")), p, name + ".conv", bn_state, training))
    x = x + 0.5 * G(ffn(RG(layer_norm(x, p, name + ".feed_forward_norm")), p, name + ".feed_forward", "swish"))
    return layer_norm(x, p, name + ".final_norm")


def encoder(xs, xlens, p, cfg, bn_state=None, training=True, chunk=0):
    """TransformerEncoder (liteasr/nets/transformer_encoder.py:107-127); returns the fp32
    residual stream after the last layer (after_norm is applied by the caller) and the
    key mask."""
    d = cfg["enc_dim"]
    xl = subsample(xs, p, "encoder.embed")
    B, T, _ = xl.shape
    x = math.sqrt(d) * G(xl)
    pos = bf16(O.sinusoid_table(T, d, x.dtype))
    kmask = O.encoder_key_mask(xlens, xs.shape[1])
    mask = kmask[:, None, :]
    if chunk > 0:
        mask = mask | O.triangle_mask(T, stage=chunk)[None]
    for i in range(cfg["enc_layers"]):
        x = conformer_layer(x, pos, mask, p, f"encoder.enc_layers.{i}", cfg["enc_heads"], bn_state, training)
    return x, kmask


def decoder(ys_in, dec_mask, memory, mem_mask, p, cfg):
    """TransformerDecoder (liteasr/nets/transformer_decoder.py:70-93), DecoderLayer
    (liteasr/nets/transformer_layer.py:179-221), dropout 0; logits bf16 with a bf16
    gradient."""
    d = cfg["dec_dim"]
    H = cfg["dec_heads"]
    y = F.embedding(ys_in, p["decoder.embed.weight"]) * math.sqrt(d) + O.sinusoid_table(ys_in.shape[1], d,
                                                                                         memory.dtype)[None]
    mm = mem_mask[:, None, :]
    for i in range(cfg["dec_layers"]):
        n = f"decoder.dec_layers.{i}"
        y = y + G(mha(RG(layer_norm(y, p, n + ".self_attn_norm")), None, dec_mask, p, n + ".self_attn", H))
        y = y + G(mha(RG(layer_norm(y, p, n + ".src_attn_norm")), memory, mm, p, n + ".src_attn", H))
        y = y + G(ffn(RG(layer_norm(y, p, n + ".feed_forward_norm")), p, n + ".feed_forward", "relu"))
    return RG(linear(RG(layer_norm(y, p, "decoder.after_norm")), p, "decoder.linear_out"))


def u2_forward(xs, xlens, ys, ylens, p, cfg, bn_state=None, training=True, chunk=0):
    """U2.forward (liteasr/models/u2.py:116-159); CTC-head dropout 0.  Returns (h_attn,
    h_ctc, h_enc, tgt) like u2_oracle.u2_forward."""
    V = cfg["vocab_size"]
    x, kmask = encoder(xs, xlens, p, cfg, bn_state, training, chunk)
    h_enc = R(layer_norm(x, p, "encoder.after_norm"))  # gradient accumulates in fp32 (HeadsFn)
    ys_in, dec_mask, tgt = O.decoder_io(ys, ylens, V - 1, V - 1)
    h_attn = decoder(ys_in, dec_mask, h_enc, kmask, p, cfg)
    h_ctc = RG(linear(h_enc, p, "ctc.ctc_lo"))
    return h_attn, h_ctc, h_enc, tgt


def loss_and_grads(params, buffers, batch, cfg, ctc_weight=0.3, smoothing=0.1, chunk=0, training=True):
    """Hybrid loss (liteasr/criterions/hybrid_ctc_attn.py:39-79, computed from the bf16
    logits) and every parameter gradient, in float64 with the bf16 build's roundings.
    Returns (loss, loss_ctc, loss_att, grads, h_attn, h_ctc)."""
    xs, xlens, ys, ylens = batch
    names = [k for k in params if params[k].is_floating_point()]
    leaf = {k: params[k].detach().clone().requires_grad_() for k in names}
    h_attn, h_ctc, _, tgt = u2_forward(xs, xlens, ys, ylens, leaf, cfg, buffers, training, chunk)
    loss, lc, la = O.hybrid_loss(h_attn, h_ctc, tgt, ys, xlens, ylens, ctc_weight, smoothing)
    loss.backward()
    grads = {k: (leaf[k].grad if leaf[k].grad is not None else torch.zeros_like(leaf[k])) for k in names}
    return loss.detach(), lc.detach(), la.detach(), grads, h_attn.detach(), h_ctc.detach()
