"""Fused forward/backward of the U2 hot path on the HIP kernels.

Granularity (one autograd node each, so torch's engine only chains a handful of
nodes and never casts/sums tensors itself):
  EmbedConvFn      Conv2d subsampling convolutions                      subsampling.py:42-46
  EmbedOutFn       its output projection + x*sqrt(d) (+dropout)        subsampling.py:47-48, positional_encoding.py:68-75
  ConformerLayerFn one RelativeEncoderLayer (macaron FFN, rel-pos MHSA,  conformer_layer.py:130-147
                   conv module, FFN, final LN)
  HeadsFn          encoder after_norm + CTC head (input dropout always   transformer_encoder.py:126, ctc.py:28-30,
                   on) + the whole Transformer decoder                  transformer_decoder.py:70-93
  HybridLossFn     label-smoothed KL + CTC, combined                    criterions/hybrid_ctc_attn.py:39-79

Weight gradients never travel through autograd: the backward kernels accumulate them
(beta = 1) straight into the flat fp32 grad buffer of FlatParams; autograd only
carries the residual-stream gradient between nodes.  Each node takes one "anchor"
parameter as an input so that its output requires grad whenever the model does.

Storage: residual streams fp32; GEMM operands / activations in the model's compute
dtype ``adt`` (bf16, or fp32 for the parity build); attention scores fp32.
"""

from __future__ import annotations

import math
import os
from types import SimpleNamespace

import torch

from .. import kernels as K
from .._native import ACT_GATE, ACT_NONE, ACT_RELU, ACT_SWISH, ACT_TANH
from ..utils.markers import ranged

F32 = torch.float32
LN_EPS = 1e-12


def _e(shape, dtype, dev):
    return torch.empty(shape, dtype=dtype, device=dev)


def ld_scores(T):
    return (T + 7) // 8 * 8


def _seed(base, k):
    return (base * 0x100000001B3 + k * 0x9E3779B1 + 1) & 0xFFFFFFFFFFFFFFFF


# ===================================================================== helpers ===
def ln_forward(x, g, b, adt, y2=False, p2=0.0, seed2=0):
    rows, D = x.shape
    dev = x.device
    y = _e((rows, D), adt, dev)
    mean = _e(rows, F32, dev)
    rstd = _e(rows, F32, dev)
    yd = _e((rows, D), adt, dev) if y2 else None
    K.layernorm_fwd(x, g, b, LN_EPS, y, mean, rstd, yd, p2, seed2)
    return y, yd, mean, rstd


# Full-row GEMM tiles with the next LayerNorm in the epilogue (gemm_row.hip): a residual
# projection and the norm after it, or an input-gradient GEMM and the norm backward before
# it, in one launch, bit-identical to the two launches.  LASR_ROW_LN=0 keeps two launches
# (benchmark A/B); shapes the kernel does not take (fp32 build, other widths) keep them too.
ROW_LN = os.environ.get("LASR_ROW_LN", "1") != "0"
# the decoder's norms after / before its attention projections on the row kernel (A/B switch)
DEC_ROW_LN = os.environ.get("LASR_DEC_ROW_LN", "1") != "0"
# K >= 1024 GEMMs whose plan splits K (the decoder's FFN on B*(L+1) rows) run the following
# LayerNorm (forward) / the preceding one's backward in their split-K reduction launch
# (gemm_ln.hip); False: separate launches (tests/test_fusions_gpu.py pins the two bit for bit)
SPLITK_LN = True
# the encoder attention's positional-bias gradient (qbias_bwd) in the positional-projection
# gradient GEMM's split-K reduction launch (gemm_ln.hip lasr_gemm_qbias_bwd); False: its own launch
QBIAS_IN_REDUCE = True
# a Conformer layer's first-norm backward and the previous layer's final-norm backward in one
# launch (lasr_layernorm2_bwd, the reverse of FUSED_LN2's chained forward): the previous layer
# receives its final norm's input gradient instead of computing it; False: two launches with
# the fp32 gradient between them (tests/test_fusions_gpu.py pins the two bit for bit)
LN2_BWD_CHAIN = True
# the conv module's BatchNorm + activation backward folded into the depthwise-conv / GLU
# backward (lasr_bn_act_glu_dwconv_bwd: dy computed in its window load, never stored); False: the
# two launches with the fp32 dy between them (tests/test_fusions_gpu.py pins the two bit for bit)
BN_GLU_FUSED = True
# the encoder layers' parameter-gradient reductions (LayerNorm gamma / beta, split-K weight
# slabs, positional biases, depthwise conv) queued across layer nodes and launched together at
# the lowest layer of each backward segment (kernels.deferred_reductions(hold=True)); the
# layers' gradient-ready hooks fire after that launch.  False: one reduction launch per layer
# (tests/test_fusions_gpu.py pins the two bit for bit)
LAYER_RED_HOLD = True


def _red_hold(env, layer):
    """Whether this encoder layer's backward node may leave its reductions queued: not the
    last layer node of its backward segment (the model lists those in env.red_flush)."""
    fl = getattr(env, "red_flush", None)
    return LAYER_RED_HOLD and fl is not None and id(layer) not in fl


class PostLN(SimpleNamespace):
    """A LayerNorm to run on a residual projection's output row in the same launch:
    g, b (its parameters), f32 (y1 stored fp32: a layer's final norm), nxt (optional
    (g2, b2) of a chained second norm, bf16 out).  After the call: y1, m1, r1 (+ y2, m2, r2)."""


def res_proj(x, W, bias, res, res_scale, p_res, s_res, post=None):
    """out = res + res_scale * drop(x W^T + bias) (fp32 residual stream); when `post` names
    the following LayerNorm and the row kernel takes the shape, the norm runs in the same
    launch and its outputs are set on `post` (post.y1 stays None otherwise)."""
    M, D = x.shape[0], W.shape[0]
    dev = x.device
    out = _e((M, D), F32, dev)
    if post is not None:
        post.y1 = None
    if post is None or not ROW_LN or not K.row_ln_ok(x, W, D):
        if post is not None and SPLITK_LN and post.nxt is None and x.dtype == torch.bfloat16 and W.shape[1] >= 1024:
            # the norm in the GEMM's split-K reduction launch (lasr_gemm_ln_fwd; two launches
            # when the plan does not split K)
            post.y1 = _e((M, D), F32 if post.f32 else x.dtype, dev)
            post.m1, post.r1 = _e(M, F32, dev), _e(M, F32, dev)
            K.linear(x, W, out, bias=bias, res=res, res_scale=res_scale, drop_p=p_res, drop_seed=s_res,
                     ln_fwd=(post.g, post.b, LN_EPS, post.y1, post.m1, post.r1))
            return out
        K.linear(x, W, out, bias=bias, res=res, res_scale=res_scale, drop_p=p_res, drop_seed=s_res)
        return out
    post.y1 = _e((M, D), F32 if post.f32 else x.dtype, dev)
    post.m1, post.r1 = _e(M, F32, dev), _e(M, F32, dev)
    kw = {}
    if post.nxt is not None:
        post.y2 = _e((M, D), x.dtype, dev)
        post.m2, post.r2 = _e(M, F32, dev), _e(M, F32, dev)
        kw = dict(g2=post.nxt[0], b2=post.nxt[1], y2=post.y2, mean2=post.m2, rstd2=post.r2)
    K.linear_res_ln(x, W, out, post.y1, post.m1, post.r1, post.g, post.b, LN_EPS, bias=bias, res=res,
                    res_scale=res_scale, drop_p=p_res, drop_seed=s_res, **kw)
    return out


class LnBwd(SimpleNamespace):
    """The LayerNorm backward that consumes an input-gradient GEMM's output dln (the norm
    in front of a sub-block, liteasr/nets/conformer_layer.py:37-66): x, g (gamma), mean,
    rstd, dx (fp32 out), dgamma, dbeta, and optionally dres (fp32 residual gradient added),
    gb (+ bscale, bp, bseed: the preceding branch's gradient, layernorm_bwd's gb)."""


def dx_ln(dy, W, lnb):
    """dln = dy @ W ([M, K] x [K, D]); with `lnb` the LayerNorm backward of dln follows (one
    launch on the row kernel when it takes the shape) and None is returned, else dln.
    lnb.chain (an LnBwd on lnb.dx: the previous layer's final norm, ConformerLayerFn) runs
    right after it -- in the same launch as lnb's (lasr_layernorm2_bwd, lnb.dx never stored)
    when lnb is not on the row kernel."""
    M, D = dy.shape[0], W.shape[1]
    ch = getattr(lnb, "chain", None) if lnb is not None else None
    if lnb is not None and ROW_LN and K.row_ln_ok(dy, W, D) and lnb.x.dtype == F32 and lnb.dx.dtype == F32:
        K.linear_dx_ln_bwd(dy, W, lnb.x, lnb.g, lnb.mean, lnb.rstd, lnb.dx, lnb.dgamma, lnb.dbeta,
                           dres=lnb.dres, gb=lnb.gb, bscale=lnb.bscale, bp=lnb.bp, bseed=lnb.bseed)
        if ch is not None:
            ln_bwd_of(lnb.dx, ch)
        return None
    dln = _e((M, D), dy.dtype, dy.device)
    if ch is not None:
        assert lnb.gb is None and lnb.dres is not None and ch.dres is None and lnb.x.dtype == F32
        K.gemm(dy, W, dln)
        K.layernorm2_bwd(lnb.x, dln, lnb.dres, lnb.g, lnb.mean, lnb.rstd, lnb.dgamma, lnb.dbeta, ch.x, ch.g,
                         ch.mean, ch.rstd, ch.dx, ch.dgamma, ch.dbeta, gb2=ch.gb, bscale=ch.bscale, bp=ch.bp,
                         bseed=ch.bseed)
        return None
    if lnb is not None and SPLITK_LN and dy.dtype == torch.bfloat16 and W.shape[0] >= 1024:
        # the norm backward in the GEMM's split-K reduction launch (lasr_gemm_ln_bwd; two
        # launches when the plan does not split K)
        K.gemm(dy, W, dln, ln_bwd=lnb)
        return None
    K.gemm(dy, W, dln)
    if lnb is None:
        return dln
    ln_bwd_of(dln, lnb)
    return None


def ln_bwd_of(dln, lnb):
    """The LayerNorm backward `lnb` describes, on an already computed dln (the paths whose
    input-gradient GEMM is not the row kernel's: dx_ln does both in one launch)."""
    K.layernorm_bwd(lnb.x, dln, lnb.g, lnb.mean, lnb.rstd, lnb.dx, lnb.dgamma, lnb.dbeta, dres=lnb.dres,
                    gb=lnb.gb, bscale=lnb.bscale, bp=lnb.bp, bseed=lnb.bseed)


def ffn_forward(ln, W1, b1, W2, b2, act, p_ff, s_ff, res, res_scale, p_res, s_res, post=None):
    """Returns (out, g, h).  g is the gate act'(u) * keep the backward needs, stored in the
    compute dtype by the fc1 epilogue (zout_mode 1): h = drop(act(u)) and g come out of the
    same launch, and the backward's dz GEMM multiplies by g (no recompute of u).  `post`:
    the LayerNorm after the residual add (res_proj)."""
    M = ln.shape[0]
    dev, adt = ln.device, ln.dtype
    h = _e((M, W1.shape[0]), adt, dev)
    g = _e((M, W1.shape[0]), adt, dev)
    K.linear(ln, W1, h, bias=b1, act=act, zout=g, zout_mode=1, drop_p=p_ff, drop_seed=s_ff)
    out = res_proj(h, W2, b2, res, res_scale, p_res, s_res, post)
    return out, g, h


def ffn_backward(gb, ln, g, h, W1, W2, gW1, gb1, gW2, gb2, act, p_ff, s_ff, lnb=None):
    """gb: gradient of the FFN output (after the residual-branch dropout/scale); g: the
    forward's stored gate act'(z) * keep.  Returns dln, or None when `lnb` (the norm in
    front of the FFN) consumed it (dx_ln)."""
    M = gb.shape[0]
    dev, adt = gb.device, gb.dtype
    K.gemm(gb.t(), h, gW2, beta=1.0, split_k=0, rowsum=gb2, group=True)
    dz = _e((M, W1.shape[0]), adt, dev)
    # dz = (gb W2) * scale * g: the dropout scale as alpha, the gate as aux
    K.gemm(gb, W2, dz, alpha=K.dropout_scale(p_ff), aux=g, aux_act=ACT_GATE)
    K.gemm(dz.t(), ln, gW1, beta=1.0, split_k=0, rowsum=gb1, group=True)
    return dx_ln(dz, W1, lnb)


def _heads(t, B, T, H, dk):
    """[B*T, H*dk] (row stride arbitrary) -> (B, H, T, dk) view."""
    return t.view(B, T, H, dk).permute(0, 2, 1, 3) if t.is_contiguous() else \
        t.unflatten(0, (B, T)).unflatten(2, (H, dk)).permute(0, 2, 1, 3)


def _slot(t, B, T, nslot, k, H, dk):
    """Slot k of a fused [B*T, nslot*H*dk] projection (row stride arbitrary) as (B, H, T, dk)."""
    if t.is_contiguous():
        return t.view(B, T, nslot, H, dk)[:, :, k].permute(0, 2, 1, 3)
    return t.unflatten(0, (B, T)).unflatten(2, (nslot, H, dk))[:, :, k].permute(0, 2, 1, 3)


# ============================================================ rel-pos MHSA ======
FUSED_RELATTN = True


def fused_relattn(adt, dk, p_att):
    """The fused kernels (attn_flash.hip) cover bf16, d_k 32 or 64, no attention dropout
    (the my_U2 preset); other shapes take the materialised-score kernels."""
    return FUSED_RELATTN and adt == torch.bfloat16 and dk in (32, 64) and p_att == 0.0


BATCH_POS_PROJ = os.environ.get("LASR_BATCH_POS_PROJ", "1") != "0"
# a layer's final norm and the next layer's first norm in one launch (lasr_layernorm2_fwd)
FUSED_LN2 = os.environ.get("LASR_FUSED_LN2", "1") != "0"


def pos_projections(pos, Ws):
    """p_j = pos @ Wpos_j^T of every encoder layer in ONE batched GEMM (positional_encoding +
    attention.py:95 linear_pos; the table is the same for all layers): the layers' weights
    sit at a constant stride in the flat parameter store, so they form one strided batch.
    None when they do not (the layers then project their own)."""
    n = len(Ws)
    if n < 2 or not all(W.is_contiguous() for W in Ws):
        return None
    base = Ws[0].untyped_storage().data_ptr()
    if any(W.untyped_storage().data_ptr() != base for W in Ws):
        return None
    offs = [W.storage_offset() for W in Ws]
    st = offs[1] - offs[0]
    if st <= 0 or any(offs[j] - offs[0] != j * st for j in range(n)):
        return None
    dout, din = Ws[0].shape
    Wt = torch.as_strided(Ws[0], (n, din, dout), (st, 1, din), offs[0])  # W_j^T
    T = pos.shape[0]
    out = _e((n, T, dout), pos.dtype, pos.device)
    K.gemm(pos.unsqueeze(0).expand(n, T, din), Wt, out)
    return [out[j] for j in range(n)]


def relmha_forward(ln, pos, w, env, x_in, p_att, s_att, p_res, s_res, p=None, post=None):
    B, T, H = env.B, env.T, env.H
    d = ln.shape[1]
    dk = d // H
    dev, adt = ln.device, ln.dtype
    M = B * T
    scale = dk ** -0.5
    qkv = _e((M, 3 * d), adt, dev)
    K.linear(ln, w.Wqkv, qkv, bias=w.bqkv)
    if p is None:  # else precomputed for all layers at once (pos_projections)
        p = _e((T, d), adt, dev)
        K.linear(pos, w.Wpos, p)
    qu = _e((M, d), adt, dev)
    qv = _e((M, d), adt, dev)
    if fused_relattn(adt, dk, p_att):
        # scores never materialised (attn_flash.hip); row stats kept for the backward; the
        # kernel forms qu / qv from q and the biases itself (lasr_relattn_fwd_qb)
        stats = _e((B * H * T * 2,), F32, dev)
        ctx = _e((M, d), adt, dev)
        K.relattn_fwd_qb(qkv[:, :d], w.u, w.v, qu, qv, qkv[:, d:2 * d], qkv[:, 2 * d:], p, B, H, T, env.mask,
                         env.msb, env.msq, scale, stats, ctx)
        out = res_proj(ctx, w.Wo, w.bo, x_in, 1.0, p_res, s_res, post)
        return out, SimpleNamespace(qkv=qkv, p=p, qu=qu, qv=qv, ctx=ctx, stats=stats)
    K.qbias_fwd(qkv, B, T, H, dk, w.u, w.v, qu, qv)
    ldS = ld_scores(T)
    Sac = _e((B, H, T, ldS), F32, dev)
    Sbd = _e((B, H, T, ldS), F32, dev)
    k4 = _slot(qkv, B, T, 3, 1, H, dk)
    v4 = _slot(qkv, B, T, 3, 2, H, dk)
    p4 = p.view(T, H, dk).permute(1, 0, 2).unsqueeze(0).expand(B, H, T, dk)
    K.gemm(_heads(qu, B, T, H, dk), k4.transpose(-1, -2), Sac[..., :T], alpha=scale)
    K.gemm(_heads(qv, B, T, H, dk), p4.transpose(-1, -2), Sbd[..., :T], alpha=scale)
    P = _e((B, H, T, ldS), adt, dev)
    Praw = _e((B, H, T, ldS), adt, dev) if p_att > 0 else None
    K.attn_softmax_fwd(Sac, Sbd, B, H, T, T, ldS, env.mask, env.msb, env.msq, P, p_att, s_att, Praw)
    ctx = _e((M, d), adt, dev)
    K.gemm(P[..., :T], v4, _heads(ctx, B, T, H, dk))
    out = res_proj(ctx, w.Wo, w.bo, x_in, 1.0, p_res, s_res, post)
    saved = SimpleNamespace(qkv=qkv, p=p, qu=qu, qv=qv, P=P, Praw=Praw, ctx=ctx, stats=None)
    return out, saved


def relmha_backward(gb, ln, pos, sv, w, g, env, p_att, s_att, lnb=None):
    B, T, H = env.B, env.T, env.H
    d = ln.shape[1]
    dk = d // H
    dev, adt = ln.device, ln.dtype
    M = B * T
    scale = dk ** -0.5
    ldS = ld_scores(T)
    K.gemm(gb.t(), sv.ctx, g.Wo, beta=1.0, split_k=0, rowsum=g.bo, group=True)
    dctx = _e((M, d), adt, dev)
    K.gemm(gb, w.Wo, dctx)
    dqkv = _e((M, 3 * d), adt, dev)
    dqu = _e((M, d), adt, dev)
    if sv.stats is not None:
        # fused recompute backward: dqu, dk, dv and the pre-shift bd gradient, head-major
        # ([H][B][T][ldS]) so the positional gradient is one K = B*T GEMM per head
        dBDh = _e((H, B, T, ldS), adt, dev)
        Dbuf = _e((B * H * T,), F32, dev)
        K.relattn_bwd(sv.qu, sv.qv, sv.qkv[:, d:2 * d], sv.qkv[:, 2 * d:], sv.p, B, H, T, env.mask,
                      env.msb, env.msq, scale, sv.stats, sv.ctx, dctx, Dbuf, dqu, dBDh, ldS,
                      dqkv[:, d:2 * d], dqkv[:, 2 * d:], dbd_head_major=True)
        p4 = sv.p.view(T, H, dk).permute(1, 0, 2).unsqueeze(0).expand(B, H, T, dk)
        dqv = _e((M, d), adt, dev)
        K.gemm(dBDh.permute(1, 0, 2, 3)[..., :T], p4, _heads(dqv, B, T, H, dk), alpha=scale)
        dp = _e((T, d), adt, dev)
        # (qbias_bwd's blocks ride in this GEMM's split-K reduction launch: QBIAS_IN_REDUCE)
        qb = (dqu, dqv, B, T, H, dk, dqkv, g.u, g.v)
        K.gemm(dBDh.view(H, B * T, ldS)[..., :T].transpose(-1, -2), sv.qv.view(M, H, dk).permute(1, 0, 2),
               dp.view(T, H, dk).permute(1, 0, 2), alpha=scale, split_k=0, qbias=qb if QBIAS_IN_REDUCE else None)
        if not QBIAS_IN_REDUCE:
            K.qbias_bwd(*qb)
        K.gemm(dp.t(), pos, g.Wpos, beta=1.0, split_k=0, group=True)
        K.gemm(dqkv.t(), ln, g.Wqkv, beta=1.0, split_k=0, rowsum=g.bqkv, group=True)
        return dx_ln(dqkv, w.Wqkv, lnb)
    dBD = _e((B, H, T, ldS), adt, dev)
    # materialised-score backward (fp32 build, attention dropout, other d_k)
    dctx4 = _heads(dctx, B, T, H, dk)
    v4 = _slot(sv.qkv, B, T, 3, 2, H, dk)
    k4 = _slot(sv.qkv, B, T, 3, 1, H, dk)
    dPd = _e((B, H, T, ldS), F32, dev)
    K.gemm(dctx4, v4.transpose(-1, -2), dPd[..., :T])
    K.gemm(sv.P[..., :T].transpose(-1, -2), dctx4, _slot(dqkv, B, T, 3, 2, H, dk))
    dS = _e((B, H, T, ldS), adt, dev)
    K.attn_softmax_bwd(sv.Praw if sv.Praw is not None else sv.P, dPd, B, H, T, T, ldS, env.mask,
                       env.msb, env.msq, dS, p_att, s_att)
    K.relshift_bwd(dS.view(B * H, T, ldS), B * H, T, ldS, dBD)
    K.gemm(dS[..., :T], k4, _heads(dqu, B, T, H, dk), alpha=scale)
    K.gemm(dS[..., :T].transpose(-1, -2), _heads(sv.qu, B, T, H, dk), _slot(dqkv, B, T, 3, 1, H, dk),
           alpha=scale)
    p4 = sv.p.view(T, H, dk).permute(1, 0, 2).unsqueeze(0).expand(B, H, T, dk)
    dqv = _e((M, d), adt, dev)
    K.gemm(dBD[..., :T], p4, _heads(dqv, B, T, H, dk), alpha=scale)
    dpb = _e((B, H, T, dk), F32, dev)
    K.gemm(dBD[..., :T].transpose(-1, -2), _heads(sv.qv, B, T, H, dk), dpb, alpha=scale)
    dp = _e((T, d), adt, dev)
    K.reduce_batch(dpb, B, H, T, dk, dp)
    K.qbias_bwd(dqu, dqv, B, T, H, dk, dqkv, g.u, g.v)
    K.gemm(dp.t(), pos, g.Wpos, beta=1.0, split_k=0, group=True)
    K.gemm(dqkv.t(), ln, g.Wqkv, beta=1.0, split_k=0, rowsum=g.bqkv, group=True)
    return dx_ln(dqkv, w.Wqkv, lnb)


# ============================================================ plain MHA =========
# Decoder attention on the fused kernels (attn_flash.hip, lasr_attn_fwd/bwd: the relative-
# position kernels without the positional term, Tq queries x Tk keys): scores / softmax /
# P.V (3 launches forward, 5 backward) become 1 + 2 launches, for the self attention (causal +
# padding mask) and the source attention over the encoder output (key padding).
# LASR_FUSED_DEC_ATTN=0 keeps the materialised path.
FUSED_DEC_ATTN = os.environ.get("LASR_FUSED_DEC_ATTN", "1") != "0"
# the decoder FFN branch gradients written by the LayerNorm backward that produces each layer's
# output gradient (False: a branch_grad launch per layer; the test pins the two bit for bit)
DEC_GB_IN_LN = True


def _fused_dec(adt, dk, p_att):
    return FUSED_DEC_ATTN and fused_relattn(adt, dk, p_att)


def mha_forward(ln, mem, w, B, Tq, Tk, H, mask, msb, msq, x_in, p_att, s_att, p_res, s_res, kv=None, post=None):
    """Decoder self (mem None) / source attention (liteasr/nets/attention.py:61-71).  kv: the
    memory's key/value projection [B*Tk, 2d] already computed (decoder_layers_fwd batches it
    over the layers); None computes it here.  post: the LayerNorm after the residual add, in
    the output projection's launch when the row kernel takes it (res_proj)."""
    d = ln.shape[1]
    dk = d // H
    dev, adt = ln.device, ln.dtype
    R = B * Tq
    scale = dk ** -0.5
    if _fused_dec(adt, dk, p_att):
        if mem is None:
            qkv = _e((R, 3 * d), adt, dev)
            K.linear(ln, w.Wqkv, qkv, bias=w.bqkv)
            q, k, v, kv = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], None
        else:
            qkv = None
            q = _e((R, d), adt, dev)
            K.linear(ln, w.Wq, q, bias=w.bq)
            if kv is None:
                kv = _e((B * Tk, 2 * d), adt, dev)
                K.linear(mem, w.Wkv, kv, bias=w.bkv)
            k, v = kv[:, :d], kv[:, d:]
        stats = _e((B * H * Tq * 2,), F32, dev)
        ctx = _e((R, d), adt, dev)
        K.attn_fwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx)
        out = res_proj(ctx, w.Wo, w.bo, x_in, 1.0, p_res, s_res, post)
        return out, SimpleNamespace(qkv=qkv, q=q if mem is not None else None, kv=kv, P=None, Praw=None, ctx=ctx,
                                    stats=stats)
    if mem is None:
        qkv = _e((R, 3 * d), adt, dev)
        K.linear(ln, w.Wqkv, qkv, bias=w.bqkv)
        q4 = _slot(qkv, B, Tq, 3, 0, H, dk)
        k4 = _slot(qkv, B, Tk, 3, 1, H, dk)
        v4 = _slot(qkv, B, Tk, 3, 2, H, dk)
        q = kv = None
    else:
        q = _e((R, d), adt, dev)
        K.linear(ln, w.Wq, q, bias=w.bq)
        if kv is None:
            kv = _e((B * Tk, 2 * d), adt, dev)
            K.linear(mem, w.Wkv, kv, bias=w.bkv)
        q4 = _heads(q, B, Tq, H, dk)
        k4 = _slot(kv, B, Tk, 2, 0, H, dk)
        v4 = _slot(kv, B, Tk, 2, 1, H, dk)
        qkv = None
    ldS = ld_scores(Tk)
    S = _e((B, H, Tq, ldS), F32, dev)
    K.gemm(q4, k4.transpose(-1, -2), S[..., :Tk], alpha=scale)
    P = _e((B, H, Tq, ldS), adt, dev)
    Praw = _e((B, H, Tq, ldS), adt, dev) if p_att > 0 else None
    K.attn_softmax_fwd(S, None, B, H, Tq, Tk, ldS, mask, msb, msq, P, p_att, s_att, Praw)
    ctx = _e((R, d), adt, dev)
    K.gemm(P[..., :Tk], v4, _heads(ctx, B, Tq, H, dk))
    out = res_proj(ctx, w.Wo, w.bo, x_in, 1.0, p_res, s_res, post)
    return out, SimpleNamespace(qkv=qkv, q=q, kv=kv, P=P, Praw=Praw, ctx=ctx, stats=None)


def mha_backward(gb, ln, mem, sv, w, g, B, Tq, Tk, H, mask, msb, msq, p_att, s_att, dmem, dkv=None, lnb=None):
    """dkv: [B*Tk, 2d] destination of the key/value projection's gradient, whose weight /
    memory gradients the caller then computes (decoder_layers_bwd, batched over the layers);
    None computes them here (dmem accumulates).  lnb: the LayerNorm in front of the attention,
    whose backward the input-gradient GEMM runs (dx_ln; None is returned when it did)."""
    own_kv = dkv is None
    d = ln.shape[1]
    dk = d // H
    dev, adt = ln.device, ln.dtype
    R = B * Tq
    scale = dk ** -0.5
    ldS = ld_scores(Tk)
    K.gemm(gb.t(), sv.ctx, g.Wo, beta=1.0, split_k=0, rowsum=g.bo, group=True)
    dctx = _e((R, d), adt, dev)
    K.gemm(gb, w.Wo, dctx)
    if getattr(sv, "stats", None) is not None:  # fused attention (mha_forward)
        Dbuf = _e((B * H * Tq,), F32, dev)
        if mem is None:
            dqkv = _e((R, 3 * d), adt, dev)
            K.attn_bwd(sv.qkv[:, :d], sv.qkv[:, d:2 * d], sv.qkv[:, 2 * d:], B, H, Tq, Tk, mask, msb, msq, scale,
                       sv.stats, sv.ctx, dctx, Dbuf, dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:])
            K.gemm(dqkv.t(), ln, g.Wqkv, beta=1.0, split_k=0, rowsum=g.bqkv, group=True)
            return dx_ln(dqkv, w.Wqkv, lnb)
        dq = _e((R, d), adt, dev)
        if own_kv:
            dkv = _e((B * Tk, 2 * d), adt, dev)
        K.attn_bwd(sv.q, sv.kv[:, :d], sv.kv[:, d:], B, H, Tq, Tk, mask, msb, msq, scale, sv.stats, sv.ctx, dctx,
                   Dbuf, dq, dkv[:, :d], dkv[:, d:])
        K.gemm(dq.t(), ln, g.Wq, beta=1.0, split_k=0, rowsum=g.bq, group=True)
        if own_kv:
            K.gemm(dkv.t(), mem, g.Wkv, beta=1.0, split_k=0, rowsum=g.bkv, group=True)
            K.gemm(dkv, w.Wkv, dmem, beta=1.0)
        return dx_ln(dq, w.Wq, lnb)
    dctx4 = _heads(dctx, B, Tq, H, dk)
    if mem is None:
        q4 = _slot(sv.qkv, B, Tq, 3, 0, H, dk)
        k4 = _slot(sv.qkv, B, Tk, 3, 1, H, dk)
        v4 = _slot(sv.qkv, B, Tk, 3, 2, H, dk)
        dqkv = _e((R, 3 * d), adt, dev)
        dq4, dk4, dv4 = (_slot(dqkv, B, Tq, 3, i, H, dk) for i in range(3))
    else:
        q4 = _heads(sv.q, B, Tq, H, dk)
        k4 = _slot(sv.kv, B, Tk, 2, 0, H, dk)
        v4 = _slot(sv.kv, B, Tk, 2, 1, H, dk)
        dq = _e((R, d), adt, dev)
        if own_kv:
            dkv = _e((B * Tk, 2 * d), adt, dev)
        dq4 = _heads(dq, B, Tq, H, dk)
        dk4 = _slot(dkv, B, Tk, 2, 0, H, dk)
        dv4 = _slot(dkv, B, Tk, 2, 1, H, dk)
    dPd = _e((B, H, Tq, ldS), F32, dev)
    K.gemm(dctx4, v4.transpose(-1, -2), dPd[..., :Tk])
    K.gemm(sv.P[..., :Tk].transpose(-1, -2), dctx4, dv4)
    dS = _e((B, H, Tq, ldS), adt, dev)
    K.attn_softmax_bwd(sv.Praw if sv.Praw is not None else sv.P, dPd, B, H, Tq, Tk, ldS, mask, msb,
                       msq, dS, p_att, s_att)
    K.gemm(dS[..., :Tk], k4, dq4, alpha=scale)
    K.gemm(dS[..., :Tk].transpose(-1, -2), q4, dk4, alpha=scale)
    if mem is None:
        K.gemm(dqkv.t(), ln, g.Wqkv, beta=1.0, split_k=0, rowsum=g.bqkv, group=True)
        return dx_ln(dqkv, w.Wqkv, lnb)
    K.gemm(dq.t(), ln, g.Wq, beta=1.0, split_k=0, rowsum=g.bq, group=True)
    if own_kv:
        K.gemm(dkv.t(), mem, g.Wkv, beta=1.0, split_k=0, rowsum=g.bkv, group=True)
        K.gemm(dkv, w.Wkv, dmem, beta=1.0)
    return dx_ln(dq, w.Wq, lnb)


# ========================================================= conformer conv =======
def conv_forward(ln, w, env, x_in, p_res, s_res, training, post=None):
    B, T = env.B, env.T
    M, d = ln.shape
    dev, adt = ln.device, ln.dtype
    z1 = _e((M, 2 * d), adt, dev)
    K.linear(ln, w.Wpw1, z1, bias=w.bpw1)
    y = _e((M, d), adt, dev)
    nparts = K.dwconv_nparts(B, T)
    stats = _e(nparts * 3 * d, F32, dev)
    K.glu_dwconv_fwd(z1, B, T, d, w.kernel, w.wdw, w.bdw, y, stats)
    mean, rstd, scale, shift = (_e(d, F32, dev) for _ in range(4))
    K.bn_finalize(stats, nparts, d, 1e-5, 0.1, w.gamma, w.beta, w.rmean, w.rvar, w.nbt, mean, rstd,
                  scale, shift, 1 if training else 2)
    h3 = _e((M, d), adt, dev)
    K.bn_act_fwd(y, scale, shift, h3, act=getattr(w, "act", ACT_SWISH))
    out = res_proj(h3, w.Wpw2, w.bpw2, x_in, 1.0, p_res, s_res, post)
    return out, SimpleNamespace(z1=z1, y=y, mean=mean, rstd=rstd, scale=scale, shift=shift, h3=h3,
                                training=training)


def conv_backward(gb, ln, sv, w, g, env, lnb=None):
    B, T = env.B, env.T
    M, d = ln.shape
    dev, adt = ln.device, ln.dtype
    K.gemm(gb.t(), sv.h3, g.Wpw2, beta=1.0, split_k=0, rowsum=g.bpw2, group=True)
    dh3 = _e((M, d), adt, dev)
    K.gemm(gb, w.Wpw2, dh3)
    dz1 = _e((M, 2 * d), adt, dev)
    if BN_GLU_FUSED and d % 8 == 0:
        # the BN backward's dy computed inside the depthwise backward's window load (never stored)
        K.bn_act_glu_dwconv_bwd(sv.y, dh3, sv.scale, sv.shift, sv.mean, sv.rstd, w.gamma, g.gamma, g.beta, sv.z1,
                                B, T, d, w.kernel, w.wdw, dz1, g.wdw, g.bdw, batch_stats=sv.training,
                                act=getattr(w, "act", ACT_SWISH))
    else:
        dy = _e((M, d), F32, dev)
        K.bn_act_bwd(sv.y, dh3, sv.scale, sv.shift, sv.mean, sv.rstd, w.gamma, g.gamma, g.beta, dy,
                     batch_stats=sv.training, act=getattr(w, "act", ACT_SWISH))
        K.glu_dwconv_bwd(sv.z1, dy, B, T, d, w.kernel, w.wdw, dz1, g.wdw, g.bdw)
    K.gemm(dz1.t(), ln, g.Wpw1, beta=1.0, split_k=0, rowsum=g.bpw1, group=True)
    return dx_ln(dz1, w.Wpw1, lnb)


def _conv2_implicit(adt, C):
    """conv2 on the implicit-GEMM instances (bf16 build, C % 128 == 0); the fp32 parity build
    and other widths take explicit im2col + the GEMM."""
    return adt == torch.bfloat16 and C % 128 == 0


# ============================================================ autograd nodes ====
@ranged
class EmbedConvFn(torch.autograd.Function):
    """Conv2DLayer's two convolutions (liteasr/nets/subsampling.py:42-46): y2 = relu(conv2(
    relu(conv1(x)))), channels-last, as [roundup32(M2 + 1), C] rows (the rows past M2 are the
    zero tail the implicit backward GEMMs read in dy2; EmbedOutFn's backward returns dy2 in
    that shape).  Its backward finishes conv2's and conv1's weight gradients and reports the
    data-parallel unit ``<embed>.conv``."""

    @staticmethod
    def forward(ctx, xs, anchor, mod, env):
        B, Tx, Fd = xs.shape
        w = mod.weights()
        C = w.C
        adt, dev = env.adt, xs.device
        T1, F1 = (Tx - 3) // 2 + 1, (Fd - 3) // 2 + 1
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        M2 = B * T2 * F2
        xs = xs.contiguous()
        y1 = _e((B, T1, F1, C), adt, dev)
        K.conv1_fwd(xs, w.W1, w.b1, y1)
        y2_full = _e((K.conv2_dy2_rows(M2), C), adt, dev)
        y2_full[M2:].zero_()  # the tail rows are part of the autograd output: defined (zero)
        y2 = y2_full[:M2]
        implicit = _conv2_implicit(adt, C)
        if implicit:  # conv2 as implicit GEMM: im2col(y1) is never materialised
            col = None
            K.conv2_fwd(y1, w.W2p, w.b2, y2)
        else:  # fp32 parity build: explicit im2col + GEMM
            col = _e((M2, 9 * C), adt, dev)
            K.im2col(y1, col)
            K.linear(col, w.W2p, y2, bias=w.b2, act=ACT_RELU)
        ctx.sv = SimpleNamespace(xs=xs, y1=y1, col=col, dims=(B, T1, F1, T2, F2, C), implicit=implicit)
        ctx.mod, ctx.env = mod, env
        return y2_full

    @staticmethod
    def backward(ctx, dy2_full):
        sv, mod = ctx.sv, ctx.mod
        B, T1, F1, T2, F2, C = sv.dims
        w, g = mod.weights(), mod.grads()
        M2 = B * T2 * F2
        dev = dy2_full.device
        dW2 = _e((C, 9 * C), F32, dev)
        if sv.implicit and K.conv2_dx_w1_ok(C):
            # dW2 = dy2^T im2col(y1); dy1 = col2im(dy2 W2p) * relu'(y1) is consumed inside the
            # data-gradient GEMM's epilogue by conv1's weight gradient (never written or re-read)
            K.conv2_dw(dy2_full, sv.y1, dW2, rowsum=g.b2)
            K.permute_last2(dW2, C, C, 9, g.conv2_w, reverse=True, accumulate=True)
            K.conv2_dx_w1(dy2_full, w.W2p, sv.y1, sv.xs, g.W1, g.b1)
        else:
            dy1 = torch.empty_like(sv.y1)
            if sv.implicit:
                K.conv2_dw(dy2_full, sv.y1, dW2, rowsum=g.b2)
                K.permute_last2(dW2, C, C, 9, g.conv2_w, reverse=True, accumulate=True)
                K.conv2_dx(dy2_full, w.W2p, sv.y1, dy1)
            else:
                dy2 = dy2_full[:M2]
                K.gemm(dy2.t(), sv.col, dW2, split_k=0, rowsum=g.b2)
                K.permute_last2(dW2, C, C, 9, g.conv2_w, reverse=True, accumulate=True)
                dcol = _e((M2, 9 * C), dy2.dtype, dev)
                K.gemm(dy2, w.W2p, dcol)
                K.col2im(dcol, sv.y1, dy1)
            K.conv1_bwd(sv.xs, dy1, g.W1, g.b1)
        mod.unit_ready("conv")
        return None, None, None, None


@ranged
class EmbedOutFn(torch.autograd.Function):
    """Conv2DLayer's output projection (subsampling.py:47-48) + RelativePositionalEncoding's
    x*sqrt(d) and dropout (positional_encoding.py:68-75).  The c-major flatten of the
    reference is folded into a column permutation of embed.out.weight (repacked working
    copy).  Its backward returns dy2 = (dx W_out) * relu'(y2) with the zero tail rows and
    reports the data-parallel unit ``<embed>.out`` before the convolutions' backward runs."""

    @staticmethod
    def forward(ctx, y2_full, anchor, mod, env):
        B, Tx, Fd = env.embed_in_shape
        w = mod.weights()
        C, d = w.C, w.d
        T1, F1 = (Tx - 3) // 2 + 1, (Fd - 3) // 2 + 1
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        dev = y2_full.device
        xl = _e((B * T2, d), F32, dev)
        y2f = y2_full[:B * T2 * F2].view(B * T2, F2 * C)
        K.linear(y2f, w.Woutp, xl, bias=w.bout)
        x0 = _e((B * T2, d), F32, dev)
        # relative PE: x * sqrt(d) (positional_encoding.py:68-75); absolute (use_rel False):
        # x * sqrt(d) + pe[t] (:49-56); dropout either way
        K.pe_fwd(xl, B * T2, T2, d, getattr(env, "abs_pe", None), math.sqrt(d), x0, env.p_pos, env.seed + 1)
        ctx.sv = SimpleNamespace(y2_full=y2_full, dims=(B, T2, F2, C))
        ctx.mod, ctx.env = mod, env
        return x0

    @staticmethod
    def backward(ctx, dx0):
        sv, mod, env = ctx.sv, ctx.mod, ctx.env
        B, T2, F2, C = sv.dims
        w, g = mod.weights(), mod.grads()
        adt, dev = env.adt, dx0.device
        d = w.d
        M, M2 = B * T2, B * T2 * F2
        gb = _e((M, d), adt, dev)
        K.branch_grad(dx0.contiguous(), gb, math.sqrt(d), env.p_pos, env.seed + 1)
        y2f = sv.y2_full[:M2].view(M, F2 * C)
        dWo = _e((d, F2 * C), F32, dev)
        K.gemm(gb.t(), y2f, dWo, split_k=0, rowsum=g.bout)
        K.permute_last2(dWo, d, C, F2, g.out_w, reverse=True, accumulate=True)
        mod.unit_ready("out")
        # dy2 with its zero tail rows (the implicit GEMMs' K padding / out-of-range taps): one
        # buffer kept per subsampling module, its tail zeroed once when it is allocated (it is
        # produced here and consumed by EmbedConvFn.backward right after, in the same backward)
        key = (tuple(sv.y2_full.shape), adt, dev)
        if getattr(mod, "_dy2_key", None) != key:
            mod._dy2_buf = torch.zeros(sv.y2_full.shape, dtype=adt, device=dev)
            mod._dy2_key = key
        dy2_full = mod._dy2_buf
        K.gemm(gb, w.Woutp, dy2_full[:M2].view(M, F2 * C), aux=y2f, aux_act=ACT_RELU)
        return dy2_full, None, None, None


class EmbedFn:
    """The subsampling node (Conv2DLayer, subsampling.py:42-48, + the positional encoding's
    scale and dropout) as two autograd nodes, EmbedConvFn -> EmbedOutFn, so a segmented
    backward can launch the output projection's gradient bucket before the convolutions'
    backward runs (``cut``: the model's segment cut between them)."""

    @staticmethod
    def apply(xs, anchor, mod, env, cut=None):
        env.embed_in_shape = tuple(xs.shape)
        y2 = EmbedConvFn.apply(xs, mod.conv_anchor(), mod, env)
        if cut is not None:
            y2 = cut(y2)
        return EmbedOutFn.apply(y2, anchor, mod, env)


def enc_attn_forward(ln, pos, w, env, x_in, p_att, s_att, p_res, s_res, p=None, post=None):
    """An encoder layer's self-attention sub-block: relative-position attention
    (attention.py:120-154) when the layer has a positional projection, else the plain
    multi-head attention (:61-71) over the same key-padding / chunk mask (use_rel False)."""
    if w.Wpos is not None:
        return relmha_forward(ln, pos, w, env, x_in, p_att, s_att, p_res, s_res, p=p, post=post)
    if post is not None:
        post.y1 = None  # plain attention: the following norm runs on its own
    return mha_forward(ln, None, w, env.B, env.T, env.T, env.H, env.mask, env.msb, env.msq, x_in, p_att, s_att,
                       p_res, s_res)


def enc_attn_backward(gb, ln, pos, sv, w, g, env, p_att, s_att, lnb):
    if w.Wpos is not None:
        return relmha_backward(gb, ln, pos, sv, w, g, env, p_att, s_att, lnb=lnb)
    dln = mha_backward(gb, ln, None, sv, w, g, env.B, env.T, env.T, env.H, env.mask, env.msb, env.msq, p_att, s_att,
                       None)
    ln_bwd_of(dln, lnb)
    return None


@ranged
class ConformerLayerFn(torch.autograd.Function):
    """RelativeEncoderLayer.forward (liteasr/nets/conformer_layer.py:130-147), pre-norm."""

    @staticmethod
    def forward(ctx, x0, pos, anchor, layer, env):
        w = layer.weights()
        s = layer.seed
        tr = env.training
        pd = env.p_drop if tr else 0.0
        pff = env.p_ff if tr else 0.0
        pat = env.p_att if tr else 0.0
        adt = env.adt
        x0 = x0.contiguous()
        # (a) macaron FFN, scale 0.5
        pre = getattr(env, "pre_ln", None)  # this layer's first norm, computed by the previous layer
        prev = None  # the previous layer's final norm, when its forward chained into ours
        if pre is not None and pre[0] == id(layer) and pre[1] == x0.data_ptr():
            ln_a, ma, ra, prev = pre[2:]
            env.pre_ln = None
        else:
            ln_a, _, ma, ra = ln_forward(x0, w.ln_a.g, w.ln_a.b, adt)
        # every residual projection runs the following norm in its epilogue when the row
        # kernel takes the shape (res_proj); ln_forward covers the rest
        pb_ = PostLN(g=w.ln_b.g, b=w.ln_b.b, f32=False, nxt=None)
        x1, za, ha = ffn_forward(ln_a, w.ffm.W1, w.ffm.b1, w.ffm.W2, w.ffm.b2, w.act, pff,
                                 _seed(s, 1), x0, 0.5, pd, _seed(s, 2), post=pb_)
        # (b) relative-position MHSA
        if pb_.y1 is not None:
            ln_b, mb, rb = pb_.y1, pb_.m1, pb_.r1
        else:
            ln_b, _, mb, rb = ln_forward(x1, w.ln_b.g, w.ln_b.b, adt)
        pp = getattr(env, "pos_proj", None)
        pc_ = PostLN(g=w.ln_c.g, b=w.ln_c.b, f32=False, nxt=None)
        x2, svb = enc_attn_forward(ln_b, pos, w.att, env, x1, pat, _seed(s, 3), pd, _seed(s, 4),
                                   p=pp.get(id(layer)) if pp else None, post=pc_)
        # (c) convolution module
        if pc_.y1 is not None:
            ln_c, mc, rc = pc_.y1, pc_.m1, pc_.r1
        else:
            ln_c, _, mc, rc = ln_forward(x2, w.ln_c.g, w.ln_c.b, adt)
        pd_ = PostLN(g=w.ln_d.g, b=w.ln_d.b, f32=False, nxt=None)
        x3, svc = conv_forward(ln_c, w.conv, env, x2, pd, _seed(s, 5), tr, post=pd_)
        # (d) FFN, scale 0.5
        if pd_.y1 is not None:
            ln_d, md, rd = pd_.y1, pd_.m1, pd_.r1
        else:
            ln_d, _, md, rd = ln_forward(x3, w.ln_d.g, w.ln_d.b, adt)
        # final LN -> next layer's residual stream (fp32); with the next layer's first norm
        # chained when the encoder loop names it (env.next_ln): in fc2's epilogue, or in one
        # lasr_layernorm2_fwd launch
        nxt = getattr(env, "next_ln", None)
        chain = FUSED_LN2 and nxt is not None and adt == torch.bfloat16
        pf_ = PostLN(g=w.ln_f.g, b=w.ln_f.b, f32=True, nxt=(nxt[1], nxt[2]) if chain else None)
        x4, zd, hd = ffn_forward(ln_d, w.ff.W1, w.ff.b1, w.ff.W2, w.ff.b2, w.act, pff,
                                 _seed(s, 6), x3, 0.5, pd, _seed(s, 7), post=pf_)
        if pf_.y1 is not None:
            x5, mf, rf = pf_.y1, pf_.m1, pf_.r1
            if chain:
                env.pre_ln = (id(nxt[0]), x5.data_ptr(), pf_.y2, pf_.m2, pf_.r2,
                              SimpleNamespace(layer=layer, x4=x4, mf=mf, rf=rf))
        else:
            x5 = _e(x4.shape, F32, x4.device)
            mf = _e(x4.shape[0], F32, x4.device)
            rf = _e(x4.shape[0], F32, x4.device)
            if chain:
                z = _e(x4.shape, adt, x4.device)
                m2 = _e(x4.shape[0], F32, x4.device)
                r2 = _e(x4.shape[0], F32, x4.device)
                K.layernorm2_fwd(x4, w.ln_f.g, w.ln_f.b, nxt[1], nxt[2], LN_EPS, x5, mf, rf, z, m2, r2)
                env.pre_ln = (id(nxt[0]), x5.data_ptr(), z, m2, r2, SimpleNamespace(layer=layer, x4=x4, mf=mf, rf=rf))
            else:
                K.layernorm_fwd(x4, w.ln_f.g, w.ln_f.b, LN_EPS, x5, mf, rf)
        if torch.is_grad_enabled() or anchor.requires_grad:
            ctx.sv = SimpleNamespace(x=(x0, x1, x2, x3, x4), ln=(ln_a, ln_b, ln_c, ln_d),
                                     st=((ma, ra), (mb, rb), (mc, rc), (md, rd), (mf, rf)),
                                     za=za, ha=ha, zd=zd, hd=hd, svb=svb, svc=svc, pos=pos,
                                     p=(pd, pff, pat), prev=prev)
        ctx.layer, ctx.env = layer, env
        return x5

    @staticmethod
    def backward(ctx, dx5):
        sv, layer, env = ctx.sv, ctx.layer, ctx.env
        w, g = layer.weights(), layer.grads()
        s = layer.seed
        pd, pff, pat = sv.p
        x0, x1, x2, x3, x4 = sv.x
        ln_a, ln_b, ln_c, ln_d = sv.ln
        (ma, ra), (mb, rb), (mc, rc), (md, rd), (mf, rf) = sv.st
        dev, adt = dx5.device, env.adt
        M, d = x4.shape
        dx5 = dx5.contiguous()
        # parameter-gradient reductions of the whole layer finish in one launch at the end (or,
        # held, with the layers below it in the same backward segment)
        rx = getattr(env, "bwd_chain", None)
        with K.deferred_reductions(hold=_red_hold(env, layer), on_done=layer.on_grads_ready):
            if rx is not None and rx[0] == id(layer):
                # the next layer ran this final norm's backward with its own first norm's
                # (LN2_BWD_CHAIN): dx5 is already dx4, and gb came with it
                # (this layer's output has one consumer, the next layer -- directly or through a
                # backward-segment cut, which may hand over a copy -- so dx5 holds exactly the
                # dx4 values that layer produced)
                env.bwd_chain = None
                if rx[1] != (tuple(dx5.shape), dx5.dtype):
                    raise RuntimeError("ConformerLayerFn: the chained final-norm gradient did not arrive as produced")
                dx4, gb = dx5, rx[2]
            else:
                # final LN; emits the (d)-branch gradient 0.5*drop(dx4)
                dx4 = _e((M, d), F32, dev)
                gb = _e((M, d), adt, dev)
                K.layernorm_bwd(x4, dx5, w.ln_f.g, mf, rf, dx4, g.ln_f.g, g.ln_f.b, gb=gb, bscale=0.5,
                                bp=pd, bseed=_seed(s, 7))
            # each sub-block's input-gradient GEMM runs its norm's backward in its epilogue
            # (dx_ln); the branch-gradient buffers are fresh: grouped dW GEMMs read them at the
            # end of the node
            dx3 = _e((M, d), F32, dev)
            gb3 = _e((M, d), adt, dev)
            ffn_backward(gb, ln_d, sv.zd, sv.hd, w.ff.W1, w.ff.W2, g.ff.W1, g.ff.b1, g.ff.W2, g.ff.b2,
                         w.act, pff, _seed(s, 6),
                         lnb=LnBwd(x=x3, g=w.ln_d.g, mean=md, rstd=rd, dx=dx3, dgamma=g.ln_d.g, dbeta=g.ln_d.b,
                                   dres=dx4, gb=gb3, bscale=1.0, bp=pd, bseed=_seed(s, 5)))
            dx2 = _e((M, d), F32, dev)
            gb2 = _e((M, d), adt, dev)
            conv_backward(gb3, ln_c, sv.svc, w.conv, g.conv, env,
                          lnb=LnBwd(x=x2, g=w.ln_c.g, mean=mc, rstd=rc, dx=dx2, dgamma=g.ln_c.g, dbeta=g.ln_c.b,
                                    dres=dx3, gb=gb2, bscale=1.0, bp=pd, bseed=_seed(s, 4)))
            dx1 = _e((M, d), F32, dev)
            gb1 = _e((M, d), adt, dev)
            enc_attn_backward(gb2, ln_b, sv.pos, sv.svb, w.att, g.att, env, pat, _seed(s, 3),
                              lnb=LnBwd(x=x1, g=w.ln_b.g, mean=mb, rstd=rb, dx=dx1, dgamma=g.ln_b.g, dbeta=g.ln_b.b,
                                        dres=dx2, gb=gb1, bscale=0.5, bp=pd, bseed=_seed(s, 2)))
            dx0 = _e((M, d), F32, dev)
            lnb_a = LnBwd(x=x0, g=w.ln_a.g, mean=ma, rstd=ra, dx=dx0, dgamma=g.ln_a.g, dbeta=g.ln_a.b,
                          dres=dx1, gb=None, bscale=1.0, bp=0.0, bseed=0)
            pv = sv.prev if LN2_BWD_CHAIN else None
            if pv is not None:
                # the previous layer's final norm on dx0 in the same launch: it receives dx4 / gb
                pw, pgr = pv.layer.weights(), pv.layer.grads()
                dx4p, gbp = _e((M, d), F32, dev), _e((M, d), adt, dev)
                lnb_a.chain = LnBwd(x=pv.x4, g=pw.ln_f.g, mean=pv.mf, rstd=pv.rf, dx=dx4p, dgamma=pgr.ln_f.g,
                                    dbeta=pgr.ln_f.b, dres=None, gb=gbp, bscale=0.5, bp=pd,
                                    bseed=_seed(pv.layer.seed, 7))
            ffn_backward(gb1, ln_a, sv.za, sv.ha, w.ffm.W1, w.ffm.W2, g.ffm.W1, g.ffm.b1, g.ffm.W2, g.ffm.b2,
                         w.act, pff, _seed(s, 1), lnb=lnb_a)
            if pv is not None:
                env.bwd_chain = (id(pv.layer), (tuple(dx4p.shape), dx4p.dtype), gbp)
                dx0 = dx4p
        ctx.sv = None
        return dx0, None, None, None, None


@ranged
class TransformerLayerFn(torch.autograd.Function):
    """Transformer encoder layer (enc_arch "transformer"; liteasr/nets/transformer_layer.py:
    EncoderLayer.forward :64-76 / RelativeEncoderLayer.forward :119-136), pre-norm:
    x1 = x0 + drop(MHA(LN_b(x0))), x2 = x1 + drop(FFN(LN_d(x1))) -- no macaron half-step,
    no convolution module, no final norm (the encoder's after_norm follows the stack)."""

    @staticmethod
    def forward(ctx, x0, pos, anchor, layer, env):
        w = layer.weights()
        s = layer.seed
        tr = env.training
        pd = env.p_drop if tr else 0.0
        pff = env.p_ff if tr else 0.0
        pat = env.p_att if tr else 0.0
        adt = env.adt
        x0 = x0.contiguous()
        ln_b, _, mb, rb = ln_forward(x0, w.ln_b.g, w.ln_b.b, adt)
        pp = getattr(env, "pos_proj", None)
        pd_ = PostLN(g=w.ln_d.g, b=w.ln_d.b, f32=False, nxt=None)
        x1, svb = enc_attn_forward(ln_b, pos, w.att, env, x0, pat, _seed(s, 3), pd, _seed(s, 4),
                                   p=pp.get(id(layer)) if pp else None, post=pd_)
        if pd_.y1 is not None:
            ln_d, md, rd = pd_.y1, pd_.m1, pd_.r1
        else:
            ln_d, _, md, rd = ln_forward(x1, w.ln_d.g, w.ln_d.b, adt)
        x2, zd, hd = ffn_forward(ln_d, w.ff.W1, w.ff.b1, w.ff.W2, w.ff.b2, w.act, pff, _seed(s, 6), x1, 1.0, pd,
                                 _seed(s, 7))
        if torch.is_grad_enabled() or anchor.requires_grad:
            ctx.sv = SimpleNamespace(x=(x0, x1), ln=(ln_b, ln_d), st=((mb, rb), (md, rd)), zd=zd, hd=hd, svb=svb,
                                     pos=pos, p=(pd, pff, pat))
        ctx.layer, ctx.env = layer, env
        return x2

    @staticmethod
    def backward(ctx, dx2):
        sv, layer, env = ctx.sv, ctx.layer, ctx.env
        w, g = layer.weights(), layer.grads()
        s = layer.seed
        pd, pff, pat = sv.p
        x0, x1 = sv.x
        ln_b, ln_d = sv.ln
        (mb, rb), (md, rd) = sv.st
        dev, adt = dx2.device, env.adt
        M, d = x1.shape
        dx2 = dx2.contiguous()
        with K.deferred_reductions(hold=_red_hold(env, layer), on_done=layer.on_grads_ready):
            gb = _e((M, d), adt, dev)
            K.branch_grad(dx2, gb, 1.0, pd, _seed(s, 7))
            dx1 = _e((M, d), F32, dev)
            gb1 = _e((M, d), adt, dev)
            ffn_backward(gb, ln_d, sv.zd, sv.hd, w.ff.W1, w.ff.W2, g.ff.W1, g.ff.b1, g.ff.W2, g.ff.b2, w.act, pff,
                         _seed(s, 6),
                         lnb=LnBwd(x=x1, g=w.ln_d.g, mean=md, rstd=rd, dx=dx1, dgamma=g.ln_d.g, dbeta=g.ln_d.b,
                                   dres=dx2, gb=gb1, bscale=1.0, bp=pd, bseed=_seed(s, 4)))
            dx0 = _e((M, d), F32, dev)
            enc_attn_backward(gb1, ln_b, sv.pos, sv.svb, w.att, g.att, env, pat, _seed(s, 3),
                              lnb=LnBwd(x=x0, g=w.ln_b.g, mean=mb, rstd=rb, dx=dx0, dgamma=g.ln_b.g, dbeta=g.ln_b.b,
                                        dres=dx1, gb=None, bscale=1.0, bp=0.0, bseed=0))
        ctx.sv = None
        return dx0, None, None, None, None


def _rows2d(g, rows):
    """(…, V) logits gradient -> [rows, V] view with unit column stride (padded row stride
    kept); anything else is made contiguous."""
    g2 = g.reshape(rows, g.shape[-1])
    return g2 if g2.stride(1) == 1 else g2.contiguous()


def decoder_layers_fwd(dec, wd, y, h, B, L1, T, masks, p, adt, seed_shift=0):
    """Decoder layers + after_norm + linear_out (transformer_decoder.py:84-93,
    transformer_layer.py:179-221; also ParallelDecoder, parallel_decoder.py:54-66) on the
    fp32 input rows y [B*L1, d]; memory h [B*T, d] (compute dtype).  masks = (self mask,
    its batch stride, its query stride (0: key padding), memory key mask); p = dropout
    rates (residual, ffn, self-attn, src-attn).  Returns (h_attn [B*L1, V] padded rows,
    saved state for decoder_layers_bwd)."""
    smask, smsb, smsq, mmask = masks
    pd, pff, pat, pca = p
    R = B * L1
    layers_sv = []
    # every layer's source attention projects the same memory: its keys / values for all
    # layers are one GEMM against the cross-layer [n_layer * 2d, d] matrix (decoder_kv_groups)
    kvm = _e((B * T, len(wd.layers) * 2 * wd.d), adt, y.device)
    K.linear(h, wd.kv_all.W, kvm, bias=wd.kv_all.b)
    def post_ln(ln):  # the norm after a residual projection, in its launch (res_proj)
        return PostLN(g=ln.g, b=ln.b, f32=False, nxt=None) if DEC_ROW_LN else None

    def ln_after(x, post, ln):  # post's outputs, or the norm as its own launch
        if post is not None and post.y1 is not None:
            return post.y1, post.m1, post.r1
        l_, _, m_, r_ = ln_forward(x, ln.g, ln.b, adt)
        return l_, m_, r_

    nxt = None  # (l1, m1, r1) of the next layer, formed in this layer's fc2 launch
    for i, lw in enumerate(wd.layers):
        s = dec.dec_layers[i].seed + seed_shift
        if nxt is None:
            l1, _, m1, r1 = ln_forward(y, lw.ln1.g, lw.ln1.b, adt)
        else:
            l1, m1, r1 = nxt
        p2 = post_ln(lw.ln2)
        y1, sa = mha_forward(l1, None, lw.sa, B, L1, L1, wd.H, smask, smsb, smsq, y, pat, _seed(s, 1), pd,
                             _seed(s, 2), post=p2)
        l2, m2, r2 = ln_after(y1, p2, lw.ln2)
        p3 = post_ln(lw.ln3)
        y2, ca = mha_forward(l2, h, lw.ca, B, L1, T, wd.H, mmask, T, 0, y1, pca, _seed(s, 3), pd, _seed(s, 4),
                             kv=kvm[:, 2 * wd.d * i: 2 * wd.d * (i + 1)], post=p3)
        l3, m3, r3 = ln_after(y2, p3, lw.ln3)
        # the next norm (the next layer's first, or after_norm) after the FFN's residual add
        ln_n = wd.layers[i + 1].ln1 if i + 1 < len(wd.layers) else wd.ln_f
        p4 = PostLN(g=ln_n.g, b=ln_n.b, f32=False, nxt=None)
        y3, z, hh = ffn_forward(l3, lw.ff.W1, lw.ff.b1, lw.ff.W2, lw.ff.b2, ACT_RELU, pff, _seed(s, 5), y2, 1.0, pd,
                                _seed(s, 6), post=p4)
        nxt = ln_after(y3, p4, ln_n)
        layers_sv.append(SimpleNamespace(y=(y, y1, y2), ln=(l1, l2, l3), st=((m1, r1), (m2, r2), (m3, r3)), sa=sa,
                                         ca=ca, z=z, hh=hh))
        y = y3
    if nxt is None:
        yf, _, mf, rf = ln_forward(y, wd.ln_f.g, wd.ln_f.b, adt)
    else:
        yf, mf, rf = nxt
    h_attn = K.padded_rows(R, wd.Wout.shape[0], adt, y.device)
    K.linear(yf, wd.Wout, h_attn, bias=wd.bout)
    return h_attn, SimpleNamespace(layers=layers_sv, yL=y, yf=yf, mf=mf, rf=rf, p=p, masks=masks,
                                   seed_shift=seed_shift)


def decoder_layers_bwd(g_attn, sv, dec, wd, gd, h, B, L1, T, dh, adt):
    """Backward of decoder_layers_fwd: parameter gradients into gd, the memory gradient
    accumulated into dh [B*T, d] fp32; returns the gradient of the input rows (fp32)."""
    smask, smsb, smsq, mmask = sv.masks
    pd, pff, pat, pca = sv.p
    dev = g_attn.device
    R, d = B * L1, wd.d
    K.gemm(g_attn.t(), sv.yf, gd.Wout, beta=1.0, split_k=0, rowsum=gd.bout)
    dyf = _e((R, d), adt, dev)
    K.gemm(g_attn, wd.Wout, dyf)
    dy = _e((R, d), F32, dev)
    nl = len(wd.layers)
    # the FFN branch gradient of each layer (its residual dropout's backward, seed 6 of the
    # layer) comes out of the LayerNorm backward that produces the layer's output gradient:
    # the final norm's for the top layer, the next layer's first norm's below (no separate
    # branch_grad launch; same product per element)
    ffn_seed = lambda i: _seed(dec.dec_layers[i].seed + sv.seed_shift, 6)  # noqa: E731
    fused_gb = DEC_GB_IN_LN
    gb_next = _e((R, d), adt, dev) if fused_gb else None
    K.layernorm_bwd(sv.yL, dyf, wd.ln_f.g, sv.mf, sv.rf, dy, gd.ln_f.g, gd.ln_f.b, gb=gb_next, bscale=1.0, bp=pd,
                    bseed=ffn_seed(nl - 1))
    dkvm = _e((B * T, nl * 2 * d), adt, dev)  # the batched memory K/V's gradient
    for i in range(nl - 1, -1, -1):
        lw, lg, ls = wd.layers[i], gd.layers[i], sv.layers[i]
        s = dec.dec_layers[i].seed + sv.seed_shift
        y0, y1, y2 = ls.y
        l1, l2, l3 = ls.ln
        (m1, r1), (m2, r2), (m3, r3) = ls.st
        # fresh gb per branch: the grouped dW GEMMs read it at the end of the node
        gb = gb_next
        if not fused_gb:  # the separate branch-gradient launch (kept for the bit-identity test)
            gb = _e((R, d), adt, dev)
            K.branch_grad(dy, gb, 1.0, pd, ffn_seed(i))
        dy2 = _e((R, d), F32, dev)
        gb3 = _e((R, d), adt, dev)
        lnb3 = LnBwd(x=y2, g=lw.ln3.g, mean=m3, rstd=r3, dx=dy2, dgamma=lg.ln3.g, dbeta=lg.ln3.b, dres=dy, gb=gb3,
                     bscale=1.0, bp=pd, bseed=_seed(s, 4))
        dln = ffn_backward(gb, l3, ls.z, ls.hh, lw.ff.W1, lw.ff.W2, lg.ff.W1, lg.ff.b1, lg.ff.W2, lg.ff.b2,
                           ACT_RELU, pff, _seed(s, 5), lnb=lnb3)
        if dln is not None:
            ln_bwd_of(dln, lnb3)
        gb = gb3
        # the norms in front of the two attentions run in their input-gradient GEMMs (dx_ln)
        dy1 = _e((R, d), F32, dev)
        gb1 = _e((R, d), adt, dev)
        lnb2 = LnBwd(x=y1, g=lw.ln2.g, mean=m2, rstd=r2, dx=dy1, dgamma=lg.ln2.g, dbeta=lg.ln2.b, dres=dy2,
                     gb=gb1, bscale=1.0, bp=pd, bseed=_seed(s, 2))
        dln = mha_backward(gb, l2, h, ls.ca, lw.ca, lg.ca, B, L1, T, wd.H, mmask, T, 0, pca, _seed(s, 3), dh,
                           dkv=dkvm[:, 2 * d * i: 2 * d * (i + 1)], lnb=lnb2 if DEC_ROW_LN else None)
        if dln is not None:
            ln_bwd_of(dln, lnb2)
        dy0 = _e((R, d), F32, dev)
        gb_next = _e((R, d), adt, dev) if i > 0 and fused_gb else None
        lnb1 = LnBwd(x=y0, g=lw.ln1.g, mean=m1, rstd=r1, dx=dy0, dgamma=lg.ln1.g, dbeta=lg.ln1.b, dres=dy1,
                     gb=gb_next, bscale=1.0, bp=pd if gb_next is not None else 0.0,
                     bseed=ffn_seed(i - 1) if gb_next is not None else 0)
        dln = mha_backward(gb1, l1, None, ls.sa, lw.sa, lg.sa, B, L1, L1, wd.H, smask, smsb, smsq, pat,
                           _seed(s, 1), None, lnb=lnb1 if DEC_ROW_LN else None)
        if dln is not None:
            ln_bwd_of(dln, lnb1)
        dy = dy0
    K.gemm(dkvm.t(), h, gd.kv_all.W, beta=1.0, split_k=0, rowsum=gd.kv_all.b, group=True)
    K.gemm(dkvm, wd.kv_all.W, dh, beta=1.0)
    return dy


@ranged
class HeadsFn(torch.autograd.Function):
    """Encoder after_norm (transformer_encoder.py:126), CTC head with its always-on
    input dropout (ctc.py:28-30) and the full Transformer decoder
    (transformer_decoder.py:70-93, transformer_layer.py:179-221)."""

    @staticmethod
    def forward(ctx, x, anchor, model, env):
        dev, adt = x.device, env.adt
        enc, dec = model.encoder, model.decoder
        B, T, L1 = env.B, env.T, env.L1
        M, R = B * T, B * L1
        tr = env.training
        x = x.contiguous()
        we = enc.after_norm_weights()
        h, hd, me, re = ln_forward(x, we.g, we.b, adt, y2=True, p2=env.p_ctc, seed2=env.seed + 2)
        wc = model.ctc.weights()
        V = wc.W.shape[0]
        h_ctc = K.padded_rows(M, V, adt, dev)  # [M, V] view of [M, roundup8(V)]
        K.linear(hd, wc.W, h_ctc, bias=wc.b)
        # ---- decoder
        wd = dec.weights()
        d = wd.d
        p = (env.p_dec if tr else 0.0, env.p_dec_ff if tr else 0.0, env.p_dec_att if tr else 0.0,
             env.p_dec_src_att if tr else 0.0)
        y = _e((R, d), F32, dev)
        K.embed_pe_fwd(env.ys_in, L1, wd.E, wd.pe, math.sqrt(d), y, env.p_dec_pos if tr else 0.0,
                       env.seed + 3)
        masks = (env.dec_mask, env.dec_mask.stride(0), env.dec_mask.stride(1), env.mask_k)
        h_attn, dsv = decoder_layers_fwd(dec, wd, y, h, B, L1, T, masks, p, adt)
        ctx.sv = SimpleNamespace(x=x, h=h, hd=hd, me=me, re=re, dec=dsv)
        ctx.model, ctx.env = model, env
        return h_attn, h_ctc

    @staticmethod
    def backward(ctx, g_attn, g_ctc):
        sv, model, env = ctx.sv, ctx.model, ctx.env
        enc, dec = model.encoder, model.decoder
        dev, adt = sv.x.device, env.adt
        B, T, L1 = env.B, env.T, env.L1
        M, R = B * T, B * L1
        d_enc = sv.x.shape[1]
        dh = _e((M, d_enc), F32, dev)  # accumulated gradient of h_enc
        # ---- CTC head
        wc, gc = model.ctc.weights(), model.ctc.grads()
        if g_ctc is not None:
            g_ctc = _rows2d(g_ctc, M)
            K.gemm(g_ctc.t(), sv.hd, gc.W, beta=1.0, split_k=0, rowsum=gc.b)
            dhd = _e((M, d_enc), F32, dev)
            K.gemm(g_ctc, wc.W, dhd)
            K.branch_grad(dhd, dh, 1.0, env.p_ctc, env.seed + 2)
        else:
            K.fill(dh, 0.0)
        model.ctc.on_grads_ready()
        # ---- decoder
        wd, gd = dec.weights(), dec.grads()
        d = wd.d
        with K.deferred_reductions():  # decoder parameter-gradient reductions: one launch
            if g_attn is not None:
                dy = decoder_layers_bwd(_rows2d(g_attn, R), sv.dec, dec, wd, gd, sv.h, B, L1, T, dh, adt)
                K.embed_bwd(env.ys_in, dy, math.sqrt(d), gd.E, env.p_dec_pos if env.training else 0.0,
                            env.seed + 3)
        dec.on_grads_ready()
        # ---- encoder after_norm
        we, ge = enc.after_norm_weights(), enc.after_norm_grads()
        dx = _e((M, d_enc), F32, dev)
        K.layernorm_bwd(sv.x, dh, we.g, sv.me, sv.re, dx, ge.g, ge.b)
        enc.after_norm_ready()
        ctx.sv = None
        return dx, None, None, None


@ranged
class ParaformerHeadsFn(torch.autograd.Function):
    """Everything of Paraformer.forward after the conformer layers (liteasr/models/
    paraformer.py:97-113): encoder after_norm, the CIF predictor (predictor.py:24-118:
    conv1d k3 + ReLU and linear + sigmoid as GEMMs, the integrate-and-fire scan in
    csrc/cif.hip), target embedding + PE, the no-grad first decoder pass and its argmax,
    the glancing sampler (host ``random.sample`` per utterance, the reference's RNG calls),
    the mix and the second decoder pass.  Returns (hs_attn [B*L, V], sum_alpha [B])."""

    @staticmethod
    def forward(ctx, x, anchor, model, env, ys, ylens_host, rng):
        dev, adt = x.device, env.adt
        enc, dec, pr = model.encoder, model.decoder, model.predictor
        B, T = env.B, env.T
        L = ys.shape[1]
        M, R = B * T, B * L
        tr = env.training
        x = x.contiguous()
        d = x.shape[1]
        # ---- encoder after_norm: fp32 for the predictor, compute dtype for the decoder memory
        we = enc.after_norm_weights()
        h32, me, re = _e((M, d), F32, dev), _e(M, F32, dev), _e(M, F32, dev)
        K.layernorm_fwd(x, we.g, we.b, LN_EPS, h32, me, re)
        hm = h32.to(adt)
        # ---- predictor: conv1d(k3, pad 1) as one GEMM over overlapping row windows of a
        # zero-padded copy, then the scalar head
        wp = pr.weights()
        xpad = torch.zeros(B, T + 2, d, dtype=adt, device=dev)
        xpad[:, 1:T + 1] = hm.view(B, T, d)
        wc = _e((d, 3 * d), adt, dev)
        K.permute_last2(wp.Wc.reshape(d, d, 3), d, d, 3, wc)  # [out][in][tap] -> [out][tap][in]
        win = xpad.as_strided((B, T, 3 * d), ((T + 2) * d, d, 1))
        cv = _e((B, T, d), adt, dev)
        K.gemm(win, wc.t().unsqueeze(0).expand(B, 3 * d, d), cv, bias=wp.bc, act=ACT_RELU)
        z = _e((M, 1), F32, dev)
        K.gemm(cv.view(M, d), wp.Wl.t(), z, bias=wp.bl)
        # ---- CIF
        plen = env.pred_len
        ylen = env.ylen
        cs = SimpleNamespace(alpha=_e(M, F32, dev), acc=_e(M, F32, dev), fired=_e(M, torch.uint8, dev),
                             row=_e(M, torch.int32, dev), sum_alpha=_e(B, F32, dev), mae=_e(B, F32, dev),
                             out=_e((B, L, d), F32, dev))
        K.cif_fwd(z, plen, ylen, h32, B, T, L, cs)
        # ---- target embedding + PE (paraformer.py:103)
        eos = model.eos
        ys_in = ys.masked_fill(ys == model.ignore, eos).to(torch.int32).contiguous()
        emb = _e((R, d), F32, dev)
        p_pos = model.pos_dropout_rate if tr else 0.0
        K.embed_pe_fwd(ys_in, L, model.embed_weight(), model.pe.table(L), math.sqrt(d), emb, p_pos, env.seed + 5)
        # ---- first decoder pass, no grad (paraformer.py:106-109)
        wd = dec.weights()
        rates = dec.rates
        p = (rates.drop if tr else 0.0, rates.ff if tr else 0.0, rates.self_att if tr else 0.0,
             rates.src_att if tr else 0.0)
        nomask = torch.zeros(B, L, dtype=torch.uint8, device=dev)
        masks = (nomask, L, 0, env.mask_k)
        cif_rows = cs.out.view(R, d)
        hat, _ = decoder_layers_fwd(dec, wd, cif_rows, hm, B, L, T, masks, p, adt, seed_shift=8)
        _, ids, _ = K.logsoftmax_topk(hat, 1)
        # ---- glancing sampler on the host (glancing_sampler.py:16-30)
        ys_hat = ids.view(B, L).long().cpu()
        ys_in_h = ys_in.cpu().long()
        pad = torch.arange(L)[None, :] >= ylens_host[:, None]
        ys_hat = ys_hat.masked_fill(pad, eos)
        num = torch.ceil(model.sample_ratio * (ys_hat != ys_in_h).sum(-1)).long()
        rep = torch.zeros(B, L, dtype=torch.uint8)
        for b in range(B):
            rep[b, rng.sample(range(int(ylens_host[b])), int(num[b]))] = 1
        rep = rep.to(dev)
        mix = _e((R, d), F32, dev)
        K.glancing_mix(rep, emb, cif_rows, mix)
        # ---- second pass, with gradients
        hs_attn, dsv = decoder_layers_fwd(dec, wd, mix, hm, B, L, T, masks, p, adt)
        model.last_glance = SimpleNamespace(ys_hat=ys_hat, replace=rep.cpu().bool(), cif=cs)
        ctx.sv = SimpleNamespace(x=x, me=me, re=re, h32=h32, hm=hm, xpad=xpad, cv=cv, cs=cs, rep=rep,
                                 ys_in=ys_in, dec=dsv, dims=(B, T, L, d), p_pos=p_pos)
        ctx.model, ctx.env = model, env
        return hs_attn, cs.sum_alpha

    @staticmethod
    def backward(ctx, g_attn, g_sum):
        sv, model, env = ctx.sv, ctx.model, ctx.env
        enc, dec, pr = model.encoder, model.decoder, model.predictor
        B, T, L, d = sv.dims
        M, R = B * T, B * L
        dev, adt = sv.x.device, env.adt
        dh = torch.zeros(M, d, dtype=F32, device=dev)  # gradient of the after_norm output
        wd, gd = dec.weights(), dec.grads()
        with K.deferred_reductions():
            if g_attn is not None:
                dmix = decoder_layers_bwd(_rows2d(g_attn, R), sv.dec, dec, wd, gd, sv.hm, B, L, T, dh, adt)
            else:
                dmix = torch.zeros(R, d, dtype=F32, device=dev)
        dec.on_grads_ready()
        g_emb, g_cif = _e((R, d), F32, dev), _e((R, d), F32, dev)
        K.glancing_mix(sv.rep, dmix, None, g_emb, g_cif, backward=True)
        K.embed_bwd(sv.ys_in, g_emb, math.sqrt(d), model.embed_grad(), sv.p_pos, env.seed + 5)
        model.unit_ready("embed")
        # ---- CIF backward -> predictor logits / encoder output
        dz = _e(M, F32, dev)
        dh_cif = _e((B, T, d), F32, dev)
        gs = g_sum.contiguous().float() if g_sum is not None else None
        K.cif_bwd(env.pred_len, env.ylen, sv.h32, B, T, L, sv.cs, g_cif, gs, dz, dh_cif)
        # ---- predictor head and conv1d backward
        wp, gp = pr.weights(), pr.grads()
        dza = dz.to(adt).view(M, 1)
        K.gemm(dza.t(), sv.cv.view(M, d), gp.Wl, beta=1.0, rowsum=gp.bl)
        dpre = _e((M, d), adt, dev)
        K.gemm(dza, wp.Wl, dpre, aux=sv.cv.view(M, d), aux_act=ACT_RELU)
        P = torch.zeros(B, T + 2, d, dtype=adt, device=dev)
        P[:, 1:T + 1] = dpre.view(B, T, d)
        Pk = P.view(-1, d)[1:-1]
        kw = Pk.shape[0]
        win = sv.xpad.view(-1)[: (kw - 1) * d + 3 * d].as_strided((kw, 3 * d), (d, 1))
        dwc = _e((d, 3 * d), F32, dev)
        K.gemm(Pk.t(), win, dwc, split_k=0, rowsum=gp.bc)
        K.permute_last2(dwc, d, d, 3, gp.Wc.view(d, d, 3), reverse=True, accumulate=True)
        wflip = wp.Wc.reshape(d, d, 3).flip(-1).permute(1, 2, 0).reshape(d, 3 * d).to(adt)
        pwin = P.as_strided((B, T, 3 * d), ((T + 2) * d, d, 1))
        dh_pred = _e((B, T, d), F32, dev)
        K.gemm(pwin, wflip.t().unsqueeze(0).expand(B, 3 * d, d), dh_pred)
        pr.on_grads_ready()
        dh += dh_cif.view(M, d)
        dh += dh_pred.view(M, d)
        # ---- encoder after_norm
        we, ge = enc.after_norm_weights(), enc.after_norm_grads()
        dx = _e((M, d), F32, dev)
        K.layernorm_bwd(sv.x, dh, we.g, sv.me, sv.re, dx, ge.g, ge.b)
        enc.after_norm_ready()
        ctx.sv = None
        return dx, None, None, None, None, None, None


@ranged
class ParaformerLossFn(torch.autograd.Function):
    """ParaformerLoss.__call__ (liteasr/criterions/paraformer_loss.py:39-56):
    gamma * CE(hs_attn, ys; ignore -1, mean over targets) + mean |sum_alpha - ylens|."""

    @staticmethod
    def forward(ctx, hs_attn, sum_alpha, ys, ylens, count, gamma, cif):
        dev = hs_attn.device
        R, V = hs_attn.shape
        B = sum_alpha.shape[0]
        tgt = ys.reshape(-1).to(torch.int32).contiguous()
        lse, rows = _e(R, F32, dev), _e(R, F32, dev)
        K.lsm_kl_fwd(hs_attn, tgt, -1, 0.0, lse, rows)
        loss = _e(1, F32, dev)
        K.loss_combine(rows, gamma / max(count, 1), cif.mae, 1.0 / B, loss)
        ctx.sv = SimpleNamespace(ha=hs_attn, tgt=tgt, lse=lse, scale=gamma / max(count, 1), B=B,
                                 sign=torch.sign(sum_alpha.detach() - ylens.to(F32)))
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        sv = ctx.sv
        g = g.contiguous().float()
        ga = K.padded_rows(sv.ha.shape[0], sv.ha.shape[1], sv.ha.dtype, g.device)
        K.lsm_kl_bwd(sv.ha, sv.tgt, -1, 0.0, sv.lse, ga, sv.scale, gdev=g)
        gsum = sv.sign * (g / sv.B)
        ctx.sv = None
        return ga, gsum, None, None, None, None, None


@ranged
class HybridLossFn(torch.autograd.Function):
    """HybridCTCLoss.__call__ (liteasr/criterions/hybrid_ctc_attn.py:39-79):
    ctc_weight * CTC(sum)/B + (1 - ctc_weight) * smoothed-KL(sum)/B.
    Forward computes losses only; backward computes both logits gradients scaled by the
    incoming (device) gradient without a host round trip."""

    @staticmethod
    def forward(ctx, h_attn, h_ctc, prep, ctc_weight, smoothing, ignore):
        dev = h_attn.device
        B, L1 = prep.ys_in.shape
        V = h_attn.shape[-1]
        Tp = h_ctc.shape[1]
        ha = h_attn.reshape(B * L1, V)
        hc = h_ctc.reshape(B, Tp, V)
        L = prep.tgt_ctc.shape[1]
        lse_a = _e(B * L1, F32, dev)
        rows = _e(B * L1, F32, dev)
        K.lsm_kl_fwd(ha, prep.tgt, ignore, smoothing, lse_a, rows)
        S = 2 * L + 1
        lse = _e(B * Tp, F32, dev)
        lp = _e(B * Tp * (L + 1), F32, dev)
        alpha = _e(B * Tp * S, F32, dev)
        beta = _e(B * Tp * S, F32, dev)  # computed alongside alpha (one launch)
        nll = _e(B, F32, dev)
        K.ctc_fwd(hc, prep.tgt_ctc, prep.pred_len, prep.ylen, lse, lp, alpha, nll, beta=beta)
        loss = _e(1, F32, dev)
        K.loss_combine(nll, ctc_weight / B, rows, (1.0 - ctc_weight) / B, loss)
        ctx.sv = SimpleNamespace(ha=ha, hc=hc, prep=prep, lse_a=lse_a, lse=lse, lp=lp, alpha=alpha,
                                 beta=beta, nll=nll, w=ctc_weight, s=smoothing, ign=ignore, B=B,
                                 shapes=(h_attn.shape, h_ctc.shape))
        ctx.parts = (nll, rows)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        sv = ctx.sv
        g = g.contiguous().float()
        dev = g.device
        B = sv.B
        ga = K.padded_rows(sv.ha.shape[0], sv.ha.shape[1], sv.ha.dtype, dev)
        K.lsm_kl_bwd(sv.ha, sv.prep.tgt, sv.ign, sv.s, sv.lse_a, ga, (1.0 - sv.w) / B, gdev=g)
        gc = K.padded_rows(sv.hc.shape[0] * sv.hc.shape[1], sv.hc.shape[2], sv.hc.dtype, dev).view(sv.hc.shape)
        L = sv.prep.tgt_ctc.shape[1]
        K.ctc_bwd(sv.hc, sv.prep.tgt_ctc, sv.prep.pred_len, sv.prep.ylen, sv.lse, sv.lp, sv.alpha,
                  sv.nll, sv.beta, gc, sv.w / B, gdev=g, beta_ready=True)
        ctx.sv = None
        return ga.view(sv.shapes[0]), gc.view(sv.shapes[1]), None, None, None, None


@ranged
class EncoderOutFn(torch.autograd.Function):
    """Encoder after_norm (transformer_encoder.py:126) as its own autograd node, for heads
    other than U2's HeadsFn (encoder reuse, SURVEY §8 f4: Transducer / Paraformer heads
    consume `self.encoder(xs, mask)`, transducer.py:128, paraformer.py:96).  Returns the
    fp32 encoder output; backward writes the after_norm parameter gradients and hands
    dx to the conformer layers' fused backward."""

    @staticmethod
    def forward(ctx, x, anchor, model, adt):
        x = x.contiguous()
        we = model.encoder.after_norm_weights()
        rows, d = x.shape
        h = _e((rows, d), F32, x.device)
        mean = _e(rows, F32, x.device)
        rstd = _e(rows, F32, x.device)
        K.layernorm_fwd(x, we.g, we.b, LN_EPS, h, mean, rstd)
        ctx.sv = (x, mean, rstd)
        ctx.model = model
        return h

    @staticmethod
    def backward(ctx, dh):
        x, mean, rstd = ctx.sv
        enc = ctx.model.encoder
        we, ge = enc.after_norm_weights(), enc.after_norm_grads()
        dx = _e(x.shape, F32, x.device)
        K.layernorm_bwd(x, dh.float().contiguous(), we.g, mean, rstd, dx, ge.g, ge.b)
        enc.after_norm_ready()
        ctx.sv = None
        return dx, None, None, None


# ============================================================== transducer ======
def lstm_layer_fwd(X, w, B, U1, H, adt, p_out, seed):
    """One LSTMCell layer over U1 time-major steps (liteasr/nets/rnn_decoder.py:49-80):
    G = X W_ih^T + b_ih for all steps in one GEMM, then per step G[t] += h_{t-1} W_hh^T (GEMM,
    beta 1) and the cell kernel (b_hh added there).  X [U1*B, in] (compute dtype).  Returns
    (Y [U1*B, H] the output sequence after the layer's dropout, saved state)."""
    dev = X.device
    G = _e((U1, B, 4 * H), F32, dev)
    K.linear(X, w.Wih, G.view(U1 * B, 4 * H), bias=w.bih)
    hs = _e((U1 + 1, B, H), adt, dev)  # hs[0] = zero state, hs[t+1] = h_t
    K.fill(hs[0], 0.0)
    cs = _e((U1, B, H), F32, dev)
    for t in range(U1):
        if t > 0:
            K.gemm(hs[t], w.Whh.t(), G[t], beta=1.0)
        K.lstm_cell_fwd(G[t], w.bhh, cs[t - 1] if t > 0 else None, cs[t], hs[t + 1])
    Y = hs[1:].reshape(U1 * B, H)
    if p_out > 0:
        Yd = _e((U1 * B, H), adt, dev)
        K.pe_fwd(Y, U1 * B, 1, H, None, 1.0, Yd, p_out, seed)
        Y = Yd
    return Y, SimpleNamespace(X=X, G=G, hs=hs, cs=cs)


def lstm_layer_bwd(dY, sv, w, g, B, U1, H, adt, p_out, seed):
    """Backward of lstm_layer_fwd: dY [U1*B, H] fp32 gradient of the output sequence ->
    parameter gradients into g, returns dX [U1*B, in] fp32.  Per step (reversed) the cell
    kernel forms the gate gradients dG[t] and dc, and dh_{t-1} = dG[t] W_hh (GEMM); the
    weight gradients are one GEMM each over all U1*B rows (dW_hh against hs[0:U1], the
    states each step consumed)."""
    dev = dY.device
    if p_out > 0:
        dYd = _e(dY.shape, F32, dev)
        K.branch_grad(dY, dYd, 1.0, p_out, seed)
        dY = dYd
    dG = _e((U1, B, 4 * H), adt, dev)
    dh_rec = _e((B, H), F32, dev)
    dcs = [_e((B, H), F32, dev), _e((B, H), F32, dev)]
    dY3 = dY.view(U1, B, H)
    for t in range(U1 - 1, -1, -1):
        last = t == U1 - 1
        K.lstm_cell_bwd(sv.G[t], w.bhh, sv.cs[t], sv.cs[t - 1] if t > 0 else None, dY3[t],
                        None if last else dh_rec, None if last else dcs[(t + 1) & 1], dG[t],
                        dcs[t & 1] if t > 0 else None)
        if t > 0:
            K.gemm(dG[t], w.Whh, dh_rec)
    dG2 = dG.view(U1 * B, 4 * H)
    K.gemm(dG2.t(), sv.hs[:U1].reshape(U1 * B, H), g.Whh, beta=1.0, split_k=0, rowsum=g.bhh)
    K.gemm(dG2.t(), sv.X, g.Wih, beta=1.0, split_k=0, rowsum=g.bih)
    dX = _e((U1 * B, sv.X.shape[1]), F32, dev)
    K.gemm(dG2, w.Wih, dX)
    return dX


@ranged
class TransducerHeadsFn(torch.autograd.Function):
    """Everything of Transducer.forward after the conformer layers (liteasr/models/
    transducer.py:106-121,199-203): encoder after_norm, lin_enc, the prediction network
    (nets/rnn_decoder.py:69-80: embedding with padding_idx 0, LSTMCell layers, dropouts),
    lin_dec, z = tanh(enc + dec) (csrc/rnnt.hip joint_tanh_fwd), lin_jnt.  ids: the
    decoder input ys_in time-major [U1*B] int32.  Returns h_jnt as [B*T'*U1, V] rows."""

    @staticmethod
    def forward(ctx, x, anchor, model, env, ids, U1):
        dev, adt = x.device, env.adt
        enc, dec, jp = model.encoder, model.decoder, model.joint_params
        B, T = env.B, env.T
        M, R = B * T, U1 * B
        tr = env.training
        x = x.contiguous()
        we = enc.after_norm_weights()
        h, _, me, re = ln_forward(x, we.g, we.b, adt)
        wj = jp.weights()
        J = wj.We.shape[0]
        e = _e((M, J), F32, dev)
        K.linear(h, wj.We, e, bias=wj.be)
        # prediction network
        wd = dec.weights()
        p = dec.rates.drop if tr else 0.0
        emb = _e((R, dec.h_dim), adt, dev)
        K.embed_pe_fwd(ids, U1, wd.E, None, 1.0, emb, p, env.seed + 6)
        Xl, layers = emb, []
        for i, lw in enumerate(wd.layers):
            Xl, lsv = lstm_layer_fwd(Xl, lw, B, U1, dec.h_units, adt, p, env.seed + 7 + i)
            layers.append(lsv)
        d = _e((R, J), F32, dev)
        K.linear(Xl, wj.Wd, d)
        z = _e((M * U1, J), adt, dev)
        K.joint_fwd(e, d, B, T, U1, z)
        V = wj.Wj.shape[0]
        out = K.padded_rows(M * U1, V, adt, dev)
        K.linear(z, wj.Wj, out, bias=wj.bj)
        ids_bwd = ids.masked_fill(ids == 0, -1)  # padding_idx 0: no embedding gradient
        ctx.sv = SimpleNamespace(x=x, h=h, me=me, re=re, z=z, Y=Xl, layers=layers, ids=ids_bwd, dims=(B, T, U1, J),
                                 p=p)
        ctx.model, ctx.env = model, env
        return out

    @staticmethod
    def backward(ctx, g_out):
        sv, model, env = ctx.sv, ctx.model, ctx.env
        enc, dec, jp = model.encoder, model.decoder, model.joint_params
        B, T, U1, J = sv.dims
        M, R = B * T, U1 * B
        dev, adt = sv.x.device, env.adt
        wj, gj = jp.weights(), jp.grads()
        g_out = _rows2d(g_out, M * U1)
        # lin_jnt
        K.gemm(g_out.t(), sv.z, gj.Wj, beta=1.0, split_k=0, rowsum=gj.bj)
        model.unit_ready("lin_jnt")
        dz = _e((M * U1, J), adt, dev)
        K.gemm(g_out, wj.Wj, dz, aux=sv.z, aux_act=ACT_TANH)
        de, dd = _e((M, J), adt, dev), _e((R, J), adt, dev)
        K.joint_reduce(dz, B, T, U1, de, dd)
        # lin_dec and the prediction network
        K.gemm(dd.t(), sv.Y, gj.Wd, beta=1.0, split_k=0)
        model.unit_ready("lin_dec")
        dY = _e((R, dec.h_units), F32, dev)
        K.gemm(dd, wj.Wd, dY)
        wd, gd = dec.weights(), dec.grads()
        for i in range(len(wd.layers) - 1, -1, -1):
            dY = lstm_layer_bwd(dY, sv.layers[i], wd.layers[i], gd.layers[i], B, U1, dec.h_units, adt, sv.p,
                                env.seed + 7 + i)
        if sv.p > 0:
            dE = _e(dY.shape, F32, dev)
            K.branch_grad(dY, dE, 1.0, sv.p, env.seed + 6)
            dY = dE
        K.embed_bwd(sv.ids, dY, 1.0, gd.E)
        dec.on_grads_ready()
        # lin_enc
        K.gemm(de.t(), sv.h, gj.We, beta=1.0, split_k=0, rowsum=gj.be)
        model.unit_ready("lin_enc")
        dh = _e((M, sv.h.shape[1]), F32, dev)
        K.gemm(de, wj.We, dh)
        # encoder after_norm
        we, ge = enc.after_norm_weights(), enc.after_norm_grads()
        dx = _e(sv.x.shape, F32, dev)
        K.layernorm_bwd(sv.x, dh, we.g, sv.me, sv.re, dx, ge.g, ge.b)
        enc.after_norm_ready()
        ctx.sv = None
        return dx, None, None, None, None, None


@ranged
class RNNTLossFn(torch.autograd.Function):
    """RNNTLoss (liteasr/criterions/rnnt.py:53-72): batch mean of -log P(y|x) over the raw
    joint logits [B, T, U1, V] with the log-softmax fused (csrc/rnnt.hip); the backward
    writes d loss / d logits scaled by the incoming device gradient, no host sync."""

    @staticmethod
    def forward(ctx, logits, targets, ilen, tlen, blank):
        dev = logits.device
        B, T, U1, V = logits.shape
        rows = B * T * U1
        lse, lp = _e(rows, F32, dev), _e(rows * 2, F32, dev)
        alpha, beta, nll = _e(rows, F32, dev), _e(rows, F32, dev), _e(B, F32, dev)
        K.rnnt_fwd(logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll)
        loss = _e(1, F32, dev)
        K.loss_combine(nll, 1.0 / B, None, 0.0, loss)
        ctx.sv = (logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll)
        ctx.nll = nll
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll = ctx.sv
        B, T, U1, V = logits.shape
        grad = K.padded_rows(B * T * U1, V, logits.dtype, logits.device).view(B, T, U1, V)
        K.rnnt_bwd(logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll, grad, 1.0 / B,
                   gdev=g.contiguous().float())
        ctx.sv = None
        return grad, None, None, None, None


# ================================================================ inference ===
def encoder_out(x, model, adt):
    """Encoder after_norm (transformer_encoder.py:126) without the CTC dropout branch:
    x [M, d] fp32 residual stream -> h [M, d] in the compute dtype."""
    we = model.encoder.after_norm_weights()
    h, _, _, _ = ln_forward(x.contiguous(), we.g, we.b, adt)
    return h


def ctc_logits(h, model):
    """ctc_lo(h) (ctc.py:25-26, no dropout), [M, V] padded-row view."""
    wc = model.ctc.weights()
    out = K.padded_rows(h.shape[0], wc.W.shape[0], h.dtype, h.device)
    K.linear(h, wc.W, out, bias=wc.b)
    return out


def decoder_logits(model, h, ys_in, dec_mask, mem_mask, B, L1, T):
    """TransformerDecoder.forward (transformer_decoder.py:70-93) in eval mode for
    decoding: ys_in int32 [B, L1], dec_mask u8 [B, L1, L1] (1 = masked), memory h
    [B*T, d] (compute dtype), mem_mask u8 [B, T].  Returns h_attn [B*L1, V] (padded rows).
    Same kernels and order as HeadsFn.forward, without dropout and saved state."""
    wd = model.decoder.weights()
    d, adt, dev = wd.d, h.dtype, h.device
    R = B * L1
    y = _e((R, d), F32, dev)
    K.embed_pe_fwd(ys_in, L1, wd.E, wd.pe, math.sqrt(d), y, 0.0, 0)
    for lw in wd.layers:
        l1, _, _, _ = ln_forward(y, lw.ln1.g, lw.ln1.b, adt)
        y1, _ = mha_forward(l1, None, lw.sa, B, L1, L1, wd.H, dec_mask, dec_mask.stride(0), dec_mask.stride(1), y,
                            0.0, 0, 0.0, 0)
        l2, _, _, _ = ln_forward(y1, lw.ln2.g, lw.ln2.b, adt)
        y2, _ = mha_forward(l2, h, lw.ca, B, L1, T, wd.H, mem_mask, T, 0, y1, 0.0, 0, 0.0, 0)
        l3, _, _, _ = ln_forward(y2, lw.ln3.g, lw.ln3.b, adt)
        y, _, _ = ffn_forward(l3, lw.ff.W1, lw.ff.b1, lw.ff.W2, lw.ff.b2, ACT_RELU, 0.0, 0, y2, 1.0, 0.0, 0)
    yf, _, _, _ = ln_forward(y, wd.ln_f.g, wd.ln_f.b, adt)
    out = K.padded_rows(R, wd.Wout.shape[0], adt, dev)
    K.linear(yf, wd.Wout, out, bias=wd.bout)
    return out


class DecoderStepCache:
    """TransformerDecoder.forward_one_step (liteasr/nets/transformer_decoder.py:58-68,
    DecoderLayer with cache: transformer_layer.py:27-47,179-221) for the attention beam
    search (u2.py:163-216), eval mode, with a key/value cache per decoder layer: each step
    runs only the new position -- its row's projections, one-query attention over the cached
    keys, the source attention over the memory keys/values (projected ONCE per utterance:
    the memory is the same for every beam and step), the FFN and the output projection --
    instead of the whole prefix.

    Cache semantics follow the reference exactly.  Its cache (each layer's outputs for the
    earlier positions) is NOT reordered when the beam reorders its hypotheses; the first
    layer recomputes its keys from the (reordered) hypothesis embeddings, while layers >= 1
    attend to the earlier rows in the previous step's slot order.  Here: the first layer's
    key/value cache is gathered by the beam's selection each step (identical to recomputing
    it from the reordered embeddings: a row's projection does not depend on other rows);
    the caches of layers >= 1 are never permuted (tests/golden/decode_cache.npz, two
    decoder layers, pins the per-step log-probs)."""

    def __init__(self, model, mem, beam, T, max_len):
        wd = model.decoder.weights()
        self.wd, self.beam, self.T = wd, beam, T
        d, adt, dev = wd.d, mem.dtype, mem.device
        self.adt, self.dev = adt, dev
        self.kv_mem = []  # per layer [T, 2d]: linear_k / linear_v of the memory (src_attn)
        for lw in wd.layers:
            kv = _e((T, 2 * d), adt, dev)
            K.linear(mem, lw.ca.Wkv, kv, bias=lw.ca.bkv)
            self.kv_mem.append(kv)
        n = len(wd.layers)
        self.kc = [_e((beam, max_len, d), adt, dev) for _ in range(n)]
        self.vc = [_e((beam, max_len, d), adt, dev) for _ in range(n)]

    def _attend(self, q, k3, v3, Tk):
        """softmax(q k^T / sqrt(dk)) v for one query row per beam: q [beam, d] (row stride
        arbitrary), k3 / v3 [beam, >=Tk, d] views (any batch stride, 0 included)."""
        wd, beam = self.wd, self.beam
        H, d = wd.H, wd.d
        dk = d // H
        ldS = ld_scores(Tk)
        q4 = q.unflatten(1, (H, dk)).unsqueeze(2)  # (beam, H, 1, dk)
        k4 = k3[:, :Tk].unflatten(2, (H, dk)).permute(0, 2, 1, 3)  # (beam, H, Tk, dk)
        v4 = v3[:, :Tk].unflatten(2, (H, dk)).permute(0, 2, 1, 3)
        S = _e((beam, H, 1, ldS), F32, self.dev)
        K.gemm(q4, k4.transpose(-1, -2), S[..., :Tk], alpha=dk ** -0.5)
        P = _e((beam, H, 1, ldS), self.adt, self.dev)
        K.attn_softmax_fwd(S, None, beam, H, 1, Tk, ldS, None, 0, 0, P)
        ctx = _e((beam, d), self.adt, self.dev)
        K.gemm(P[..., :Tk], v4, ctx.unflatten(1, (H, dk)).unsqueeze(2))
        return ctx

    def step(self, ids, i, sel=None):
        """Log-probs' logits [beam, V] of step i (1-based: the new token sits at position
        i - 1); ids int32 [beam] = each hypothesis' last token; sel (int64 device [beam],
        optional) = the beam's selection that produced these hypotheses from the previous
        step's slots."""
        wd, beam, adt, dev = self.wd, self.beam, self.adt, self.dev
        d = wd.d
        if sel is not None and i > 1:
            for c in (self.kc[0], self.vc[0]):
                c[:, :i - 1] = c[:, :i - 1].index_select(0, sel)
        y = _e((beam, d), F32, dev)
        K.embed_pe_fwd(ids, 1, wd.E, wd.pe[i - 1:], math.sqrt(d), y, 0.0, 0)
        for j, lw in enumerate(wd.layers):
            l1, _, _, _ = ln_forward(y, lw.ln1.g, lw.ln1.b, adt)
            qkv = _e((beam, 3 * d), adt, dev)
            K.linear(l1, lw.sa.Wqkv, qkv, bias=lw.sa.bqkv)
            self.kc[j][:, i - 1] = qkv[:, d:2 * d]
            self.vc[j][:, i - 1] = qkv[:, 2 * d:]
            ctx = self._attend(qkv[:, :d], self.kc[j], self.vc[j], i)
            y1 = _e((beam, d), F32, dev)
            K.linear(ctx, lw.sa.Wo, y1, bias=lw.sa.bo, res=y, res_scale=1.0)
            l2, _, _, _ = ln_forward(y1, lw.ln2.g, lw.ln2.b, adt)
            q = _e((beam, d), adt, dev)
            K.linear(l2, lw.ca.Wq, q, bias=lw.ca.bq)
            kv = self.kv_mem[j]
            ctx2 = self._attend(q, kv[:, :d].unsqueeze(0).expand(beam, self.T, d),
                                kv[:, d:].unsqueeze(0).expand(beam, self.T, d), self.T)
            y2 = _e((beam, d), F32, dev)
            K.linear(ctx2, lw.ca.Wo, y2, bias=lw.ca.bo, res=y1, res_scale=1.0)
            l3, _, _, _ = ln_forward(y2, lw.ln3.g, lw.ln3.b, adt)
            y, _, _ = ffn_forward(l3, lw.ff.W1, lw.ff.b1, lw.ff.W2, lw.ff.b2, ACT_RELU, 0.0, 0, y2, 1.0, 0.0, 0)
        yf, _, _, _ = ln_forward(y, wd.ln_f.g, wd.ln_f.b, adt)
        out = K.padded_rows(beam, wd.Wout.shape[0], adt, dev)
        K.linear(yf, wd.Wout, out, bias=wd.bout)
        return out
