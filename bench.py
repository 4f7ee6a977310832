#!/usr/bin/env python
"""Throughput of the U2-Conformer + hybrid CTC-attention training step on MI355X.

    python bench.py [--gpus N --steps K --warmup W] [--config small|large|long|tiny]

A step = one full training iteration on one synthetic batch per rank: forward, hybrid
loss, backward, gradient all-reduce (N > 1), clip_grad_norm(5) + NaN-skip + Noam/Adam,
zero_grad -- the reference's Trainer.run body (liteasr/trainer.py:140-171) with
accum_grad = 1.  Inputs are resident on the GPU before timing starts.

Prints ONE JSON line (rank 0).  value = utterances/s over all ranks (weak scaling:
B utterances per rank per step).  Also reports, for the dominant kernel, an achieved
vs peak roofline measured live with HIP events, and the CPU baseline (the oracle
restatement, pinned to the reference by tests/test_oracle_golden.py) on a bounded
sample timed on this host.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: model widths, batch shape, hybrid weight; GFLOP/utt fwd+bwd from SURVEY §6
    "small": dict(d=256, H=4, ff=2048, enc=12, dec=6, B=32, T=1000, L=40, w=0.3, gflop=80.14, chunk=0),
    # config 4: the dynamic-chunk streaming mask (a chunk size drawn per step on the device;
    # eval / the fixed-c comparison leg use c = 16)
    "large": dict(d=512, H=16, ff=2048, enc=12, dec=6, B=32, T=1000, L=40, w=0.3, gflop=230.77, chunk=16,
                  dynamic=True),
    "long": dict(d=256, H=4, ff=2048, enc=12, dec=6, B=8, T=4000, L=150, w=1.0, gflop=364.51, chunk=0),
    "tiny": dict(d=64, H=4, ff=256, enc=2, dec=1, B=16, T=1000, L=20, w=0.3, gflop=1.74, chunk=0),
}
V = 4233
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build(cfgd, dtype, dropout, dev):
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    c = U2Config(input_dim=80, vocab_size=V, enc_dim=cfgd["d"], enc_ff_dim=cfgd["ff"], enc_attn_heads=cfgd["H"],
                 enc_layers=cfgd["enc"], dec_dim=cfgd["d"], dec_ff_dim=cfgd["ff"], dec_attn_heads=cfgd["H"],
                 dec_layers=cfgd["dec"], dropout_rate=dropout, compute_dtype=dtype, chunk_size=cfgd["chunk"],
                 dynamic_chunk=bool(cfgd.get("dynamic", False)))
    resolve_self(c)
    # my_U2.yaml: attention dropout 0, everything else model.dropout_rate
    c.enc_attn_dropout_rate = 0.0
    c.dec_self_attn_dropout_rate = 0.0
    c.dec_src_attn_dropout_rate = 0.0
    return U2(c).to(dev).train()


def synthetic(cfgd, rank, dev):
    from liteasr_amd.utils.synthetic import synthetic_batch  # SURVEY §8d input recipe

    xs, xlens, ys, ylens = synthetic_batch(cfgd["B"], cfgd["T"], cfgd["L"], V, seed=1234 + rank)
    return [t.to(dev) for t in (xs, xlens, ys, ylens)]


PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s peak


def _rows(cfgd):
    """B * T' (the encoder's GEMM rows)."""
    T1 = (cfgd["T"] - 3) // 2 + 1
    return cfgd["B"] * ((T1 - 3) // 2 + 1)


def build_key():
    """Identity of the HIP library a PMC pass measured: sha256 of libliteasr_hip.so (first
    16 hex digits).  Committed PMC byte counts are used only while the library is the same
    build, so a kernel change that keeps its template name cannot reuse stale bytes."""
    import hashlib

    path = os.path.join(ROOT, "liteasr_amd", "lib", "libliteasr_hip.so")
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def family_case(cfgd, dev):
    """The dominant kernel family of the step (profiles/r03 step summary): the GEMMs whose
    output is d = 256 columns wide, ~3.3 ms of the ~11.8 ms step.  One Conformer layer's
    twelve of them, issued through the product's own calls exactly as nets/functional.py
    issues them (same planner, tiles, epilogues and the full-row LayerNorm kernels):
      forward, fp32 residual out = res + s * dropout(X W^T + b)   (conformer_layer.py:37-78)
        fc2 of both FFNs (K = ff; 64 x 64 GEMM tiles: the row kernel is slower at K = 2048),
        linear_o and pointwise_conv2 (K = d) with the next LayerNorm in the epilogue
        (lasr_linear_res_ln: y1 = LN(out) and its row statistics written too)
      backward, input gradients dX = dY W                         (the same layers)
        fc1 of both FFNs (K = ff, bf16 out; the LayerNorm backward after it is a separate
        launch), linear_o and pointwise_conv2 (K = d, bf16 out), the fused q/k/v (K = 3d) and
        pointwise_conv1 (K = 2d) with the LayerNorm backward in the epilogue
        (lasr_linear_dx_ln_bwd: dx = dres + LN'(dY W) and the branch gradient gb written).
    Algorithmic bytes per launch: every operand the call reads, once, and every output it
    writes, once (the LayerNorm gamma/beta partial rows excluded: scratch of this design)."""
    import torch

    from liteasr_amd import kernels as K

    M, D, F = _rows(cfgd), cfgd["d"], cfgd["ff"]
    bf, f32 = torch.bfloat16, torch.float32
    g = torch.Generator(device=dev).manual_seed(7)

    def rn(*shape, dt=bf, scale=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * scale).to(dt)

    def nb(*ts):
        return float(sum(t.numel() * t.element_size() for t in ts))

    gam, bet = 1.0 + rn(D, dt=f32, scale=0.1), rn(D, dt=f32, scale=0.1)
    insts = []

    def add(name, kind, Kd, count, fn, plan, rd, wr):
        insts.append(dict(name=name, kernel=kind, M=M, N=D, K=Kd, count=count, launch=fn, plan=plan,
                          bytes=nb(*rd) + nb(*wr), flops=2.0 * M * D * Kd))

    def fwd_res(name, Kd, count):
        x, w, b, res = rn(M, Kd), rn(D, Kd, scale=Kd ** -0.5), rn(D, dt=f32, scale=0.02), rn(M, D, dt=f32)
        out = torch.empty(M, D, device=dev)
        fn = lambda: K.linear(x, w, out, bias=b, res=res, res_scale=0.5, drop_p=0.1, drop_seed=5)  # noqa: E731
        add(name, "gemm_bf16_glds_kernel", Kd, count, fn, (x, w.t(), out), (x, w, b, res), (out,))

    def fwd_res_ln(name, Kd, count):
        x, w, b, res = rn(M, Kd), rn(D, Kd, scale=Kd ** -0.5), rn(D, dt=f32, scale=0.02), rn(M, D, dt=f32)
        out, y1 = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev, dtype=bf)
        m1, r1 = torch.empty(M, device=dev), torch.empty(M, device=dev)
        if K.row_ln_ok(x, w, D):  # the product's policy (nets/functional.py res_proj)
            fn = lambda: K.linear_res_ln(x, w, out, y1, m1, r1, gam, bet, 1e-12, bias=b, res=res,  # noqa: E731
                                         drop_p=0.1, drop_seed=6)
            add(name, "row_res_ln_kernel", Kd, count, fn, None, (x, w, b, res, gam, bet), (out, y1, m1, r1))
            return

        def fn():  # the GEMM with its residual epilogue, then the LayerNorm launch
            K.linear(x, w, out, bias=b, res=res, res_scale=1.0, drop_p=0.1, drop_seed=6)
            K.layernorm_fwd(out, gam, bet, 1e-12, y1, m1, r1, None, 0.0, 0)
        add(name + " [GEMM + ln_fwd]", "gemm_bf16_glds_kernel + ln_fwd_kernel", Kd, count, fn, (x, w.t(), out),
            (x, w, b, res, gam, bet), (out, y1, m1, r1))
        insts[-1]["launches"] = 2

    def dx(name, Kd, count):
        dy, w = rn(M, Kd), rn(Kd, D, scale=Kd ** -0.5)
        out = torch.empty(M, D, device=dev, dtype=bf)
        fn = lambda: K.gemm(dy, w, out)  # noqa: E731
        add(name, "gemm_bf16_glds_kernel", Kd, count, fn, (dy, w, out), (dy, w), (out,))

    def dx_ln(name, Kd, count):
        dy, w = rn(M, Kd), rn(Kd, D, scale=Kd ** -0.5)
        x, dres = rn(M, D, dt=f32), rn(M, D, dt=f32)
        mean, rstd = rn(M, dt=f32, scale=0.1), 1.0 + rn(M, dt=f32, scale=0.1).abs()
        dxo, gb = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev, dtype=bf)
        dgam, dbet = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        if K.row_ln_ok(dy, w, D):  # the product's policy (nets/functional.py dx_ln)
            fn = lambda: K.linear_dx_ln_bwd(dy, w, x, gam, mean, rstd, dxo, dgam, dbet, dres=dres, gb=gb,  # noqa: E731
                                            bp=0.1, bseed=4)
            add(name, "row_dx_ln_bwd_kernel", Kd, count, fn, None, (dy, w, x, gam, mean, rstd, dres),
                (dxo, gb, dgam, dbet))
            return
        dln = torch.empty(M, D, device=dev, dtype=bf)

        def fn():  # the input-gradient GEMM, then the LayerNorm backward (+ its gamma/beta reduction)
            K.gemm(dy, w, dln)
            K.layernorm_bwd(x, dln, gam, mean, rstd, dxo, dgam, dbet, dres=dres, gb=gb, bp=0.1, bseed=4)
        add(name + " [GEMM + ln_bwd]", "gemm_bf16_glds_kernel + ln_bwd_kernel", Kd, count, fn, (dy, w, dln),
            (dy, w, x, gam, mean, rstd, dres), (dxo, gb, dgam, dbet))
        insts[-1]["launches"] = 3

    fwd_res("fc2 fwd (+res)", F, 2)
    fwd_res_ln("linear_o fwd (+res, +LN)", D, 1)
    fwd_res_ln("pointwise_conv2 fwd (+res, +LN)", D, 1)
    dx("fc1 dX", F, 2)
    dx("linear_o dX", D, 1)
    dx("pointwise_conv2 dX", D, 1)
    dx_ln("qkv dX (+LN bwd)", 3 * D, 1)
    dx_ln("pointwise_conv1 dX (+LN bwd)", 2 * D, 1)
    for it in insts:
        if it["plan"] is None:
            it["tile"] = f"32x{D} row, 8 waves"
            continue
        a_, b_, c_ = it["plan"]
        tm, tn, sp = K.gemm_plan(a_, b_, c_)
        it["tile"] = f"{tm}x{tn}" + (f" split {sp}" if sp > 1 else "")
    return insts


def family_roofline(cfgd, dev, iters=50):
    """Per-instance average launch time (HIP events on the launch stream, `iters` back-to-back
    launches) and the family aggregate: sum over one layer's launches of algorithmic bytes /
    sum of their times, against the 8 TB/s HBM peak (every instance's byte time exceeds its
    flop time at 2.5 PFLOP/s: bound hbm)."""
    insts = family_case(cfgd, dev)
    rows, tb, tt, tf = [], 0.0, 0.0, 0.0
    for it in insts:
        sec = _time_case(it["launch"], iters)
        bound, ach, peak, unit = _roof(it["flops"], it["bytes"], sec)
        rows.append({"name": it["name"], "kernel": it["kernel"], "shape": f"M={it['M']} N={it['N']} K={it['K']}",
                     "tile": it["tile"],
                     "per_layer": it["count"], "avg_launch_us": round(sec * 1e6, 2),
                     "algorithmic_bytes": it["bytes"], "GBps": round(it["bytes"] / sec / 1e9, 1),
                     "frac": round(it["bytes"] / sec / 1e9 / PEAK_HBM_GBS, 4), "bound": bound})
        tb += it["count"] * it["bytes"]
        tt += it["count"] * sec
        tf += it["count"] * it["flops"]
    return rows, tb, tt, tf


def roofline_case(cfgd, dev):
    """The dominant kernel family of the step (rocprof): the weight-gradient GEMMs (both
    operands M/N-contiguous, LDS transposed reads, split-K fp32 partials).  In the step they
    run grouped per backward node (lasr_gemm_dw_group, kernels.deferred_reductions); the
    representative launch is the FFN group of one Conformer layer exactly as the step issues
    it: dW1 = dZ^T LN (ff x d) and dW2 = G^T H (d x ff) of both macaron FFNs, rows = B*T',
    planned by the product (tile, 64-deep stages, K slices) and launched alone (the fixed-
    order reduction of the partials is a separate kernel, lasr_reduce_multi).
    Algorithmic bytes: each problem's bf16 operands read once + its fp32 result written
    once.  The split-K partial slabs are NOT counted: they are traffic this design adds, so
    they show up as PMC traffic above the algorithmic bytes."""
    import torch

    from liteasr_amd import _native as Nn
    from liteasr_amd import kernels as K

    T1 = (cfgd["T"] - 3) // 2 + 1
    rows = cfgd["B"] * ((T1 - 3) // 2 + 1)
    F, D = cfgd["ff"], cfgd["d"]
    probs = []
    for _ in range(2):  # ffm (macaron) and ff
        dz = torch.randn(rows, F, device=dev).bfloat16()
        ln = torch.randn(rows, D, device=dev).bfloat16()
        gb = torch.randn(rows, D, device=dev).bfloat16()
        h = torch.randn(rows, F, device=dev).bfloat16()
        probs.append((gb, h, torch.zeros(D, F, device=dev), torch.zeros(D, device=dev)))  # W2
        probs.append((dz, ln, torch.zeros(F, D, device=dev), torch.zeros(F, device=dev)))  # W1
    with K.deferred_reductions():
        for a, b, c, r in probs:
            K.gemm(a.t(), b, c, beta=1.0, split_k=0, rowsum=r, group=True)
        q = list(K._DEFER.gemms)
        # the fp32 partial buffers the queued args write into are owned by the deferred
        # reductions (segs): keep them alive with the launch, or the args point at freed memory
        parts = [sg[0] for sg in K._DEFER.segs]
        K._DEFER.gemms.clear()
        K._DEFER.segs.clear()
    assert q and all(k == q[0][0] for k, _, _ in q), "FFN weight gradients did not group"
    arr = (Nn.GemmArgs * len(q))(*[x[1] for x in q])
    wsp = {int(x[1].workspace) for x in q}
    assert wsp <= {pt.data_ptr() for pt in parts}, "a queued dW launch writes outside the kept partial buffers"
    keep = [x[2] for x in q] + [probs, parts]

    def launch():
        Nn.call("lasr_gemm_dw_group", arr, len(q), K.stream())

    launch.keep = keep
    flops = sum(2.0 * a.shape[0] * a.shape[1] * b.shape[1] for a, b, _, _ in probs)
    bytes_ = sum(2.0 * (a.numel() + b.numel()) + 4.0 * c.numel() for a, b, c, _ in probs)
    tm, tn = q[0][0]
    # the group key is the planner's family; lasr_gemm_dw_group (gemm.hip) runs the FFN-sized
    # family on 8-wave 256 x 128 tiles
    if (tm, tn) == (128, 128):
        kname = "gemm_dw_group_kernel<256, 128, 3, 1, 8>"
    else:
        S, minb = {(64, 64): (3, 3), (128, 128): (2, 2)}[(tm, tn)]
        kname = f"gemm_dw_group_kernel<{tm}, {tn}, {S}, {minb}, 4>"
    splits = sorted({-x[1].split_k for x in q})
    meta = {"kernel": kname,
            "shape": f"{len(q)} problems: 2x (M={F} N={D}) + 2x (M={D} N={F}), K={rows}, split_k={splits}",
            "build": build_key()}
    return launch, flops, bytes_, meta


def hottest_case(cfgd, dev):
    """The single hottest GEMM instance by ms/step (rocprof, profiles/r02): the FFN fc1
    forward, h = dropout(swish(LN @ W1^T + b1)) plus the gate g = swish'(u) * keep stored
    for the backward (gemm_bf16_glds_kernel<128,256,true,true,bf16,3,2,0>, 24 per step).
    Algorithmic bytes: LN and W1 read once, h and g written once (bf16)."""
    import torch

    from liteasr_amd import kernels as K
    from liteasr_amd._native import ACT_SWISH

    T1 = (cfgd["T"] - 3) // 2 + 1
    M = cfgd["B"] * ((T1 - 3) // 2 + 1)
    F, D = cfgd["ff"], cfgd["d"]
    ln = torch.randn(M, D, device=dev).bfloat16()
    w1 = (torch.randn(F, D, device=dev) * 0.05).bfloat16()
    b1 = torch.zeros(F, device=dev)
    h = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    g = torch.empty_like(h)

    def launch():
        K.linear(ln, w1, h, bias=b1, act=ACT_SWISH, zout=g, zout_mode=1, drop_p=0.1, drop_seed=11)

    flops = 2.0 * M * F * D
    bytes_ = 2.0 * (M * D + F * D) + 2 * 2.0 * M * F + 4.0 * F
    tm, tn, _, fl = K.gemm_plan(ln, w1.t(), h, flags=True, bias=b1, act=ACT_SWISH, zout=g, zout_mode=1,
                                drop_p=0.1, drop_seed=11)
    # gemm_launch.h: wide 8-wave / 4-wave 32-deep, and the compile-time epilogue it takes for this
    # call (EPI_SWISH_GATE_DROP = 1 unless LASR_EPI_SPEC=0; the wide tile has none)
    epi = 1 if not fl & 8 and os.environ.get("LASR_EPI_SPEC", "1") != "0" else 0
    inst = f"2, 1, 0, 2, 8, {epi}" if fl & 8 else f"3, 2, 0, 1, 4, {epi}"
    meta = {"kernel": f"gemm_bf16_glds_kernel<{tm}, {tn}, true, true, unsigned short, {inst}>",
            "shape": f"M={M} N={F} K={D} bias+swish+gate+dropout", "grid": [-(-F // tn), -(-M // tm), 1],
            "build": build_key()}
    return launch, flops, bytes_, meta


def attention_case(cfgd, dev):
    """The encoder's fused relative-position attention of one layer at the config's shape
    (liteasr/nets/attention.py:120-154): lasr_relattn_fwd + lasr_relattn_bwd (query-side and
    key-side flash kernels, csrc/attn_flash.hip) exactly as ConformerLayerFn issues them (bf16,
    key padding from the synthetic lengths, the chunk mask of the config).  Algorithmic flops
    per layer = 9 x 2*B*H*T'^2*d_k: forward 3 (QK^T, the positional product Qv P^T over the
    needed diagonal band, PV), backward 6 (S recomputed once: 2; dP, dQu, dK, dV: 4); the
    kernels execute 12 (the backward's two kernels each recompute S) -- the MFMA fraction is
    quoted on the algorithmic count.  Bytes: Qu, Qv, K, V, the position table, ctx and dctx
    read, ctx, dQu, dK, dV and the dBD G-space gradient written once (bound: mfma)."""
    import torch

    from liteasr_amd import kernels as K
    from liteasr_amd.utils.synthetic import synthetic_batch

    B, H, d = cfgd["B"], cfgd["H"], cfgd["d"]
    dk = d // H
    T = _rows(cfgd) // B
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(5)
    rn = lambda *sh: (torch.randn(*sh, device=dev, generator=g) * 0.5).to(bf)  # noqa: E731
    qkv, qu, qv, pos, dctx = rn(B * T, 3 * d), rn(B * T, d), rn(B * T, d), rn(T, d), rn(B * T, d)
    _, xlens, _, _ = synthetic_batch(B, cfgd["T"], cfgd["L"], V, seed=99)
    tl = (((xlens - 1) // 2 - 1) // 2).to(dev)
    pad = torch.arange(T, device=dev)[None, :] >= tl[:, None]
    if cfgd["chunk"]:
        ch = cfgd["chunk"]
        tri = (torch.arange(T, device=dev)[None, :] // ch) > (torch.arange(T, device=dev)[:, None] // ch)
        mask, msb, msq = K.pad_mask16((pad[:, None, :] | tri[None]).to(torch.uint8), B, T, T)
    else:
        mask, msb, msq = pad.to(torch.uint8).contiguous(), T, 0
    scale = dk ** -0.5
    stats = torch.empty(B * H * T * 2, device=dev)
    ctx = torch.empty(B * T, d, dtype=bf, device=dev)
    ldS = (T + 7) // 8 * 8
    Dbuf = torch.empty(B * H * T, device=dev)
    dqu = torch.empty(B * T, d, dtype=bf, device=dev)
    dbd = torch.empty(H, B, T, ldS, dtype=bf, device=dev)
    dqkv = torch.zeros(B * T, 3 * d, dtype=bf, device=dev)
    k, v = qkv[:, d:2 * d], qkv[:, 2 * d:]

    def launch():
        K.relattn_fwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx)
        K.relattn_bwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dqu, dbd, ldS,
                      dqkv[:, d:2 * d], dqkv[:, 2 * d:], dbd_head_major=True)

    unit = 2.0 * B * H * T * T * dk
    flops = 9 * unit
    bytes_ = 2.0 * (6 * B * T * d + T * d) + 2.0 * (4 * B * T * d + H * B * T * ldS)
    rm = "true" if cfgd["chunk"] else "false"
    nw = "8" if dk == 64 else "4 (fwd) / 8"
    meta = {"kernel": f"flash_fwd_kernel + flash_bwd_q_kernel + flash_bwd_kv_kernel<{dk}, {nw}, true, {rm}>",
            "match": ["flash_fwd_kernel", "flash_bwd_q_kernel", "flash_bwd_kv_kernel"],
            "shape": f"B={B} H={H} T'={T} d_k={dk}" + (f" chunk {cfgd['chunk']}" if cfgd["chunk"] else " key padding"),
            "build": build_key(), "units": {"fwd": 3, "bwd": 6, "executed": 12}}
    return launch, flops, bytes_, meta


def attention_roofline(cfgd, dev, iters=20):
    """Live HIP-event time of one layer's attention set (attention_case) and its fraction of the
    bf16 MFMA peak; the MFMA-busy counter of the same build from a committed PMC pass."""
    launch, flops, bytes_, meta = attention_case(cfgd, dev)
    sec = _time_case(launch, iters)
    out = {"kernel": meta["kernel"], "shape": meta["shape"], "bound": "mfma",
           "achieved": round(flops / sec / 1e12, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
           "frac": round(flops / sec / 1e12 / PEAK_BF16_TFLOPS, 4), "traffic": None,
           "algorithmic_flops_per_launch": flops, "algorithmic_bytes_per_launch": bytes_,
           "layer_set_us": round(sec * 1e6, 2), "flop_units": meta["units"],
           "per": "one encoder layer's attention (forward + backward launches)"}
    busy = pmc_mfma_case(meta)
    out["mfma_busy_counter"] = busy
    return out


def pmc_mfma_case(meta):
    """SQ_VALU_MFMA_BUSY_CYCLES fraction of a roofline case from a committed pass of the same build
    (profiles/*/pmc_mfma_case*.json, written by tools/pmc_mfma.py --case)."""
    import glob

    key = build_key()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_mfma_case*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("build") == key and d.get("shape") == meta["shape"]:
            return {"mfma_busy_frac": d["mfma_util"], "source": os.path.relpath(path, ROOT)}
    return None


def _time_case(launch, iters):
    """Average device time of one launch(): `iters` launches captured into one hipGraph (as the
    step runs them) and replayed between two HIP events on the launch stream.  Timing eager
    Python launches instead would measure the host's launch rate for the short kernels (a
    6 us GEMM behind ~10 us of ctypes marshalling)."""
    import torch

    for _ in range(5):  # warm-up: workspaces reach their size outside the capture
        launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # lasr_* launches go to kernels.stream() == the capture stream
        for _ in range(iters):
            launch()
    g.replay()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def _roof(flops, bytes_, sec):
    t_flop = flops / (PEAK_BF16_TFLOPS * 1e12)
    t_byte = bytes_ / (PEAK_HBM_GBS * 1e9)
    if t_byte >= t_flop:
        return "hbm", bytes_ / sec / 1e9, PEAK_HBM_GBS, "GB/s"
    return "mfma", flops / sec / 1e12, PEAK_BF16_TFLOPS, "TFLOP/s"


def _case_entry(launch, flops, bytes_, meta, iters):
    sec = _time_case(launch, iters)
    bound, ach, peak, unit = _roof(flops, bytes_, sec)
    traffic = pmc_traffic(meta)
    out = {"kernel": meta["kernel"], "shape": meta["shape"], "bound": bound, "achieved": round(ach, 2),
           "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
           "traffic": traffic["bytes_per_launch"] if traffic else None,
           "algorithmic_bytes_per_launch": bytes_, "algorithmic_flops_per_launch": flops,
           "avg_launch_us": round(sec * 1e6, 2), "achieved_tflops": round(flops / sec / 1e12, 2)}
    if traffic:
        out["traffic_source"] = traffic["source"]
    return out


def dominant_kernel_roofline(cfgd, dev, iters=50):
    """`roofline` = the dominant kernel family (family_case), measured live with HIP events
    on the stream the kernels are launched on; `traffic` = HBM bytes per layer's set of
    launches from the committed PMC passes of the same library build (pmc_traffic).
    Secondary entries: the grouped FFN weight-gradient launch (`dw_group`) and the single
    hottest GEMM instance, the FFN fc1 forward (`hottest_instance`)."""
    rows, tb, tt, tf = family_roofline(cfgd, dev, iters)
    ach = tb / tt / 1e9
    fam_meta = family_meta(cfgd)
    traffic = pmc_traffic(fam_meta)
    out = {"kernel": fam_meta["kernel"], "shape": fam_meta["shape"], "bound": "hbm", "achieved": round(ach, 2),
           "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
           "traffic": traffic["bytes_per_launch"] if traffic else None,
           "per": f"one Conformer layer's calls of the family ({sum(r['per_layer'] for r in rows)}; the GEMM + "
                  "LayerNorm pairs timed as one call); achieved = algorithmic bytes / summed launch time",
           "algorithmic_bytes_per_launch": tb, "algorithmic_flops_per_launch": tf,
           "avg_launch_us": round(tt / sum(r["per_layer"] for r in rows) * 1e6, 2),
           "layer_set_us": round(tt * 1e6, 2), "achieved_tflops": round(tf / tt / 1e12, 2),
           "instances": rows}
    if traffic:
        out["traffic_source"] = traffic["source"]
    else:
        out["traffic_note"] = f"no PMC pass for library build {build_key()}"
    out["dw_group"] = _case_entry(*roofline_case(cfgd, dev), iters)
    out["hottest_instance"] = _case_entry(*hottest_case(cfgd, dev), iters)
    return out


def family_meta(cfgd):
    from liteasr_amd import kernels as K

    M, D, F = _rows(cfgd), cfgd["d"], cfgd["ff"]
    if D <= K.ROW_LN_MAX_D:
        names = ["gemm_bf16_glds_kernel", "row_res_ln_kernel", "row_dx_ln_bwd_kernel"]
        fam = "N = d output GEMMs (64x64 tiles and the full-row LayerNorm tiles)"
    else:  # (config 4: the product runs GEMM + LayerNorm launches at d 512, kernels.ROW_LN_MAX_D)
        names = ["gemm_bf16_glds_kernel", "ln_fwd_kernel", "ln_bwd_kernel", "reduce_cols_kernel"]
        fam = "N = d output GEMMs and the LayerNorm launches beside them"
    return {"kernel": " + ".join(names[:3]), "match": names, "family": fam,
            "shape": f"one layer: 2x fc2 fwd M={M} N={D} K={F} +res, linear_o / pw2 fwd K={D} +res +LN, "
                     f"2x fc1 dX K={F}, linear_o / pw2 dX K={D}, qkv dX K={3 * D} +LN bwd, "
                     f"pw1 dX K={2 * D} +LN bwd", "build": build_key()}


def ctc_roofline(cfgd, dev, iters=20):
    """SURVEY §8(d) / BASELINE.md §3: the fused log-softmax + CTC (hybrid_ctc_attn.py:67-75)
    at the config's shape with bf16 logits, three kernels timed live: the row log-sum-exp +
    gather (lasr_ctc_fwd with alpha = NULL), the alpha / beta lattice recursion
    (lasr_ctc_lattice: serial in T', alpha and beta side by side), and the gradient
    softmax - gamma (lasr_ctc_bwd).  Algorithmic bytes = read the logits once + write the
    gradient once, 2 * B * T' * V * 2 B (bf16; BASELINE.md quotes 4 B for fp32 logits)."""
    import torch

    from liteasr_amd import _native as Nn
    from liteasr_amd import kernels as K
    from liteasr_amd.utils.synthetic import synthetic_batch

    B, L, V_ = cfgd["B"], cfgd["L"], V
    T1 = (cfgd["T"] - 3) // 2 + 1
    Tp = (T1 - 3) // 2 + 1
    xs, xlens, ys, ylens = synthetic_batch(B, cfgd["T"], L, V_, seed=99)
    ilen = (((xlens - 1) // 2 - 1) // 2).to(torch.int32).to(dev)
    tlen = ylens.to(torch.int32).to(dev)
    tgt = ys.clamp(min=0).to(torch.int32).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    logits = K.padded_rows(B * Tp, V_, torch.bfloat16, dev).view(B, Tp, V_)
    logits.copy_(torch.randn(B, Tp, V_, device=dev, generator=g))
    f32 = dict(dtype=torch.float32, device=dev)
    S = 2 * L + 1
    lse, lp = torch.empty(B * Tp, **f32), torch.empty(B * Tp * (L + 1), **f32)
    alpha, beta, nll = torch.empty(B * Tp * S, **f32), torch.empty(B * Tp * S, **f32), torch.empty(B, **f32)
    grad = K.padded_rows(B * Tp, V_, torch.bfloat16, dev).view(B, Tp, V_)

    def gather():
        K.ctc_fwd(logits, tgt, ilen, tlen, lse, lp, None, nll)

    def lattice():  # the current stream at call time (the capture stream inside _time_case)
        Nn.call("lasr_ctc_lattice", B, Tp, L, K.ptr(tgt), K.ptr(ilen), K.ptr(tlen), K.ptr(lp), K.ptr(alpha),
                K.ptr(beta), K.ptr(nll), K.stream())

    def gradk():
        K.ctc_bwd(logits, tgt, ilen, tlen, lse, lp, alpha, nll, beta, grad, 1.0 / B, beta_ready=True)

    gather()
    lattice()
    tg, tl, tr = _time_case(gather, iters), _time_case(lattice, iters), _time_case(gradk, iters)
    tot = tg + tl + tr
    byt = 2.0 * B * Tp * V_ * 2
    return {"kernels": ["ctc_lse_gather_kernel", "ctc_lattice_regs_kernel", "ctc_grad_kernel"],
            "shape": f"B={B} T'={Tp} V={V_} L={L} (S=2L+1={S}), bf16 logits",
            "gather_us": round(tg * 1e6, 2), "lattice_us": round(tl * 1e6, 2), "grad_us": round(tr * 1e6, 2),
            "total_us": round(tot * 1e6, 2), "algorithmic_bytes": byt,
            "achieved": round(byt / tot / 1e9, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(byt / tot / 1e9 / PEAK_HBM_GBS, 4),
            "alpha_beta_us_per_step": round(tl / Tp * 1e6, 4),
            "note": "frac over the three kernels; the lattice recursion is latency-bound (serial in T')"}


def pmc_traffic(meta):
    """HBM bytes per launch (per layer's set, for the family) from the committed rocprofv3 PMC
    passes (profiles/*/roofline_pmc*.json, written by tools/pmc_traffic.py: separate
    FETCH_SIZE and WRITE_SIZE passes, FETCH_SIZE doubled per the gfx950 correction), matched
    on kernel, shape AND library build (build_key); None when no pass matches this build."""
    import glob
    import json

    key = build_key()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "roofline_pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == meta["kernel"] and d.get("shape") == meta["shape"] and d.get("build") == key:
            return {"bytes_per_launch": d["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}
    return None


def pmc_mfma(cfg_name):
    """MFMA busy fraction from the committed counter pass of the same library build and config
    (profiles/*/pmc_mfma_summary*.json, tools/pmc_mfma.py over a rocprofv3
    SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE pass of an eager `bench.py --graph off` run);
    None when no pass matches this build."""
    import glob

    key = build_key()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_mfma_summary*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("build") == key and d.get("config", "small") == cfg_name:
            top = [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}
                   for t in d.get("top_kernels", [])[:6]]
            return {"mfma_busy_frac": round(d["mfma_util_all_kernels"], 4), "source": os.path.relpath(path, ROOT),
                    "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs), cycle-weighted over "
                            "the kernels of eager steps (counter mode serialises dispatches: a lower bound)",
                    "top_kernels": top}
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(cfgd_name, budget_s=25.0):
    """The oracle restatement (pinned to the reference) on this host's CPU cores: U2 of the
    same config, a bounded batch, 1 warm-up + timed steps until ~budget_s."""
    import torch

    from oracle import u2_oracle as O

    cfgd = CONFIGS[cfgd_name]
    n = len(os.sched_getaffinity(0))
    n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    torch.set_num_threads(n)
    cfg = O.default_cfg(enc_dim=cfgd["d"], enc_heads=cfgd["H"], enc_ff=cfgd["ff"], enc_layers=cfgd["enc"],
                        dec_dim=cfgd["d"], dec_heads=cfgd["H"], dec_ff=cfgd["ff"], dec_layers=cfgd["dec"],
                        vocab_size=V, dropout=0.1, ff_dropout=0.1, pos_dropout=0.1, dec_dropout=0.1,
                        dec_pos_dropout=0.1, dec_ff_dropout=0.1)
    params = O.init_params(cfg, seed=1)
    bufs = O.init_buffers(cfg)
    Bs = 2 if cfgd["T"] > 2000 else 8  # B=8 when B=32 is too slow for the budget
    batch = O.synthetic_batch(Bs, cfgd["T"], cfgd["L"], V, seed=5)
    st = None
    t0 = time.perf_counter()
    _, _, params, st, _ = O.train_step(params, bufs, batch, cfg, ctc_weight=cfgd["w"], opt_state=st,
                                       model_dim=cfgd["d"])
    warm = time.perf_counter() - t0
    steps, t0 = 0, time.perf_counter()
    while True:
        _, _, params, st, _ = O.train_step(params, bufs, batch, cfg, ctc_weight=cfgd["w"], opt_state=st,
                                           model_dim=cfgd["d"])
        steps += 1
        el = time.perf_counter() - t0
        # ~10-25 s of timed CPU work (at least 3 steps), bounded so the bench stays short
        if el + el / steps > budget_s or (steps >= 3 and el >= 12.0):
            break
    return {"value": round(Bs * steps / el, 3), "unit": "utterances/sec", "cores": n, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"oracle (torch CPU fp32) {cfgd_name} U2, B={Bs} T={cfgd['T']} L={cfgd['L']}, dropout 0.1, "
                      f"{steps} timed step(s) = {el:.1f} s after 1 warm-up ({warm:.1f} s)"}


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rank_entry(rank, world, port, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LASR_BENCH_SPAWNED="1")
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def spawn_ranks(n, argv=None, target=None):
    """`bench.py --gpus N` without a launcher: one process per GPU, as the reference's
    call_func -> mp.spawn (liteasr/distributed/utils.py:119-139).  The parent never touches
    the GPU (spawned children start fresh interpreters); each rank runs main() with
    RANK/LOCAL_RANK/WORLD_SIZE set, rendezvous on 127.0.0.1."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    argv = sys.argv[1:] if argv is None else argv
    procs = [ctx.Process(target=target or _rank_entry, args=(r, n, port, argv)) for r in range(n)]
    for p in procs:
        p.start()
    rc = 0
    for p in procs:
        p.join()
        rc = rc or (p.exitcode or 0)
    if rc:
        for p in procs:
            if p.is_alive():
                p.kill()
    return rc


def chunk_report(model, cfgd, ctr0, steps):
    """The encoder mask of the timed steps: none, a fixed chunk size, or the dynamic draw --
    its distribution and the chunk sizes the timed steps used (the device draw is a pure
    function of the step counter; the host mirror lists it without a sync per step)."""
    if cfgd.get("dynamic"):
        T = (((cfgd["T"] - 1) // 2 - 1) // 2)
        cs = [model.dynamic_chunk_size(model._seed_base + 11, ctr0 + i, T, model.chunk_max) for i in range(steps)]
        part = [c for c in cs if c < T]
        return {"mode": "dynamic", "distribution": f"per step on the device: r ~ U{{1..T'-1}} (T' = {T}); "
                f"r > T'/2 -> full context, else c = r mod {model.chunk_max} + 1 (WeNet add_optional_chunk_mask)",
                "timed_steps_full_context": len(cs) - len(part),
                "timed_steps_chunked": len(part), "timed_chunk_sizes": cs,
                "mean_chunk_of_chunked_steps": round(sum(part) / len(part), 2) if part else None}
    if cfgd["chunk"]:
        return {"mode": "fixed", "chunk": cfgd["chunk"]}
    return {"mode": "none (key padding only)"}


def fixed_chunk_leg(model, net, crit, opt, batch, cfgd, args):
    """The same model and batch with the fixed chunk (chunk_size, c = 16 at large) instead of the
    dynamic draw: a second captured step timed over the same number of steps, reported beside the
    dynamic line (the block-skipping attention kernels are cheapest at small c)."""
    import torch

    from liteasr_amd.graph_step import GraphedTrainStep

    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    model.dynamic_chunk = False
    try:
        step = GraphedTrainStep(net, crit, opt, batch, clip=5.0, warmup=2, overlap=args.overlap == "on")
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        model.dynamic_chunk = True
    return {"chunk": cfgd["chunk"], "ms_per_step": round(el / args.steps * 1e3, 3),
            "utt_per_s": round(cfgd["B"] * args.steps / el, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher's WORLD_SIZE, N > 1 spawns them")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="small", choices=sorted(CONFIGS))
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--chunk", default="config",
                    help="encoder streaming chunk mask: 'config' (large: dynamic, others: none), 'dynamic' "
                         "(a chunk size drawn per step on the device, WeNet's distribution), 'none', or a "
                         "fixed chunk size")
    ap.add_argument("--no-chunk-compare", action="store_true",
                    help="dynamic chunk: skip the second, fixed-c (chunk_size) leg timed after the main one")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--graph", default="on", choices=["on", "off"],
                    help="replay the step from hipGraphs (liteasr_amd/graph_step.py) or launch eagerly")
    ap.add_argument("--overlap", default="on", choices=["on", "off"],
                    help="N>1 graphed step: all-reduce each gradient bucket between backward segments "
                         "(on) or after the whole backward (off)")
    ap.add_argument("--comm", default="torch", choices=["torch", "native"],
                    help="gradient all-reduce path (N>1 or --force-ddp): torch.distributed over RCCL, or "
                         "the C-ABI bucketed reducer libliteasr_comm.so (lasr_reducer_*, its own RCCL "
                         "communicator and stream)")
    ap.add_argument("--single-rank-collectives", action="store_true",
                    help="--comm native at world 1: issue the 1-rank RCCL all-reduces anyway (by default "
                         "world 1 issues none: the average is the identity); measures what RCCL's kernels "
                         "cost the overlapped backward")
    ap.add_argument("--profile", action="store_true",
                    help="roctx ranges around every fused autograd node (liteasr_amd.utils.markers); "
                         "implies --graph off (ranges are host-side launch spans)")
    ap.add_argument("--force-ddp", action="store_true",
                    help="wrap in the DDP reducer even at N=1 (world-1 RCCL group; profiling the overlap)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-only", type=int, default=0, metavar="N",
                    help="only launch the roofline kernel N times (for rocprofv3 --pmc passes)")
    ap.add_argument("--roofline-case", default="family", choices=["family", "dw", "hot", "attn"],
                    help="--roofline-only: the dominant kernel family (one layer's set), the grouped "
                         "weight-gradient launch (dw) or the hottest instance (hot)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    if args.profile:
        from liteasr_amd.utils import markers

        markers.enable()
        args.graph = "off"
    if args.roofline_only:
        torch.cuda.set_device(0)
        if args.roofline_case == "family":
            cfgd = CONFIGS[args.config]
            insts = family_case(cfgd, torch.device("cuda", 0))
            meta = family_meta(cfgd)
            bytes_ = sum(it["count"] * it["bytes"] for it in insts)
            flops = sum(it["count"] * it["flops"] for it in insts)
            meta["dispatches_per_launch"] = sum(it["count"] * it.get("launches", 1) for it in insts)

            def launch():
                for it in insts:
                    for _ in range(it["count"]):
                        it["launch"]()
        else:
            case = {"dw": roofline_case, "hot": hottest_case, "attn": attention_case}[args.roofline_case]
            launch, flops, bytes_, meta = case(CONFIGS[args.config], torch.device("cuda", 0))
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        # (timed on the current stream, which these cases launch on: a quick A/B figure, eager
        # launches included; the PMC passes read the counters of the same launches)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(args.roofline_only):
            launch()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1e3 / max(args.roofline_only, 1)
        print(json.dumps({**meta, "launches": args.roofline_only + 3, "algorithmic_bytes_per_launch": bytes_,
                          "algorithmic_flops_per_launch": flops, "us_per_launch_eager": round(us, 2)}), flush=True)
        return

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    args.gpus = args.gpus or world
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_ddp = world > 1 or args.force_ddp
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    elif use_ddp:  # world-1 RCCL group: exercises the bucketed/overlapped path on one GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cfgd = dict(CONFIGS[args.config])
    if args.chunk == "dynamic":
        cfgd["dynamic"] = True
        cfgd["chunk"] = cfgd["chunk"] or 16
    elif args.chunk == "none":
        cfgd["dynamic"], cfgd["chunk"] = False, 0
    elif args.chunk != "config":
        cfgd["dynamic"], cfgd["chunk"] = False, int(args.chunk)

    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.optims.noam import Noam, NoamConfig

    torch.manual_seed(42)
    model = build(cfgd, args.dtype, args.dropout, dev)
    net = model
    if use_ddp:
        from liteasr_amd.distributed.ddp import DistributedDataParallel

        net = DistributedDataParallel(model, comm=args.comm)
        if args.single_rank_collectives and net.reducer.native is not None:
            net.reducer.native.set_single_rank_collectives(True)
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=V, smoothing=0.1, ctc_weight=cfgd["w"]))
    opt = Noam(model.parameters(), NoamConfig(model_dim=cfgd["d"]))
    batch = synthetic(cfgd, rank, dev)

    if args.graph == "on":
        from liteasr_amd.graph_step import GraphedTrainStep

        step = GraphedTrainStep(net, crit, opt, batch, clip=5.0, warmup=2, overlap=args.overlap == "on")
    else:
        def step():
            loss = crit(net, *batch)
            loss.backward()
            opt.clip_and_step(5.0)
            opt.zero_grad()
            return loss

    if args.graph == "on" and use_ddp:
        step.enable_timing()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if use_ddp:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step HIP events on the stream the step runs on (no host sync inside the loop): the
    # median step beside the wall-clock mean the contract's ms_per_step reports
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    ctr0 = int(model._drop_ctr.item())  # the first timed step's counter (dynamic chunk draws)
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        loss = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if use_ddp:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    med = per_step[len(per_step) // 2] if args.steps % 2 else 0.5 * (per_step[len(per_step) // 2 - 1] +
                                                                     per_step[len(per_step) // 2])
    if world > 1:
        t = torch.tensor([med], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        med = t.item()
    final_loss = loss.item()
    launcher = "bench.py spawn" if os.environ.get("LASR_BENCH_SPAWNED") else (
        "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "env")
    st = opt.device_state()
    utt = world * cfgd["B"] * args.steps / el
    if rank == 0:
        out = {
            "metric": "utterances/sec (U2-Conformer+CTC, 80-d fbank T≈1000) at 1/2/4/8 MI355X",
            "value": round(utt, 2), "unit": "utterances/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "ms_per_step_median": round(med, 3),
            "ms_per_step_events_min_max": [round(per_step[0], 3), round(per_step[-1], 3)],
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (SURVEY §8d: N(0,1) 80-d fbank, xlens~U[0.95T,T], random token ids), random-init weights",
            "config": {"workload": f"U2-Conformer-{args.config} hybrid CTC-attention training step "
                                    f"(fwd+loss+bwd+allreduce+clip+Noam/Adam)",
                       "model": f"U2 enc {cfgd['enc']}x conformer d{cfgd['d']} H{cfgd['H']} ff{cfgd['ff']}, "
                                f"dec {cfgd['dec']}x, V {V}", "global_batch": world * cfgd["B"],
                       "per_gpu_batch": cfgd["B"], "seq_len": cfgd["T"], "label_len": cfgd["L"],
                       "ctc_weight": cfgd["w"], "dropout": args.dropout,
                       "chunk_size": chunk_report(model, cfgd, ctr0, args.steps),
                       "parallelism": f"dp{world}", "launch": "hipgraph" if args.graph == "on" else "eager",
                       "ranks_seen": dist.get_world_size() if dist.is_initialized() else world,
                       "rank_launcher": launcher,
                       "allreduce": None if not use_ddp else
                       {"backend": dist.get_backend(), "comm": args.comm, "buckets": len(net.reducer.buckets),
                        "single_rank_collectives": bool(args.single_rank_collectives and args.comm == "native"),
                        "bucket_mb_each": [round((hi - lo) * 4 / 1e6, 2) for lo, hi in net.reducer.native_spans()],
                        "bucket_mb": 25, "overlap": args.overlap == "on" and args.graph == "on" or args.graph == "off",
                        "segments": len(step.segs) if args.graph == "on" and step.segs else None,
                        "timeline_last_step": step.overlap_report() if args.graph == "on" else None}},
            "step_tflops_per_gpu": round(cfgd["gflop"] * utt / world / 1e3, 2),
            "step_mfma_frac": round(cfgd["gflop"] * utt / world / 1e3 / PEAK_BF16_TFLOPS, 4),
            "final_loss": round(final_loss, 4), "optimizer_state": st,
        }
        if args.graph == "on":  # launches per step: the node counts of the replayed graphs
            out["graph_nodes_per_step"] = step.graph_nodes()
        if args.profile:
            out["config"]["profile"] = "roctx ranges per fused node (eager)"
        out["mfma_counter"] = pmc_mfma(args.config)
        if not args.no_roofline:
            fam = dominant_kernel_roofline(cfgd, dev)
            att = attention_roofline(cfgd, dev)
            # `roofline` = the config's dominant family by time per step (12 encoder layers each:
            # the family's layer set vs the layer's attention); the other one rides along
            if att["layer_set_us"] > fam["layer_set_us"]:
                out["roofline"] = att
                out["roofline"]["gemm_family"] = fam
            else:
                out["roofline"] = fam
                out["roofline"]["attention"] = att
            out["ctc"] = ctc_roofline(cfgd, dev)
        if cfgd.get("dynamic") and args.graph == "on" and not args.no_chunk_compare:
            del step
            out["config"]["chunk_size"]["fixed_chunk_leg"] = fixed_chunk_leg(model, net, crit, opt, batch, cfgd,
                                                                             args)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.config)
        print(json.dumps(out), flush=True)
    if use_ddp:
        net.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
