"""End-to-end parity: liteasr_amd U2 + HybridCTCLoss (+ fused Noam/Adam) on the GPU vs the
CPU oracle (oracle/u2_oracle.py, pinned to the reference by test_oracle_golden.py).

Tolerances (stated):
  fp32 build  loss rel 1e-5; logits / grads / updated params 2e-4 of each tensor's max-abs
  bf16 build  (oracle fed the same bf16-representable weights and features)
              loss rel 5e-3; logits 2e-2; grads 5e-2 of each tensor's max-abs and cosine
              >= 0.999, except the ReLU-gated weights (decoder FFN fc1, subsampling convs:
              a pre-activation within bf16 rounding of 0 takes the other branch than in
              fp64 and moves a whole output row of a dW summed over few rows -- the
              decoder's is B*(L+1) ~ 26 rows): 0.35 of max-abs and cosine >= 0.998.
              Measured worst (tools/bf16_errs.py): non-gated 3.9e-2, gated 0.29.
Bookkeeping (targets, lengths, masks) is bit-exact (checked in test_kernels_gpu.py)."""

import math
import sys
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import u2_oracle as O  # noqa: E402


def build(cfg_o, dtype, chunk=0, dropout=0.0):
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    c = U2Config(input_dim=cfg_o["input_dim"], vocab_size=cfg_o["vocab_size"], enc_dim=cfg_o["enc_dim"],
                 enc_ff_dim=cfg_o["enc_ff"], enc_attn_heads=cfg_o["enc_heads"], enc_layers=cfg_o["enc_layers"],
                 dec_dim=cfg_o["dec_dim"], dec_ff_dim=cfg_o["dec_ff"], dec_attn_heads=cfg_o["dec_heads"],
                 dec_layers=cfg_o["dec_layers"], dropout_rate=dropout, compute_dtype=dtype, chunk_size=chunk,
                 enc_arch=cfg_o.get("enc_arch", "conformer"), use_rel=cfg_o.get("use_rel", True),
                 activation=cfg_o.get("activation", "swish"))
    resolve_self(c)
    return U2(c)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)


def grad_errs(g, go):
    """Per-tensor error relative to max(|ref|max, 1e-3 * largest grad of the model):
    some gradients are analytically zero (e.g. linear_k.bias: softmax is invariant to a
    per-row constant), so their reference is ~1e-18 and a pure relative error is noise."""
    floor = 1e-3 * max(v.abs().max().item() for v in go.values())
    out = {}
    for k in go:
        a, b = g[k].double().cpu(), go[k].double().cpu()
        out[k] = (a - b).abs().max().item() / max(b.abs().max().item(), floor)
    return out, floor


def cos(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def run_case(cfg_o, B, T, L, dtype, chunk=0, ctc_weight=0.3, seed=0, training=True, round_bf16=False,
             emulate=False, feed_dec_gates=False):
    """One training step of liteasr_amd on the GPU against the oracle on the same seeded
    weights and batch.  emulate=True: the oracle is oracle/u2_bf16.py (float64 with the bf16
    build's roundings) instead of the plain fp64 oracle; weights and features are then
    bf16-representable on both sides.  feed_dec_gates=True (fp64 oracle): the decoder FFNs'
    ReLU branches the GPU build took (its stored gates) drive the oracle's ReLUs, and the
    oracle's own pre-activations are returned to check every branch difference (``dec_pre``)."""
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.optims.noam import Noam, NoamConfig

    params = O.init_params(cfg_o, seed=seed + 11)
    buffers = O.init_buffers(cfg_o)
    batch = O.synthetic_batch(B, T, L, cfg_o["vocab_size"], seed=seed)
    if round_bf16 or emulate:  # both sides see the same bf16-representable weights and features
        params = {k: (v.bfloat16().float() if v.is_floating_point() else v) for k, v in params.items()}
        batch = (batch[0].bfloat16().float(),) + tuple(batch[1:])
    p64 = {k: v.double() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in buffers.items()}
    xs, xlens, ys, ylens = batch
    # liteasr_amd on the GPU (first: its decoder gates may feed the oracle)
    model = build(cfg_o, dtype, chunk)
    missing, unexpected = model.load_state_dict({**params, **buffers}, strict=False)
    assert not unexpected and all(k.endswith(".pe.pe") for k in missing), (missing, unexpected)
    model = model.cuda().train(training)
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=cfg_o["vocab_size"], smoothing=0.1, ctc_weight=ctc_weight))
    opt = Noam(model.parameters(), NoamConfig(model_dim=cfg_o["enc_dim"]))
    opt.zero_grad()
    dev = "cuda"
    xs_d, xl_d, ys_d, yl_d = xs.to(dev), xlens.to(dev), ys.to(dev), ylens.to(dev)
    rec = {}

    class _Once(torch.nn.Module):  # one forward: BN running stats update exactly once
        def forward(self, *a):
            rec["out"] = model(*a)
            return rec["out"]

        @property
        def last_prep(self):
            return model.last_prep

    loss = crit(_Once(), xs_d, xl_d, ys_d, yl_d)
    h_attn, h_ctc = rec["out"]
    gates = None
    if feed_dec_gates:  # the heads node's saved decoder state (HeadsFn ctx), before backward frees it
        L1 = h_attn.shape[1]  # (B, L+1, V): a view of the heads node's padded rows
        node = h_attn.grad_fn
        while not hasattr(node, "sv"):
            node = node.next_functions[0][0]
        gates = [lay.z.double().cpu().view(B, L1, -1) for lay in node.sv.dec.layers]
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    opt.clip_and_step(5.0)
    st = opt.device_state()
    torch.cuda.synchronize()
    # the oracle on the same weights and batch
    new_o = norm_o = None
    dec_pre = [] if feed_dec_gates else None
    if emulate:
        from oracle import u2_bf16 as E

        loss_o, _, _, grads_o, ha_o, hc_o = E.loss_and_grads(p64, b64, (xs.double(), xlens, ys, ylens), cfg_o,
                                                             ctc_weight=ctc_weight, smoothing=0.1, chunk=chunk,
                                                             training=training)
    else:
        with torch.no_grad():
            ha_o, hc_o, _, _ = O.u2_forward(xs.double(), xlens, ys, ylens, p64, cfg_o,
                                            {k: v.clone() for k, v in b64.items()}, training, chunk, dec_gates=gates)
        loss_o, grads_o, new_o, _, norm_o = O.train_step(p64, b64, (xs.double(), xlens, ys, ylens), cfg_o,
                                                           ctc_weight=ctc_weight, smoothing=0.1, clip=5.0,
                                                           model_dim=cfg_o["enc_dim"], chunk=chunk, training=training,
                                                           dec_gates=gates, dec_pre=dec_pre)
    return dict(loss=(loss.item(), loss_o.item()), h_attn=(h_attn, ha_o), h_ctc=(h_ctc, hc_o),
                grads=(grads, grads_o), params=(dict(model.named_parameters()), new_o),
                bn=(dict(model.named_buffers()), b64), norm=(st["grad_norm"], norm_o), st=st,
                dec_gates=gates, dec_pre=dec_pre)


TINY = O.default_cfg(enc_dim=64, enc_heads=4, enc_ff=256, enc_layers=2, dec_dim=64, dec_heads=4, dec_ff=256,
                     dec_layers=1, vocab_size=30)
SMALL = O.default_cfg(enc_layers=2, dec_layers=1)  # small-model widths (d 256, ff 2048, V 4233), 2+1 layers


@pytest.mark.parametrize("cfg,B,T,L", [(TINY, 3, 130, 8), (SMALL, 2, 210, 12)])
def test_parity_fp32(cfg, B, T, L):
    r = run_case(cfg, B, T, L, "fp32")
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 1e-5 * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < 2e-4
    assert rel(*r["h_ctc"]) < 2e-4
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    # Subsampling conv grads sit behind two ReLUs over ~5e5 units: a pre-activation within
    # fp32 rounding of 0 can take the other branch than in the fp64 oracle and moves one
    # output channel's weight grad (observed: 1 channel of 256, 7.6e-3).  Allow 2e-2 there.
    kink = {k for k in errs if k.startswith("encoder.embed.conv.")}
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    assert worst[0] < 2e-4, worst
    assert max(errs[k] for k in kink) < 2e-2, {k: errs[k] for k in kink}
    assert abs(r["norm"][0] - r["norm"][1]) <= 1e-4 * r["norm"][1]
    p, po = r["params"]
    worst = max((rel(p[k].detach(), po[k]), k) for k in po)
    assert worst[0] < 2e-4, worst
    # Noam step 1: lr = d^-0.5 * warmup^-1.5 (the update itself is below fp32 resolution of
    # the weights at step 1; the Adam arithmetic is pinned by test_kernels_gpu.py::test_adam_noam_clip)
    assert abs(r["st"]["lr"] - O.noam_lr(1, cfg["enc_dim"])) <= 1e-6 * O.noam_lr(1, cfg["enc_dim"])
    assert r["st"]["step"] == 1 and not r["st"]["skipped"]
    bufs, bo = r["bn"]
    for k, v in bo.items():
        if v.is_floating_point():
            assert rel(bufs[k], v) < 1e-4, k
        else:
            assert int(bufs[k]) == int(v), k


def relu_gated(k):
    return k.startswith("encoder.embed.conv.") or (k.startswith("decoder.") and ".feed_forward.fc1." in k)


def _check_bf16(r):
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 5e-3 * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < 2e-2
    assert rel(*r["h_ctc"]) < 2e-2
    g, go = r["grads"]
    errs, floor = grad_errs(g, go)
    for k in go:
        gated = relu_gated(k)
        if go[k].abs().max().item() > floor:
            c = cos(g[k], go[k])
            assert c >= (0.998 if gated else 0.999), (k, c)
        assert errs[k] < (0.35 if gated else 5e-2), (k, errs[k])


@pytest.mark.parametrize("cfg,B,T,L", [(TINY, 3, 130, 8), (SMALL, 2, 210, 12)])
def test_parity_bf16(cfg, B, T, L):
    _check_bf16(run_case(cfg, B, T, L, "bf16", round_bf16=True))


# ---- the whole bf16 model against the bf16-emulating oracle (oracle/u2_bf16.py).  Through
# 12 + 6 layers the bf16 build is chaotic at the 1e-3 level (every fp32-vs-fp64 difference
# flips a few bf16 roundings per layer and the flips compound), so the emulating oracle
# tightens these whole-model bars only a little over the fp64 one (DESIGN.md §2 measures
# both); the tight bar (1e-2 of max for every tensor, ReLU-gated included) is held per node
# at the same shapes in tests/test_nodes_gpu.py.  Whole-model bars: every gradient 0.15 of
# its max, logits 5e-2, loss 2e-3 relative.  The ReLU-gated decoder FFN fc1 weight is a sum
# over only B*(L+1) rows (22 here), so one pre-activation that an fp32-vs-fp64 difference
# puts on the other side of 0 moves a whole row of it: 0.25 there (measured worst 0.159 at
# d 512 / chunk 16, 0.090 at config 2; the node tests hold it to 1e-2 with the kernel's own
# gate).  Exactly-zero gradients (linear_k.bias, depthwise_conv.bias: rounding noise only)
# against 1e-2 of the largest.
EMU_GRAD, EMU_GRAD_GATED, EMU_LOGIT, EMU_LOSS = 0.15, 0.25, 5e-2, 2e-3
NOISE = ("linear_k.bias", "depthwise_conv.bias")


def emu_errors(r):
    """(loss rel, h_attn, h_ctc, worst (err, name) over the gradients) of an emulate=True case."""
    lg, lo = r["loss"]
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    gmax = max(v.abs().max().item() for v in go.values())
    for k in errs:
        if k.endswith(NOISE):
            errs[k] = (g[k].double().cpu() - go[k].double().cpu()).abs().max().item() / (1e-2 * gmax)
    gated = max(((v, k) for k, v in errs.items() if relu_gated(k)), default=(0.0, None))
    worst = max((v, k) for k, v in errs.items() if not relu_gated(k))
    return (abs(lg - lo) / abs(lo), rel(*r["h_attn"]), rel(*r["h_ctc"]), worst, gated)


def _check_emulated(r):
    loss, ha, hc, worst, gated = emu_errors(r)
    print(f"emulated: loss {loss:.3e} h_attn {ha:.3e} h_ctc {hc:.3e} worst grad {worst[0]:.4f} ({worst[1]}) "
          f"ReLU-gated {gated[0]:.4f} ({gated[1]})")
    assert loss <= EMU_LOSS, r["loss"]
    assert ha < EMU_LOGIT and hc < EMU_LOGIT, (ha, hc)
    assert worst[0] < EMU_GRAD, worst
    assert gated[0] < EMU_GRAD_GATED, gated


@pytest.mark.parametrize("cfg,B,T,L", [(TINY, 3, 130, 8), (SMALL, 2, 210, 12)])
def test_parity_bf16_emulated(cfg, B, T, L):
    _check_emulated(run_case(cfg, B, T, L, "bf16", emulate=True))


# d_k 32 with the streaming chunk mask (config 4's attention shape) through the fused kernels
LARGE_HEADS = O.default_cfg(enc_dim=128, enc_heads=4, enc_ff=256, enc_layers=2, dec_dim=128, dec_heads=4,
                            dec_ff=256, dec_layers=1, vocab_size=30)


def test_parity_bf16_dk32_chunk_mask():
    _check_bf16(run_case(LARGE_HEADS, 2, 150, 6, "bf16", chunk=8, round_bf16=True))


# config 4's layer shape at model level: d 512, 16 heads (d_k 32), ff 2048, V 4233, chunk 16
LARGE = O.default_cfg(enc_dim=512, enc_heads=16, enc_ff=2048, enc_layers=2, dec_dim=512, dec_heads=16, dec_ff=2048,
                      dec_layers=1, vocab_size=4233)
# full depth (12 encoder / 6 decoder layers) at reduced width
DEEP = O.default_cfg(enc_dim=128, enc_heads=4, enc_ff=256, enc_layers=12, dec_dim=128, dec_heads=4, dec_ff=256,
                     dec_layers=6, vocab_size=64)


def _check_dec_gates(r, max_flips=8):
    """The GPU build's stored decoder ReLU gates (which drove the oracle's ReLUs) against the
    oracle's own relu'(u): every branch difference must lie within the worst-case error of an
    fp32 dot product at that element, |u| <= K 2^-23 (|x| |W|^T + |b|) (the oracle's bound,
    oracle/u2_oracle.py ffn), and at most ``max_flips`` elements per layer may differ -- a real
    decoder-FFN error that moves pre-activations across 0 fails either bar."""
    nflip = 0
    assert len(r["dec_pre"]) == len(r["dec_gates"])  # train_step's pass, one per decoder layer
    for i, (gate, (u, bound)) in enumerate(zip(r["dec_gates"], r["dec_pre"])):
        u, bound = u.view_as(gate), bound.view_as(gate)
        flip = (gate > 0) != (u > 0)
        n = int(flip.sum())
        nflip += n
        assert n <= max_flips, (i, n)
        if n:
            assert (u[flip].abs() <= bound[flip]).all(), (i, (u[flip].abs() / bound[flip]).max().item())
    print(f"decoder ReLU branches that differ from the fp64 oracle's: {nflip} (each within its fp32 dot-product bound)")


def _check_fp32(r, tol, loss_tol=1e-5):
    lg, lo = r["loss"]
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    kink = {k for k in errs if k.startswith("encoder.embed.conv.")}  # see test_parity_fp32
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    print(f"fp32 parity: loss rel {abs(lg - lo) / abs(lo):.2e}, logits {rel(*r['h_attn']):.2e} / "
          f"{rel(*r['h_ctc']):.2e}, worst grad {worst[0]:.2e} ({worst[1]})")
    assert abs(lg - lo) <= loss_tol * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < tol and rel(*r["h_ctc"]) < tol
    assert worst[0] < tol, worst
    assert max(errs[k] for k in kink) < 2e-2, {k: errs[k] for k in kink}


def test_parity_large_width_chunk_fp32():
    """d 512 / 16 heads / ff 2048 / V 4233 with the streaming chunk mask (stage 16), fp32
    build vs the fp64 oracle.  5e-4: chunk-masked rows carry more cancellation (see
    test_parity_chunk_mask_fp32)."""
    _check_fp32(run_case(LARGE, 2, 200, 10, "fp32", chunk=16), 5e-4)


def test_parity_large_width_chunk_bf16():
    """Config 4's shape (d 512, 16 heads, chunk 16) in the bf16 build (fused d_k 32 attention)."""
    _check_bf16(run_case(LARGE, 2, 200, 10, "bf16", chunk=16, round_bf16=True))


def test_parity_large_width_chunk_bf16_emulated():
    """Config 4's layer shape (d 512, 16 heads, d_k 32, chunk 16) in the bf16 build against
    the bf16-emulating oracle."""
    _check_emulated(run_case(LARGE, 2, 200, 10, "bf16", chunk=16, emulate=True))


# BASELINE config 2's whole model (12 encoder / 6 decoder layers, d 256, ff 2048, V 4233) at
# its real utterance length T 1000 (T' 249), two utterances
CONFIG2 = O.default_cfg()


def test_parity_config2_full_model_fp32():
    """liteasr/models/u2.py:116-159 -> criterions/hybrid_ctc_attn.py:39-79 at config 2's
    full shape, fp32 build vs the fp64 oracle: loss 1e-5 relative, logits and every gradient
    1e-3 of max (measured worst 5.0e-4: the last layer's positional-projection weight, a
    K = T' = 249 sum with cancellation behind 12 fp32 layers; the subsampling convs'
    ReLU-kink bar as in test_parity_fp32).  This case first exposed the fp32 build's
    split-K rowsum scratch overwriting the weight-gradient partials (K >= 512)."""
    _check_fp32(run_case(CONFIG2, 2, 1000, 40, "fp32"), 1e-3)


def test_parity_config2_full_model_bf16_emulated():
    """Config 2's full model in the default bf16 build (fused attention, bf16 GEMMs, the
    kernels the bench times) against the bf16-emulating oracle."""
    _check_emulated(run_case(CONFIG2, 2, 1000, 40, "bf16", emulate=True))


# BASELINE config 4's per-rank workload at its real size: U2-Conformer-large, 12 encoder / 6
# decoder layers, d 512, 16 heads (d_k 32), ff 2048, V 4233, dynamic-chunk streaming mask at
# chunk 16, T 1000 (T' 249), two utterances
CONFIG4 = O.default_cfg(enc_dim=512, enc_heads=16, enc_ff=2048, enc_layers=12, dec_dim=512, dec_heads=16,
                        dec_ff=2048, dec_layers=6, vocab_size=4233)


@pytest.mark.parametrize("L", [10, 40])
def test_prep_with_chunk_mask_keeps_every_other_output(L):
    """The streaming chunk mask is a second bookkeeping pass: every other output (decoder mask
    with its 16-B padded rows, targets, lengths, key mask) must be what the chunk-free pass
    gives (round 4: the chunk pass wrote the decoder mask in the unpadded layout over the
    padded view)."""
    B, T = 3, 400
    xs, xlens, ys, ylens = O.synthetic_batch(B, T, L, TINY["vocab_size"], seed=5)
    preps = []
    for chunk in (0, 16):
        m = build(TINY, "bf16", chunk).cuda()
        preps.append(m._prep(xs.cuda(), xlens.cuda(), ys.cuda(), ylens.cuda()))
    a, b = preps
    for k in ("ys_in", "tgt", "tgt_ctc", "dec_mask", "enc_mask", "pred_len", "ylen"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert a.dec_mask.stride(1) % 16 == 0
    assert a.chunk_mask is None and b.chunk_mask is not None and b.chunk_mask.stride(1) % 16 == 0


def test_parity_config4_full_model_fp32():
    """liteasr/nets/transformer_encoder.py:107-127 with the chunk mask of liteasr/utils/mask.py:
    30-90 and the 16-head relative attention of liteasr/nets/attention.py:120-154, full depth
    and length, fp32 build vs the fp64 oracle: loss 1e-5 relative, logits and every gradient
    1e-3 of max, the decoder FFNs included; the ReLU-kink bar (2e-2) only for the subsampling
    convs as in test_parity_fp32.  The decoder's ReLU branches the GPU build took (its stored
    gates) drive the oracle's (transformer_layer.py:161-221 via feed_forward.py:18-19), and every
    branch that differs from the oracle's own relu'(u) must sit at |u| <= 2e-3 of the layer's
    largest pre-activation: a decoder fc1 row sums only B*(L+1) = 82 rows, so one pre-activation
    within fp32 rounding of 0 taking the other side moved decoder layer 4's fc1 weight gradient
    by 1.32e-2 of max in round 4.  This case caught the round-4 padded decoder mask being
    overwritten by the chunk-mask preparation (decoder logits 9.9e-2 of max)."""
    r = run_case(CONFIG4, 2, 1000, 40, "fp32", chunk=16, feed_dec_gates=True)
    _check_dec_gates(r)
    _check_fp32(r, 1e-3)


def test_parity_config4_full_model_fp32_unfed_gates():
    """Cross-check of the gate feeding above: the same case with the oracle's own ReLU branches
    (nothing fed from the GPU). Every tensor but the decoder FFNs' ReLU-gated ones and the norms in
    front of them holds 1e-3; those hold the ReLU-kink bar of the subsampling convs (2e-2): one
    pre-activation within fp32
    rounding of 0 on the other side moves a whole row of a B*(L+1) = 82-row weight gradient
    (round 4 measured 1.32e-2 at decoder layer 4's fc1 weight)."""
    r = run_case(CONFIG4, 2, 1000, 40, "fp32", chunk=16)
    lg, lo = r["loss"]
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    # the ReLU-gated fc1 tensors and the decoder norm in front of each FFN: its gamma / beta
    # gradient sums the same B*(L+1) rows of dln that a flipped kink moves (measured 1.6e-3 on
    # decoder layer 4's feed_forward_norm.weight)
    kink = {k for k in errs if relu_gated(k) or (k.startswith("decoder.") and ".feed_forward_norm." in k)}
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    print(f"unfed gates: worst non-gated {worst}, worst gated {max((errs[k], k) for k in kink)}")
    assert abs(lg - lo) <= 1e-5 * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < 1e-3 and rel(*r["h_ctc"]) < 1e-3
    assert worst[0] < 1e-3, worst
    assert max(errs[k] for k in kink) < 2e-2, {k: errs[k] for k in kink}


def test_dynamic_chunk_graph_replays_match_eager_and_oracle():
    """BASELINE config 4's dynamic chunk inside a captured step: one hipGraph of the whole
    config-4 step (12 / 6 layers, d 512, 16 heads, fp32 build, T 1000 -> T' 249) whose prep
    reads the chunk size from the device scalar, replayed with c = 4, 16 and 249 (full context)
    written between replays.  Each replay's loss and flat gradient are bit-identical to an eager
    step built with that fixed c, and that eager step matches the fp64 oracle composed with
    padding_mask | triangle_mask(T', stage=c) (liteasr/utils/mask.py:84-89 through
    liteasr/nets/transformer_encoder.py:113-120) at the config-4 fp32 bars (loss 1e-5, logits
    and every gradient 1e-3 of max, the decoder ReLU branches fed as in
    test_parity_config4_full_model_fp32)."""
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.graph_step import GraphedTrainStep

    B, T, L = 2, 1000, 40
    params = O.init_params(CONFIG4, seed=11)
    buffers = O.init_buffers(CONFIG4)
    batch = O.synthetic_batch(B, T, L, CONFIG4["vocab_size"], seed=0)
    bd = [t.cuda() for t in batch]
    model = build(CONFIG4, "fp32")
    model.load_state_dict({**params, **buffers}, strict=False)
    model = model.cuda().train()
    model.chunk_from_device = True
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=CONFIG4["vocab_size"], smoothing=0.1, ctc_weight=0.3))
    tap = _GradTap(model.store)
    model.set_chunk(16)
    gs = GraphedTrainStep(model, crit, tap, bd, clip=5.0, warmup=1)
    for c in (4, 16, 249):
        model.set_chunk(c)
        loss_g = gs(bd).item()
        g_graph = tap.out.clone()
        assert model.last_chunk() == c
        r = run_case(CONFIG4, B, T, L, "fp32", chunk=c, feed_dec_gates=True)
        _check_dec_gates(r)
        _check_fp32(r, 1e-3)
        g_eager = torch.cat([r["grads"][0][n].reshape(-1) for n in model.store.names])
        g_flat = torch.cat([g_graph[model.store.offsets[n]:model.store.offsets[n] + model.store.shapes[n].numel()]
                            for n in model.store.names])
        assert loss_g == r["loss"][0], (c, loss_g, r["loss"][0])
        assert torch.equal(g_flat, g_eager), c


def test_dynamic_chunk_training_step_draws_per_step():
    """dynamic_chunk=True (config 4's training mode): every replay of the captured step draws
    its chunk size on the device from the step counter -- the draw the host mirror
    (dynamic_chunk_size) predicts -- and its loss equals an eager step at that fixed c, bit for
    bit; eval mode uses chunk_size."""
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.graph_step import GraphedTrainStep
    from liteasr_amd import kernels as Kn

    cfg = LARGE_HEADS
    params = O.init_params(cfg, seed=3)
    bd = [t.cuda() for t in O.synthetic_batch(2, 400, 6, cfg["vocab_size"], seed=7)]
    Tsub = ((400 - 1) // 2 - 1) // 2
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=cfg["vocab_size"], smoothing=0.1, ctc_weight=0.3))

    def fresh(chunk):
        m = build(cfg, "bf16", chunk)
        m.load_state_dict({**params, **O.init_buffers(cfg)}, strict=False)
        return m.cuda().train()

    m = fresh(16)
    m.dynamic_chunk = True
    tap = _GradTap(m.store)
    gs = GraphedTrainStep(m, crit, tap, bd, clip=5.0, warmup=1)
    seen = set()
    for _ in range(6):
        ctr = int(m._drop_ctr.item())
        loss = gs(bd).item()
        c = m.last_chunk()
        assert c == m.dynamic_chunk_size(m._seed_base + 11, ctr, Tsub, m.chunk_max)
        seen.add(c)
        e = fresh(c)
        e._drop_ctr.fill_(ctr)
        le = crit(e, *bd)
        le.backward()
        assert le.item() == loss, (c, le.item(), loss)
        assert torch.equal(e.store.grad, tap.out), c
    assert len(seen) >= 2, seen
    m.eval()
    assert m.chunk_mode() == Kn.CHUNK_FIXED


def test_parity_config4_full_model_bf16_emulated():
    """Config 4's full model in the default bf16 build (fused d_k 32 attention with the staged
    chunk-mask tiles, the full-row LayerNorm GEMMs at d 512) against the bf16-emulating
    oracle at the whole-model bars."""
    _check_emulated(run_case(CONFIG4, 2, 1000, 40, "bf16", chunk=16, emulate=True))


def test_parity_config5_long_bf16_emulated():
    """BASELINE config 5's shape: T 4000 (T' 999), CTC-only (w 1.0: the decoder runs and gets
    zero gradient), label length 150, full depth, one utterance pair."""
    _check_emulated(run_case(CONFIG2, 2, 4000, 150, "bf16", ctc_weight=1.0, emulate=True))


# The other encoders the reference's U2 builds (liteasr/nets/transformer_encoder.py:47-100;
# the oracle restatement is pinned to the reference's run by
# tests/test_oracle_golden.py::test_u2_encoder_variants_against_reference)
ENC_VARIANTS = {
    "tfm_abs": dict(enc_arch="transformer", use_rel=False),
    "tfm_rel": dict(enc_arch="transformer", use_rel=True),
    "cfm_abs_relu": dict(enc_arch="conformer", use_rel=False, activation="relu"),
    "cfm_rel_relu": dict(enc_arch="conformer", use_rel=True, activation="relu"),
}


@pytest.mark.parametrize("name", sorted(ENC_VARIANTS))
def test_parity_encoder_variants_fp32(name):
    """fp32 build vs the fp64 oracle, tiny widths (materialised attention): the bars of
    test_parity_fp32 (the ReLU conformer's conv-module / FFN kinks share the embed convs' bar)."""
    cfg = dict(TINY, **ENC_VARIANTS[name])
    r = run_case(cfg, 3, 130, 8, "fp32")
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 1e-5 * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < 2e-4 and rel(*r["h_ctc"]) < 2e-4
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    kink = {k for k in errs if k.startswith("encoder.embed.conv.")}
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    assert worst[0] < 2e-4, worst
    assert max(errs[k] for k in kink) < 2e-2, {k: errs[k] for k in kink}


@pytest.mark.parametrize("name", sorted(ENC_VARIANTS))
def test_parity_encoder_variants_bf16(name):
    """bf16 build at the small config's widths (d 256, 4 heads: d_k 64, the fused attention
    kernels -- with the positional term for use_rel, without it for the absolute PE) vs the
    fp64 oracle fed the same bf16-rounded weights: the bf16 bars of test_parity_bf16, every
    ReLU-activated encoder tensor counted as ReLU-gated.  The ReLU conformer's cosine bar is
    0.99: its conv module applies ReLU right after a BatchNorm (inputs ~N(0, 1) per channel,
    so a large share of them sits within bf16 rounding of the kink; measured worst 0.996,
    conv_norm.weight), while its fp32 build holds 2e-4 (test_parity_encoder_variants_fp32)."""
    cfg = dict(SMALL, **ENC_VARIANTS[name])
    r = run_case(cfg, 2, 210, 12, "bf16", round_bf16=True)
    relu_enc = cfg.get("activation") == "relu" or cfg["enc_arch"] == "transformer"
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 5e-3 * abs(lo), r["loss"]
    assert rel(*r["h_attn"]) < 2e-2 and rel(*r["h_ctc"]) < 2e-2
    g, go = r["grads"]
    errs, floor = grad_errs(g, go)
    for k in go:
        gated = relu_gated(k) or (relu_enc and k.startswith("encoder.enc_layers."))
        if go[k].abs().max().item() > floor:
            bar = (0.99 if cfg.get("activation") == "relu" else 0.998) if gated else 0.999
            assert cos(g[k], go[k]) >= bar, k
        assert errs[k] < (0.35 if gated else 5e-2), (k, errs[k])


def test_parity_full_depth_fp32():
    """All 12 encoder / 6 decoder layers (reduced width), B 2, T 400, fp32 build vs fp64."""
    _check_fp32(run_case(DEEP, 2, 400, 12, "fp32"), 2e-4)


def test_parity_chunk_mask_fp32():
    r = run_case(TINY, 2, 150, 6, "fp32", chunk=8)
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 1e-5 * abs(lo)
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    # 5e-4: per-channel sums over B*T rows (conv/BN/bias grads) are associated differently
    # from the CPU oracle's (fixed-order partials, deterministic); the chunk mask leaves
    # few unmasked frames per row, so these sums carry more cancellation here.
    assert max(errs.values()) < 5e-4, max((v, k) for k, v in errs.items())


def test_parity_ctc_only_fp32():
    r = run_case(TINY, 3, 120, 7, "fp32", ctc_weight=1.0)
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 1e-5 * abs(lo)
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    for k in go:
        if k.startswith("decoder."):
            assert g[k].abs().max().item() == 0.0, k  # decoder gets exactly zero gradient
        else:
            assert errs[k] < 2e-4, (k, errs[k])


def test_parity_eval_mode_grads_fp32():
    """Eval mode with gradients (BatchNorm on its running statistics: the batch-mean terms
    of the BN gradient vanish; dropout off except the CTC head's always-on one, 0 here)
    against the fp64 oracle differentiated in eval mode; BN buffers stay untouched."""
    r = run_case(TINY, 3, 130, 8, "fp32", training=False)
    lg, lo = r["loss"]
    assert abs(lg - lo) <= 1e-5 * abs(lo), r["loss"]
    g, go = r["grads"]
    errs, _ = grad_errs(g, go)
    kink = {k for k in errs if k.startswith("encoder.embed.conv.")}  # see test_parity_fp32
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    assert worst[0] < 2e-4, worst
    bufs, bo = r["bn"]
    for k, v in bo.items():
        if v.is_floating_point():
            assert torch.equal(bufs[k].double().cpu(), v), k


def test_eval_forward_uses_running_stats():
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig

    params = O.init_params(TINY, seed=3)
    buffers = O.init_buffers(TINY)
    for k in buffers:
        if k.endswith("running_mean"):
            buffers[k] = torch.randn(TINY["enc_dim"]) * 0.1
        elif k.endswith("running_var"):
            buffers[k] = torch.rand(TINY["enc_dim"]) + 0.5
    xs, xlens, ys, ylens = O.synthetic_batch(2, 100, 5, TINY["vocab_size"], seed=5)
    model = build(TINY, "fp32")
    model.load_state_dict({**params, **buffers}, strict=False)
    model = model.cuda().eval()
    with torch.no_grad():
        ha, hc = model(xs.cuda(), xlens.cuda(), ys.cuda(), ylens.cuda())
        ha_o, hc_o, _, _ = O.u2_forward(xs.double(), xlens, ys, ylens, {k: v.double() for k, v in params.items()},
                                        TINY, {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()},
                                        False)
    assert rel(ha, ha_o) < 2e-4
    assert rel(hc, hc_o) < 2e-4


def test_deferred_reductions_bit_exact(monkeypatch):
    """kernels.deferred_reductions (one lasr_reduce_multi launch per backward node) gives
    the same gradients, bit for bit, as the immediate per-call reductions.  Grouping of the
    deferred dW GEMMs is off here: it slices K differently (bit-exactness of the grouped
    launch itself at equal slicing: test_gemm_dw_group_bit_identical; the grouped step vs
    the oracle: the parity tests)."""
    import contextlib

    from liteasr_amd import kernels as Kn
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig

    monkeypatch.setattr(Kn, "DW_GROUP", False)

    params = O.init_params(SMALL, seed=5)
    xs, xlens, ys, ylens = [t.cuda() for t in O.synthetic_batch(2, 300, 9, SMALL["vocab_size"], seed=4)]
    grads = []
    @contextlib.contextmanager
    def immediate(hold=False, on_done=None):  # no deferral: every reduction in its own call
        yield
        if on_done is not None:
            on_done()

    for defer in (True, False):
        if not defer:
            monkeypatch.setattr(Kn, "deferred_reductions", immediate)
        model = build(SMALL, "bf16")
        model.load_state_dict({**params, **O.init_buffers(SMALL)}, strict=False)
        model = model.cuda().train()
        crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=SMALL["vocab_size"], smoothing=0.1, ctc_weight=0.3))
        crit(model, xs, xlens, ys, ylens).backward()
        grads.append({n: p.grad.detach().clone() for n, p in model.named_parameters()})
    assert not Kn._DEFER.segs and not Kn._DEFER.held and Kn._DEFER.depth == 0
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


def test_dropout_train_step_runs_and_is_deterministic():
    """Dropout cannot match torch's RNG bit-for-bit; check the step is finite, that the
    same device counter reproduces the same loss, and that the keep rate is right
    (kernel level: test_gemm_dropout_matches_branch_grad)."""
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig

    params = O.init_params(TINY, seed=1)
    model = build(TINY, "bf16", dropout=0.1)
    model.load_state_dict({**params, **O.init_buffers(TINY)}, strict=False)
    model = model.cuda().train()
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=30, smoothing=0.1, ctc_weight=0.3))
    xs, xlens, ys, ylens = [t.cuda() for t in O.synthetic_batch(2, 100, 5, 30, seed=2)]
    losses = []
    for _ in range(2):
        model._drop_ctr.zero_()
        l = crit(model, xs, xlens, ys, ylens)
        l.backward()
        losses.append(l.item())
    assert math.isfinite(losses[0]) and losses[0] == losses[1]
    l3 = crit(model, xs, xlens, ys, ylens).item()  # counter advanced -> new masks
    assert l3 != losses[0]


def _graph_setup(dropout):
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.optims.noam import Noam, NoamConfig

    params = O.init_params(TINY, seed=3)
    model = build(TINY, "bf16", dropout=dropout)
    model.load_state_dict({**params, **O.init_buffers(TINY)}, strict=False)
    model = model.cuda().train()
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=30, smoothing=0.1, ctc_weight=0.3))
    opt = Noam(model.parameters(), NoamConfig(model_dim=64, warmup=10))
    return model, crit, opt


def test_graphed_step_matches_eager():
    """liteasr_amd.graph_step: a replayed hipGraph step (fwd+loss+bwd+clip+Noam/Adam+zero_grad,
    dropout on) is bit-identical to the same steps launched eagerly (deterministic
    kernels, device-side dropout counter and optimizer state)."""
    from liteasr_amd.graph_step import GraphedTrainStep

    batches = [[t.cuda() for t in O.synthetic_batch(3, 120, 6, 30, seed=10 + i)] for i in range(4)]
    m1, c1, o1 = _graph_setup(0.1)
    eager = []
    for b in batches:
        l = c1(m1, *b)
        l.backward()
        o1.clip_and_step(5.0)
        o1.zero_grad()
        eager.append(l.item())
    m2, c2, o2 = _graph_setup(0.1)
    # construction runs a warm-up step and then restores parameters, optimizer state, BN
    # buffers and the dropout counter: the replays start from the initial state
    gs = GraphedTrainStep(m2, c2, o2, batches[0], clip=5.0, warmup=2)
    graphed = [gs(b).item() for b in batches]
    assert graphed == eager, (graphed, eager)
    assert torch.equal(m1.store.flat, m2.store.flat)
    assert o1.device_state() == o2.device_state()
    # the launches one replay issues (bench.py's graph_nodes_per_step): every node of the
    # kept graph templates is a kernel (the product allocates outside the capture, no
    # memcpy / memset nodes), and a replay issues at least one per fused node
    nodes = gs.graph_nodes()
    if nodes is None:  # this torch keeps no graph templates (no keep_graph / raw_cuda_graph)
        pytest.skip("graph node counts unavailable on this torch; the replay equality above held")
    assert nodes["memcpy"] == 0 and nodes["other"] == 0, nodes
    assert nodes["kernel"] > 50, nodes


def test_graphed_step_survives_workspace_growth():
    """The captured graphs address the shared kernel scratch buffer (kernels.WS); an eager
    call that needs more scratch replaces that buffer. GraphedTrainStep keeps the captured
    one alive, so replays after the growth leave live tensors alone (memory of the replaced
    buffer's size handed out again and filled with NaN stays NaN) and still match the eager
    steps bit for bit."""
    from liteasr_amd import kernels as K
    from liteasr_amd.graph_step import GraphedTrainStep

    batches = [[t.cuda() for t in O.synthetic_batch(3, 120, 6, 30, seed=20 + i)] for i in range(3)]
    m1, c1, o1 = _graph_setup(0.1)
    eager = []
    for b in batches:
        l = c1(m1, *b)
        l.backward()
        o1.clip_and_step(5.0)
        o1.zero_grad()
        eager.append(l.item())
    m2, c2, o2 = _graph_setup(0.1)
    gs = GraphedTrainStep(m2, c2, o2, batches[0], clip=5.0, warmup=1)
    graphed = [gs(batches[0]).item()]
    dev = torch.device("cuda", torch.cuda.current_device())
    old = K.WS.buf[dev.index]
    n_old = old.numel()
    del old
    grown = K.WS.get(n_old * 4, dev)  # what a longer eager batch would do
    assert grown.numel() > n_old and K.WS.buf[dev.index] is grown
    grown.fill_(float("nan"))
    reuse = torch.full((n_old,), float("nan"), device=dev)  # may land on a freed block
    graphed += [gs(b).item() for b in batches[1:]]
    torch.cuda.synchronize()
    # the replays write their scratch into the captured buffer, never into live tensors
    assert torch.isnan(reuse).all() and torch.isnan(grown).all()
    assert graphed == eager, (graphed, eager)
    assert torch.equal(m1.store.flat, m2.store.flat)
    del reuse


def _ddp_graph_worker(rank, world, port, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from liteasr_amd.distributed.ddp import DistributedDataParallel
        from liteasr_amd.graph_step import GraphedTrainStep

        out = {}
        for mode in ("eager", "graph_overlap", "graph_split"):
            m, c, o = _graph_setup(0.0)
            net = DistributedDataParallel(m, bucket_cap_mb=0.05)  # several buckets -> several segments
            bs = [[t.cuda() for t in O.synthetic_batch(2, 100, 5, 30, seed=50 + 7 * rank + i)] for i in range(3)]
            losses = []
            if mode == "eager":
                for b in bs:
                    l = c(net, *b)
                    l.backward()
                    o.clip_and_step(5.0)
                    o.zero_grad()
                    losses.append(l.item())
            else:
                gs = GraphedTrainStep(net, c, o, bs[0], clip=5.0, warmup=1, overlap=mode == "graph_overlap")
                if mode == "graph_overlap":
                    assert len(gs.segs) == len(gs.cuts) + 1 >= 3, (gs.cuts, len(net.reducer.buckets))
                losses = [gs(b).item() for b in bs]
            out[mode] = (losses, m.store.flat.double().cpu())
        le, fe = out["eager"]
        ok = True
        for mode in ("graph_overlap", "graph_split"):
            lg, fg = out[mode]
            ok = ok and max(abs(a - b) / abs(a) for a, b in zip(le, lg)) < 1e-5 and \
                (fe - fg).abs().max().item() <= 1e-6 * fe.abs().max().item()
        q.put((rank, ok, le, [out[k][0] for k in ("graph_overlap", "graph_split")]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e), None))


def _two_ranks(worker, world=2):
    import multiprocessing as mp
    import random

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    return res


def test_graphed_step_ddp_two_ranks_gloo():
    """Graphed DDP steps vs the eager DDP step with hook-driven bucket all-reduce, 2 ranks
    sharing the one GPU, gloo backend (RCCL cannot put two ranks on one device):
    'graph_overlap' = backward segments as separate graphs with each bucket's all-reduce
    launched between them (the bench path), 'graph_split' = one fwd/bwd graph, all
    buckets, update graph."""
    for rank, ok, le, lg in _two_ranks(_ddp_graph_worker):
        assert ok, (rank, le, lg)


class _GradTap:
    """Optimizer stand-in for GraphedTrainStep: 'step' copies the (all-reduced) flat
    gradient out, zero_grad clears it -- both plain stream-ordered copies, capturable."""

    def __init__(self, store):
        self.store = store
        self.out = torch.zeros_like(store.ensure_grad())

    def clip_and_step(self, clip):
        self.out.copy_(self.store.grad)

    def zero_grad(self):
        self.store.grad.zero_()


DDP_CFG = O.default_cfg(enc_dim=64, enc_heads=4, enc_ff=256, enc_layers=3, dec_dim=64, dec_heads=4, dec_ff=256,
                        dec_layers=2, vocab_size=40)


def _ddp_equiv_worker(rank, world, port, q):
    """the N-rank averaged gradient equals the single-process gradient on
    the concatenated batch.  BN in eval mode (running statistics), so per-rank batch
    statistics do not enter; dropout 0; fp32 build."""
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
        from liteasr_amd.distributed.ddp import DistributedDataParallel
        from liteasr_amd.graph_step import GraphedTrainStep

        cfg = DDP_CFG
        params = O.init_params(cfg, seed=17)
        buffers = O.init_buffers(cfg)
        for k in buffers:  # non-trivial running statistics
            if k.endswith("running_mean"):
                buffers[k] = torch.randn(cfg["enc_dim"], generator=torch.Generator().manual_seed(1)) * 0.1
            elif k.endswith("running_var"):
                buffers[k] = torch.rand(cfg["enc_dim"], generator=torch.Generator().manual_seed(2)) + 0.5
        Bfull = 4
        full = [t.cuda() for t in O.synthetic_batch(Bfull, 180, 9, cfg["vocab_size"], seed=23)]
        half = [t[rank * Bfull // world:(rank + 1) * Bfull // world].contiguous() for t in full]
        crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=cfg["vocab_size"], smoothing=0.1, ctc_weight=0.3))

        def fresh():
            m = build(cfg, "fp32")
            m.load_state_dict({**params, **buffers}, strict=False)
            return m.cuda().eval()

        # (1) single process, concatenated batch
        m1 = fresh()
        crit(m1, *full).backward()
        g_single = m1.store.grad.double().cpu()
        # (2) eager DDP, hook-driven bucket all-reduce (mean) overlapped with the backward
        m2 = fresh()
        net2 = DistributedDataParallel(m2, bucket_cap_mb=0.2)
        crit(net2, *half).backward()
        g_ddp = m2.store.grad.double().cpu()
        # (3) the graphed, segmented DDP step (bench path): all-reduce between backward segments
        m3 = fresh()
        net3 = DistributedDataParallel(m3, bucket_cap_mb=0.2)
        tap = _GradTap(m3.store)
        gs = GraphedTrainStep(net3, crit, tap, half, warmup=1)
        gs(half)
        torch.cuda.synchronize()
        g_graph = tap.out.double().cpu()
        scale = g_single.abs().max().item()
        err_ddp = (g_ddp - g_single).abs().max().item() / scale
        # per-parameter, relative to each tensor's own max (floored at 1e-3 of the largest)
        worst = 0.0
        for n in m1.store.names:
            o, k = m1.store.offsets[n], m1.store.shapes[n].numel()
            a, b = g_ddp[o:o + k], g_single[o:o + k]
            worst = max(worst, (a - b).abs().max().item() / max(b.abs().max().item(), 1e-3 * scale))
        graph_eq = torch.equal(g_graph, g_ddp)
        q.put((rank, err_ddp < 2e-4 and worst < 2e-4 and graph_eq, (err_ddp, worst, graph_eq, len(gs.segs)), None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, False, repr(e), traceback.format_exc()))


def test_ddp_grads_equal_single_process_concatenated_batch():
    """SURVEY §8(e) / trainer.py:142-171: world-2 averaged gradients (eager hook path and
    the segmented graphed path) == one process on the concatenated batch, within 2e-4 of
    each tensor's max; the graphed path bit-equal to the eager DDP path."""
    for rank, ok, info, tb in _two_ranks(_ddp_equiv_worker):
        assert ok, (rank, info, tb)


def test_ddp_grads_equal_single_process_four_ranks():
    """The same equivalence at world 4 (one utterance per rank, four ranks sharing the GPU over
    gloo): the bucket mean over four ranks == one process on the concatenated batch, and the
    segmented graphed path bit-equal to the eager DDP path."""
    res = _two_ranks(_ddp_equiv_worker, world=4)
    assert sorted(r[0] for r in res) == [0, 1, 2, 3]
    for rank, ok, info, tb in res:
        assert ok, (rank, info, tb)


@pytest.mark.gpu
def test_encoder_reuse_forward_backward():
    """U2.encode (SURVEY §8 f4 building block: the encoder as a differentiable module for
    other heads): output, key mask and encoder parameter gradients of sum(h * R) against
    the fp64 oracle encoder (transformer_encoder.py:107-127); non-encoder grads stay 0."""
    cfg = TINY
    params = O.init_params(cfg, seed=21)
    buffers = O.init_buffers(cfg)
    xs, xlens, _, _ = O.synthetic_batch(3, 140, 4, cfg["vocab_size"], seed=4)
    p64 = {k: v.double().requires_grad_(True) for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in buffers.items()}
    h_o, km_o = O.encoder(xs.double(), xlens, p64, cfg, b64, True)
    R = torch.randn(h_o.shape, generator=torch.Generator().manual_seed(9), dtype=torch.float64)
    (h_o * R).sum().backward()
    go = {k: v.grad for k, v in p64.items() if k.startswith("encoder.")}
    model = build(cfg, "fp32")
    model.load_state_dict({**params, **buffers}, strict=False)
    model = model.cuda().train()
    h, km = model.encode(xs.cuda(), xlens.cuda())
    (h * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(km.cpu(), km_o)
    assert rel(h.detach(), h_o.detach()) < 2e-4
    g = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    errs, _ = grad_errs({k: g[k] for k in go}, go)
    kink = {k for k in errs if k.startswith("encoder.embed.conv.")}  # see test_parity_fp32
    worst = max((v, k) for k, v in errs.items() if k not in kink)
    assert worst[0] < 2e-4, worst
    assert max(errs[k] for k in kink) < 2e-2
    assert all(float(g[k].abs().max()) == 0.0 for k in g if not k.startswith("encoder."))
