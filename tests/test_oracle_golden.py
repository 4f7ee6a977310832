"""Pin the CPU oracle (oracle/u2_oracle.py) to golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import u2_oracle as O  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def load(name):
    return {k: torch.from_numpy(v) for k, v in np.load(os.path.join(G, name)).items()}


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def test_rel_shift_closed_form():
    d = load("relshift.npz")
    for T in range(1, 10):
        assert torch.equal(O.rel_shift(d[f"in_{T}"]), d[f"out_{T}"]), T


def test_lengths_and_masks():
    d = load("lengths.npz")
    assert torch.equal(O.pred_len(d["xlen"]), d["pred_len"])
    sub = []
    for x in d["xlen"].tolist():
        T = max(x, 3)
        m = O.encoder_key_mask(torch.tensor([x]), T)
        sub.append(int((~m).sum()))
    assert sub == d["sub_valid"].tolist()
    # frame t' valid iff 4 t' < xlen  (closed form used by the HIP prep kernel)
    for x in d["xlen"].tolist():
        T = max(x, 3)
        Tp = O.subsampled_len(T)
        assert sum(1 for t in range(Tp) if 4 * t < x) == sub[x - 1]
    assert torch.equal(O.triangle_mask(8, stage=2).to(torch.uint8), d["tri_8_s2"])
    assert torch.equal(O.triangle_mask(3, 5, diagonal=2).to(torch.uint8), d["tri_3_5_d2"])


def _ctc_loss(h_ctc, xlens, ys, ylens, w):
    V = h_ctc.shape[-1]
    L = ys.shape[1]
    h_attn = torch.zeros(h_ctc.shape[0], L + 1, V, dtype=h_ctc.dtype)
    _, _, tgt = O.decoder_io(ys, ylens, V - 1, V - 1)
    return O.hybrid_loss(h_attn, h_ctc, tgt, ys, xlens, ylens, w, 0.1)


def test_ctc_loss_and_grad():
    d = load("ctc.npz")
    loss, lc, la = _ctc_loss(d["h_ctc"].double(), d["xlens"], d["ys"], d["ylens"], 1.0)
    assert torch.isfinite(loss).item() == bool(d["finite"])
    g = load("ctc_grad.npz")
    h = g["h_ctc"].double().requires_grad_()
    loss, _, _ = _ctc_loss(h, g["xlens"], g["ys"], g["ylens"], 1.0)
    assert abs(loss.item() - g["loss"].item()) <= 1e-5 * abs(g["loss"].item())
    loss.backward()
    assert rel(h.grad, g["grad"]) < 1e-4


def test_ctc_numpy_restatement_matches_reference():
    """Independent float64 alpha/beta recursion (oracle/ctc_ref.py) vs the reference's
    aten ctc_loss on the same logits."""
    from oracle import ctc_ref

    g = load("ctc_grad.npz")
    B = g["h_ctc"].shape[0]
    h = g["h_ctc"].double()
    tot = 0.0
    grad = np.zeros(h.shape)
    ilen = O.pred_len(g["xlens"])
    for b in range(B):
        lp = torch.log_softmax(h[b, : ilen[b]], -1).numpy()
        lab = g["ys"][b, : g["ylens"][b]].numpy()
        nll, glog = ctc_ref.ctc_nll_and_grad(lp, lab)
        tot += nll
        grad[b, : ilen[b]] = glog
    assert abs(tot / B - g["loss"].item()) <= 1e-6 * abs(g["loss"].item())
    # the golden is the reference run in fp32 (aten fp32 CTC is ~1e-4 off fp64)
    assert rel(torch.from_numpy(grad / B), g["grad"]) < 1e-4


def test_label_smoothed_kl():
    d = load("kl.npz")
    h = d["h_attn"].double().requires_grad_()
    ys, ylens = d["ys"], d["ylens"]
    V = h.shape[-1]
    _, _, tgt = O.decoder_io(ys, ylens, V - 1, V - 1)
    T = 51
    h_ctc = torch.zeros(ys.shape[0], T, V, dtype=torch.float64)
    loss, _, _ = O.hybrid_loss(h, h_ctc, tgt, ys, torch.full((ys.shape[0],), 210), ylens, 0.0, 0.1)
    assert abs(loss.item() - d["loss"].item()) <= 1e-5 * abs(d["loss"].item())
    loss.backward()
    assert rel(h.grad, d["grad"]) < 1e-5


TINY_GOLDEN = O.default_cfg(enc_dim=32, enc_heads=4, enc_ff=64, enc_layers=2, dec_dim=32, dec_heads=4,
                            dec_ff=64, dec_layers=1, vocab_size=20, input_dim=40)


def _golden_params(d, prefix):
    p, b = {}, {}
    for k, v in d.items():
        if k.startswith(prefix):
            name = k[len(prefix):]
            if "running_" in name or "num_batches" in name:
                b[name] = v.clone()
            else:
                p[name] = v.clone()
    return p, b


def test_u2_step_against_reference():
    d = load("u2_step.npz")
    params, buffers = _golden_params(d, "init.")
    p64 = {k: v.double() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()}
    batch = (d["xs"].double(), d["xlens"], d["ys"], d["ylens"])
    with torch.no_grad():
        ha, hc, _, _ = O.u2_forward(*batch, p64, TINY_GOLDEN, {k: v.clone() for k, v in b64.items()}, True)
    assert rel(ha, d["h_attn"]) < 1e-5
    assert rel(hc, d["h_ctc"]) < 1e-5
    loss, grads, new, st, norm = O.train_step(p64, b64, batch, TINY_GOLDEN, model_dim=32)
    assert abs(loss.item() - d["loss"].item()) <= 1e-5 * abs(d["loss"].item())
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, g in grads.items():
        ref = d["grad." + k].double()
        err = (g - ref).abs().max().item() / max(ref.abs().max().item(), 1e-3 * gmax)
        assert err < 1e-4, (k, err)
    assert abs(norm - d["grad_norm"].item()) <= 1e-5 * d["grad_norm"].item()
    for k, v in new.items():
        assert rel(v, d["new." + k]) < 1e-5, k
    for k, v in b64.items():
        ref = d["new." + k]
        if v.is_floating_point():
            assert rel(v, ref) < 1e-5, k
        else:
            assert int(v) == int(ref), k


# the other encoders the reference's U2 builds (tests/golden/make_golden.py U2_VARIANTS):
# golden prefix -> oracle cfg keys
U2_VARIANT_CFG = {
    "tfm_abs": dict(enc_arch="transformer", use_rel=False),
    "tfm_rel": dict(enc_arch="transformer", use_rel=True),
    "cfm_abs_relu": dict(enc_arch="conformer", use_rel=False, activation="relu"),
    "cfm_rel_relu": dict(enc_arch="conformer", use_rel=True, activation="relu"),
}


def variant_case(name):
    """(golden dict, cfg, fp64 params, fp64 buffers, batch) of one u2_variants.npz entry."""
    d = {k[len(name) + 1:]: v for k, v in load("u2_variants.npz").items() if k.startswith(name + ".")}
    params, buffers = _golden_params(d, "init.")
    cfg = dict(TINY_GOLDEN, **U2_VARIANT_CFG[name])
    p64 = {k: v.double() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()}
    return d, cfg, p64, b64, (d["xs"].double(), d["xlens"], d["ys"], d["ylens"])


@pytest.mark.parametrize("name", sorted(U2_VARIANT_CFG))
def test_u2_encoder_variants_against_reference(name):
    """Transformer encoder layers (absolute / relative PE) and the conformer with absolute PE or
    ReLU (liteasr/nets/transformer_encoder.py:47-100, transformer_layer.py:10-136): the oracle's
    restatement reproduces the reference's outputs, loss and every gradient."""
    d, cfg, p64, b64, batch = variant_case(name)
    assert set(p64) == {k[len("init."):] for k in d if k.startswith("init.") and "running_" not in k
                        and "num_batches" not in k}
    with torch.no_grad():
        ha, hc, _, _ = O.u2_forward(*batch, p64, cfg, {k: v.clone() for k, v in b64.items()}, True)
    assert rel(ha, d["h_attn"]) < 1e-5
    assert rel(hc, d["h_ctc"]) < 1e-5
    loss, grads, _, _, _ = O.train_step(p64, b64, batch, cfg, model_dim=32)
    assert abs(loss.item() - d["loss"].item()) <= 1e-5 * abs(d["loss"].item())
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, g in grads.items():
        ref = d["grad." + k].double()
        err = (g - ref).abs().max().item() / max(ref.abs().max().item(), 1e-3 * gmax)
        assert err < 1e-4, (k, err)


def test_u2_encoder_variant_init_keys():
    """The oracle's init_params produces exactly the reference's state_dict keys and shapes per
    variant (so the GPU tests can load oracle weights into liteasr_amd's U2)."""
    for name in U2_VARIANT_CFG:
        d, cfg, p64, b64, _ = variant_case(name)
        mine = O.init_params(cfg)
        assert {k: tuple(v.shape) for k, v in mine.items()} == {k: tuple(v.shape) for k, v in p64.items()}, name
        assert set(O.init_buffers(cfg)) == set(b64), name


def _golden_step_inputs():
    d = load("u2_step.npz")
    params, buffers = _golden_params(d, "init.")
    p64 = {k: v.double() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()}
    return d, p64, b64, (d["xs"].double(), d["xlens"], d["ys"], d["ylens"])


@pytest.mark.parametrize("chunk", [0, 4])
def test_bf16_oracle_without_rounding_is_the_fp64_oracle(monkeypatch, chunk):
    """oracle/u2_bf16.py with its bf16 rounding replaced by the identity is the pinned fp64
    oracle (u2_oracle.py): the blockwise online softmax, the hand-written attention backward
    (P recomputed from the row statistics, D = rowsum(dO * O), the inverse rel_shift
    scatter), the stored-gate activation backward and the fused residual layout give the
    same loss, logits and every gradient to 1e-9 -- so the emulating oracle differs from the
    one the reference goldens pin ONLY by the roundings it inserts."""
    from oracle import u2_bf16 as E

    monkeypatch.setattr(E, "bf16", lambda x: x)
    d, p64, b64, batch = _golden_step_inputs()
    loss, _, _, grads, ha, hc = E.loss_and_grads(p64, {k: v.clone() for k, v in b64.items()}, batch, TINY_GOLDEN,
                                                 chunk=chunk)
    bref = {k: v.clone() for k, v in b64.items()}
    names = list(p64)
    leaf = {k: p64[k].clone().requires_grad_() for k in names}
    ha_o, hc_o, _, tgt = O.u2_forward(*batch, leaf, TINY_GOLDEN, bref, True, chunk)
    lo, _, _ = O.hybrid_loss(ha_o, hc_o, tgt, batch[2], batch[1], batch[3], 0.3, 0.1)
    lo.backward()
    assert abs(loss.item() - lo.item()) <= 1e-12 * abs(lo.item())
    assert rel(ha, ha_o.detach()) < 1e-10 and rel(hc, hc_o.detach()) < 1e-10
    go = {k: (leaf[k].grad if leaf[k].grad is not None else torch.zeros_like(leaf[k])) for k in names}
    gmax = max(v.abs().max().item() for v in go.values())
    for k in names:  # relative to each tensor's max, floored for analytically-zero gradients
        scale = max(go[k].abs().max().item(), 1e-6 * gmax)
        assert (grads[k] - go[k]).abs().max().item() <= 1e-9 * scale, k
    if chunk == 0:  # and hence the reference's own step
        assert abs(loss.item() - d["loss"].item()) <= 1e-5 * abs(d["loss"].item())


def test_bf16_oracle_tracks_fp64():
    """With the roundings in, the emulating oracle stays within bf16 distance of the
    reference's fp32 step (u2_step.npz): loss 1e-2 relative, every gradient cosine >= 0.99."""
    from oracle import u2_bf16 as E

    d, p64, b64, batch = _golden_step_inputs()
    loss, _, _, grads, _, _ = E.loss_and_grads(p64, b64, batch, TINY_GOLDEN)
    assert abs(loss.item() - d["loss"].item()) <= 1e-2 * abs(d["loss"].item())
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, g in grads.items():
        ref = d["grad." + k].double()
        if ref.abs().max().item() < 1e-3 * gmax:
            continue
        c = (g.flatten() @ ref.flatten()) / (g.norm() * ref.norm())
        assert c.item() >= 0.99, (k, c.item())


def test_chunk_mask_composition_against_reference():
    d = load("u2_step.npz")
    params, buffers = _golden_params(d, "init.")
    p64 = {k: v.double() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()}
    with torch.no_grad():
        h, _ = O.encoder(d["xs"].double(), d["xlens"], p64, TINY_GOLDEN, b64, True, chunk=4)
    assert rel(h, d["h_enc_chunk4"]) < 1e-5


def test_liteasr_amd_init_matches_reference():
    """torch.manual_seed(42); U2(cfg) builds bit-identical weights + identical keys."""
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    d = load("u2_step.npz")
    c = U2Config(input_dim=40, vocab_size=20, enc_dim=32, enc_ff_dim=64, enc_attn_heads=4, enc_layers=2,
                 dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=1)
    resolve_self(c)
    torch.manual_seed(42)
    m = U2(c)
    sd = {k: v for k, v in m.state_dict().items() if not k.endswith(".pe.pe")}
    ref = {k[5:]: v for k, v in d.items() if k.startswith("init.")}
    assert set(sd) == set(ref)
    for k in ref:
        assert torch.equal(sd[k].to(ref[k].dtype), ref[k]), k


@pytest.mark.parametrize("name", sorted(U2_VARIANT_CFG))
def test_liteasr_amd_init_matches_reference_variants(name):
    """The same for the other encoders: identical keys and bit-identical seed-42 weights."""
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    d, cfg, _, _, _ = variant_case(name)
    c = U2Config(input_dim=40, vocab_size=20, enc_dim=32, enc_ff_dim=64, enc_attn_heads=4, enc_layers=2,
                 dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=1, enc_arch=cfg["enc_arch"],
                 use_rel=cfg["use_rel"], activation=cfg.get("activation", "swish"))
    resolve_self(c)
    torch.manual_seed(42)
    m = U2(c)
    sd = {k: v for k, v in m.state_dict().items() if not k.endswith(".pe.pe")}
    ref = {k[5:]: v for k, v in d.items() if k.startswith("init.")}
    assert set(sd) == set(ref)
    for k in ref:
        assert torch.equal(sd[k].to(ref[k].dtype), ref[k]), k


def _ctc_large_case(name):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from inputs import ctc_large_inputs

    d = load("ctc_large.npz")
    Tp, B, V, L, seed = d[f"{name}_dims"].tolist()
    xlens, ys, ylens, h = ctc_large_inputs(Tp, B, V, L, seed)
    # the regenerated logits must be the ones the reference saw
    ref_sum = d[f"{name}_logit_sum"].item()  # (parallel float64 sum: order-dependent last bits)
    assert abs(h.double().sum().item() - ref_sum) <= 1e-9 * abs(ref_sum)
    assert torch.equal(h.reshape(-1)[:64], d[f"{name}_logit_head"])
    assert torch.equal(xlens, d[f"{name}_xlens"]) and torch.equal(ys, d[f"{name}_ys"])
    return d, (Tp, B, V, L), xlens, ys, ylens, h


@pytest.mark.parametrize("name", ["t249", "t999"])
def test_ctc_restatement_at_full_sizes(name):
    """SURVEY §8(c) F-c: the float64 CTC restatement vs the reference's HybridCTCLoss
    (ctc_weight 1) at (T' 249, B 4, V 4233, L 40) and (T' 999, B 2, V 4233, L 150).
    Loss within 1e-5 relative per utterance.  The golden gradient is the reference's fp32
    aten CTC, which itself sits 1.38e-3 (T' 249) and 8.1e-3 (T' 999) of max away from the
    float64 result on these logits (measured with torch fp64 ctc_loss); the exact float64
    restatement must agree with it within that error (bound: 2e-3 / 1.2e-2)."""
    from oracle import ctc_ref

    d, (Tp, B, V, L), xlens, ys, ylens, h = _ctc_large_case(name)
    ilen = O.pred_len(xlens)
    cols = d[f"{name}_cols"]
    per, gcols = [], torch.zeros(B, Tp, len(cols), dtype=torch.float64)
    for b in range(B):
        lp = torch.log_softmax(h[b, : ilen[b]].double(), -1).numpy()
        nll, g = ctc_ref.ctc_nll_and_grad(lp, ys[b, : ylens[b]].numpy())
        per.append(nll)
        gcols[b, : ilen[b]] = torch.from_numpy(g)[:, cols]
    ref_per = d[f"{name}_loss_per_utt"].numpy()
    assert np.allclose(per, ref_per, rtol=1e-5, atol=0), (per, ref_per)
    assert abs(sum(per) / B - d[f"{name}_loss"].item()) <= 1e-5 * abs(d[f"{name}_loss"].item())
    err = rel(gcols / B, d[f"{name}_grad_cols"])
    assert err < (2e-3 if Tp < 500 else 1.2e-2), err


def test_host_policies_match_reference():
    """SeqBatch / FrameBatch grouping (incl. an utterance alone over the frame budget, which
    the reference answers with an empty minibatch first), Trigger firing and Vocab
    conversions vs the reference's own classes (tests/golden/host_policies.npz)."""
    from types import SimpleNamespace

    from liteasr_amd.dataclass.vocab import Vocab
    from liteasr_amd.utils.batchify import FrameBatch, SeqBatch
    from liteasr_amd.utils.trigger import Trigger

    d = np.load(os.path.join(ROOT, "tests", "golden", "host_policies.npz"))
    samples = [SimpleNamespace(xlen=int(a), ylen=int(b)) for a, b in zip(d["xlen"], d["ylen"])]
    cfgs = [("seq", dict(batch_size=8, min_batch_size=1, max_len_in=400, max_len_out=30)),
            ("seq", dict(batch_size=5, min_batch_size=2, max_len_in=800, max_len_out=100)),
            ("seq", dict(batch_size=3, min_batch_size=3, max_len_in=100, max_len_out=10)),
            ("frame", dict(max_frame_in=1500, max_frame_out=None, max_frame_inout=None)),
            ("frame", dict(max_frame_in=None, max_frame_out=120, max_frame_inout=None)),
            ("frame", dict(max_frame_in=3000, max_frame_out=200, max_frame_inout=2600))]
    saw_empty = False
    for ci, (kind, c) in enumerate(cfgs):
        pol = (SeqBatch if kind == "seq" else FrameBatch)(SimpleNamespace(**c))
        pol.batchify(list(range(len(samples))), samples)
        sizes = [len(pol[b]) for b in range(len(pol))]
        assert sizes == d[f"c{ci}_sizes"].tolist(), (ci, sizes)
        assert sum((list(pol[b]) for b in range(len(pol))), []) == d[f"c{ci}_idx"].tolist()
        saw_empty |= 0 in sizes
    assert saw_empty  # the oversize edge was exercised
    pokes = [(int(e), int(i), "iteration" if u == 0 else "epoch") for e, i, u in d["pokes"]]
    for ti, (interval, unit) in enumerate([(1, "epoch"), (2, "epoch"), (3, "iteration"), (5, "iteration")]):
        fired = []
        ev = Trigger(interval, unit)(lambda: fired.append(None))
        got = []
        for k, (e, i, u) in enumerate(pokes):
            n0 = len(fired)
            ev(SimpleNamespace(epoch=e, iter=i), u)
            if len(fired) > n0:
                got.append(k)
        assert got == d[f"trig{ti}_fired"].tolist(), ti
    v = Vocab(os.path.join(ROOT, "tests", "golden", "loader", "vocab.txt"))
    assert list(v.lookup(list(range(len(v))), convert=True)) == d["vocab_conv"].tolist()
    assert list(v.lookup(list(range(len(v))))) == d["vocab_tokens"].tolist()


@pytest.mark.parametrize("case", [0, 1])
def test_paraformer_oracle_matches_reference(case):
    """oracle/paraformer_ref.py (CIF predictor, glancing sampler, parallel decoder,
    ParaformerLoss) vs the reference Paraformer run (tests/golden/paraformer.npz): every
    intermediate, the loss and every gradient, same Python ``random`` seed."""
    import random

    from oracle import paraformer_ref as PR

    z = np.load(os.path.join(G, "paraformer.npz"))
    pre = f"c{case}."
    g = lambda k: torch.from_numpy(z[pre + k])  # noqa: E731
    cfg = PR.default_cfg(enc_dim=64, enc_heads=4, enc_ff=128, enc_layers=2, dec_dim=64, dec_heads=4, dec_ff=128,
                         dec_layers=1, vocab_size=20, input_dim=40)
    init = {k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("init.")}
    isbn = lambda k: "running" in k or "num_batches" in k  # noqa: E731
    bn = {k: v.clone() for k, v in init.items() if isbn(k)}
    p = {k: v.clone().requires_grad_() for k, v in init.items() if not isbn(k)}
    random.seed(int(z[pre + "random_seed"]))
    hs, sa, ex = PR.paraformer_forward(g("xs"), g("xlens"), g("ys"), g("ylens"), p, cfg, bn, True)
    loss, _, _ = PR.paraformer_loss(hs, sa, g("ys"), g("ylens"))
    loss.backward()
    rel = lambda a, b: ((a.detach().double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30)).item()  # noqa: E731
    assert torch.equal(ex["ys_hat"], g("ys_hat")) and torch.equal(ex["replace"], g("replace"))
    assert rel(ex["h_enc"], g("h_enc")) < 1e-5 and rel(ex["hs_cif"], g("h_cif")) < 1e-5
    assert rel(sa, g("sum_alpha")) < 1e-6 and rel(hs, g("hs_attn")) < 1e-5
    assert abs(loss.item() - float(z[pre + "loss"])) < 1e-5 * abs(float(z[pre + "loss"]))
    gold = {k[len(pre) + 5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre + "grad.")}
    assert set(gold) == set(p)
    floor = 1e-3 * max(v.abs().max().item() for v in gold.values())
    for k, v in gold.items():
        err = (p[k].grad.double() - v.double()).abs().max().item() / max(v.abs().max().item(), floor)
        assert err < 1e-4, (k, err)


TRANSDUCER_GOLDEN = O.default_cfg(enc_dim=64, enc_heads=4, enc_ff=128, enc_layers=2, vocab_size=20, input_dim=40,
                                  dec_layers=2, dec_units=48)


def test_transducer_oracle_matches_reference():
    """oracle/transducer_ref.py (encoder + LSTM prediction network + joint) against the
    reference Transducer's own run (transducer.npz): encoder / decoder outputs and the joint
    logits 1e-5; every parameter gradient of the RNN-T loss (the loss and its logits gradient
    from oracle/rnnt_ref.py in both runs) 1e-4 of the tensor's max."""
    from oracle import rnnt_ref
    from oracle import transducer_ref as TR

    d = load("transducer.npz")
    params, buffers = _golden_params(d, "init.")
    leaf = {k: v.double().requires_grad_() for k, v in params.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in buffers.items()}
    hj, he, hd = TR.transducer_forward(d["xs"].double(), d["xlens"], d["ys"], d["ylens"], leaf, TRANSDUCER_GOLDEN,
                                       b64, True)
    assert rel(he, d["h_enc"]) < 1e-5 and rel(hd, d["h_dec"]) < 1e-5 and rel(hj, d["h_jnt"]) < 1e-5
    plen = O.pred_len(d["xlens"])
    loss, nll, dz = rnnt_ref.rnnt_batch(hj.detach().numpy(), d["ys"].clamp(min=0).numpy(), plen.numpy(),
                                        d["ylens"].numpy())
    assert abs(loss - d["loss"].item()) <= 1e-5 * abs(loss)
    hj.backward(torch.from_numpy(dz))
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, v in leaf.items():
        ref = d["grad." + k].double()
        g = v.grad if v.grad is not None else torch.zeros_like(v)
        assert (g - ref).abs().max().item() <= 1e-4 * max(ref.abs().max().item(), 1e-3 * gmax), k
