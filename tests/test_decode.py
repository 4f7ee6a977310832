"""Inference searches (liteasr/models/u2.py:160-317).

CPU: the Python restatement (oracle/decode_ref.py) reproduces the reference's n-best
exactly on the reference's own CTC log-probs (tests/golden/decode.npz, made by
tests/golden/make_golden.py::gen_decode), and the native C++ prefix beam search
(libliteasr_decode.so) matches both bit for bit (token sequences and double scores),
also on random flat / peaked posteriors with ties in the sort.
GPU: lasr_logsoftmax_topk against torch fp32, and the full U2 decode methods on the
golden tiny model against the reference's results.
"""

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import decode_ref as R  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "decode.npz")


def _gold():
    return np.load(GOLD)


def _nbest(d, u):
    lens, toks, sc = d[f"u{u}.nbest_len"], d[f"u{u}.nbest_tok"], d[f"u{u}.nbest_score"]
    out, o = [], 0
    for n, s in zip(lens, sc):
        out.append((toks[o:o + n].tolist(), float(s)))
        o += n
    return out


def _topk(logp, k):
    v = np.empty((logp.shape[0], k), np.float32)
    i = np.empty((logp.shape[0], k), np.int32)
    for t in range(logp.shape[0]):
        v[t], i[t] = R.topk_desc(logp[t], k)
    return v, i


@pytest.mark.parametrize("u", [0, 1, 2])
def test_oracle_prefix_beam_matches_reference(u):
    d = _gold()
    got = R.ctc_prefix_beam_search(d[f"u{u}.ctc_logp"], beam=10)
    assert got == _nbest(d, u)
    assert got[0][0] == d[f"u{u}.ctc_best"].tolist()


@pytest.mark.parametrize("u", [0, 1, 2])
def test_native_prefix_beam_matches_reference(u):
    from liteasr_amd import decoding as D

    d = _gold()
    v, i = _topk(d[f"u{u}.ctc_logp"], 10)
    assert D.prefix_beam_search(v, i, beam=10) == _nbest(d, u)


@pytest.mark.parametrize("seed,T,V,beam,temp", [(0, 60, 30, 10, 1.0), (1, 80, 12, 4, 0.2),
                                                (2, 40, 50, 10, 4.0), (3, 1, 5, 3, 1.0),
                                                (4, 120, 8, 8, 0.05)])
def test_native_prefix_beam_matches_oracle(seed, T, V, beam, temp):
    from liteasr_amd import decoding as D

    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((T, V)) / temp).astype(np.float32)
    logp = (x - np.log(np.exp(x.astype(np.float64)).sum(-1, keepdims=True))).astype(np.float32)
    v, i = _topk(logp, beam)
    assert D.prefix_beam_search(v, i, beam=beam) == R.ctc_prefix_beam_search(logp, beam=beam)


def test_native_prefix_beam_ties_and_empty():
    from liteasr_amd import decoding as D

    # identical candidate log-probs: ordering decided by insertion order + stable sort
    logp = np.log(np.full((6, 4), 0.25, np.float32))
    v, i = _topk(logp, 4)
    assert D.prefix_beam_search(v, i, beam=4) == R.ctc_prefix_beam_search(logp, beam=4)
    # T = 0: the single empty hypothesis with score 0
    e = np.zeros((0, 3), np.float32)
    assert D.prefix_beam_search(e, e.astype(np.int32), beam=3) == [([], 0.0)]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_rescore_pick_matches_oracle(seed):
    """Host half of attention rescoring: gathered log-probs -> best index, as the oracle's
    restatement of u2.py:300-315 (incl. ties: first strict maximum wins)."""
    from liteasr_amd import decoding as D

    rng = np.random.default_rng(seed)
    n, V, eos = 10, 12, 11
    hyps = [(rng.integers(1, V - 1, rng.integers(0, 7)).tolist(), float(rng.normal() * 3)) for _ in range(n)]
    if seed == 2:
        hyps[3] = hyps[1]  # exact tie: the earlier one wins
    L1 = max(len(t) for t, _ in hyps) + 1
    attn = np.log(rng.dirichlet(np.ones(V), size=(n, L1))).astype(np.float32)
    g = np.full((n, L1), -np.inf, np.float32)
    for i, (t, _) in enumerate(hyps):
        for j, w in enumerate(t + [eos]):
            g[i, j] = attn[i, j, w]
    assert D.pick_best(hyps, g) == R.rescore_pick(hyps, attn, eos)


# ------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_logsoftmax_topk_kernel(dtype):
    from liteasr_amd import kernels as K

    g = torch.Generator().manual_seed(5)
    rows, V, k = 37, 4233, 10
    x = (torch.randn(rows, V + 7, generator=g) * 3).to(dtype)[:, :V].cuda()
    gi = torch.randint(-2, V + 2, (rows,), generator=g, dtype=torch.int32).cuda()
    vals, idx, gat = K.logsoftmax_topk(x, k, gather_idx=gi)
    ref = torch.log_softmax(x.float().cpu(), -1)
    rv, ri = torch.sort(ref, dim=-1, descending=True, stable=True)  # ties -> smaller index
    rv, ri = rv[:, :k], ri[:, :k]
    torch.cuda.synchronize()
    assert torch.equal(idx.cpu().long(), ri), "top-k ids"
    assert torch.allclose(vals.cpu(), rv, atol=2e-6, rtol=0)
    gic = gi.cpu().long()
    ok = (gic >= 0) & (gic < V)
    exp = torch.full((rows,), -float("inf"))
    exp[ok] = ref[ok.nonzero()[:, 0], gic[ok]]
    assert torch.equal(torch.isinf(gat.cpu()), ~ok)
    assert torch.allclose(gat.cpu()[ok], exp[ok], atol=2e-6, rtol=0)
    # strided row subset (the attention beam's last-position rows)
    v2, i2, _ = K.logsoftmax_topk(x[2:], 3, rows=5, ld=7 * x.stride(0))
    sel = torch.arange(5) * 7 + 2
    rv2, ri2 = torch.sort(ref[sel], dim=-1, descending=True, stable=True)
    rv2, ri2 = rv2[:, :3], ri2[:, :3]
    assert torch.equal(i2.cpu().long(), ri2)
    assert torch.allclose(v2.cpu(), rv2, atol=2e-6, rtol=0)


def _golden_model():
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    d = _gold()
    c = U2Config(input_dim=40, vocab_size=30, enc_dim=64, enc_ff_dim=256, enc_attn_heads=4, enc_layers=2,
                 dec_dim=64, dec_ff_dim=256, dec_attn_heads=4, dec_layers=1, compute_dtype="fp32")
    resolve_self(c)
    m = U2(c)
    sd = {k[5:]: torch.from_numpy(np.array(v)) for k, v in d.items() if k.startswith("init.")}
    m.load_state_dict(sd, strict=False)
    return m.cuda().eval(), d


@pytest.mark.gpu
def test_u2_decode_against_reference():
    model, d = _golden_model()
    for u in range(int(d["n_utt"])):
        x = torch.from_numpy(d[f"u{u}.x"]).unsqueeze(0).cuda()
        hyps, h = model._ctc_prefix_beam_search(x)
        torch.cuda.synchronize()
        assert torch.allclose(h[0].float().cpu(), torch.from_numpy(d[f"u{u}.enc"]), atol=1e-4, rtol=0)
        ref = _nbest(d, u)
        assert [list(t) for t, _ in hyps] == [t for t, _ in ref], f"utt {u} n-best tokens"
        assert np.allclose([s for _, s in hyps], [s for _, s in ref], atol=1e-4, rtol=0)
        assert list(model.ctc_prefix_beam_search(x)) == d[f"u{u}.ctc_best"].tolist()
        assert list(model.attention_rescore(x)) == d[f"u{u}.rescore_best"].tolist()
        assert list(model.inference(x)) == d[f"u{u}.rescore_best"].tolist()
        assert list(model.attention(x)) == d[f"u{u}.attn_best"].tolist()


@pytest.mark.gpu
def test_attention_beam_decoder_cache_against_reference():
    """The attention beam search with TWO decoder layers (tests/golden/decode_cache.npz, the
    reference's own u2.py:163-216 run step by step): at every step the hypotheses fed to the
    decoder are the reference's, and the top-k log-probs of the KV-cached decoder step equal
    the reference's forward_one_step log-probs (its never-reordered cache of layers >= 1
    included) within 1e-4; the best hypothesis is identical.  fp32 build."""
    from liteasr_amd import decoding as D
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    d = np.load(os.path.join(os.path.dirname(GOLD), "decode_cache.npz"))
    c = U2Config(input_dim=40, vocab_size=30, enc_dim=64, enc_ff_dim=256, enc_attn_heads=4, enc_layers=2,
                 dec_dim=64, dec_ff_dim=256, dec_attn_heads=4, dec_layers=2, compute_dtype="fp32")
    resolve_self(c)
    m = U2(c)
    sd = {k[5:]: torch.from_numpy(np.array(v)) for k, v in d.items() if k.startswith("init.")}
    m.load_state_dict(sd, strict=False)
    m = m.cuda().eval()
    for u in range(int(d["n_utt"])):
        x = torch.from_numpy(d[f"u{u}.x"]).unsqueeze(0).cuda()
        trace = []
        with torch.no_grad():
            best = D.attention_beam_search(m, x, beam=10, trace=trace)
        assert best == d[f"u{u}.attn_best"].tolist(), u
        assert len(trace) == int(d[f"u{u}.steps"]), (u, len(trace))
        for i, (hyps, vals) in enumerate(trace):
            assert np.array_equal(hyps, d[f"u{u}.hyps{i}"]), (u, i)
            ref = np.sort(d[f"u{u}.logp{i}"], axis=-1)[:, ::-1][:, :10]
            assert np.allclose(vals, ref, atol=1e-4, rtol=0), (u, i, np.abs(vals - ref).max())


@pytest.mark.gpu
def test_graphed_encode_matches_eager():
    """hipGraph-replayed batch-1 encoder == eager launches, bit for bit, across replays with
    new contents and after a weight update (re-capture)."""
    from liteasr_amd import decoding as D

    model, d = _golden_model()
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for it in range(3):
            x = torch.randn(1, 100, 40, generator=g).cuda()
            he, Te = D.encode(model, x, graph=False)
            he = he.clone()
            hg, Tg = D.encode(model, x, graph=True)
            torch.cuda.synchronize()
            assert Te == Tg and torch.equal(he, hg), it
            if it == 1:  # weight update -> new flat version -> re-capture
                model.ctc.ctc_lo.weight.mul_(1.0)
                model.encoder.after_norm.weight.add_(0.01)
    # a train()/eval() switch re-captures: BatchNorm uses batch statistics in train mode
    x = torch.randn(2, 100, 40, generator=g).cuda()
    with torch.no_grad():
        for mode in (True, False, True):
            model.train(mode)
            he, _ = D.encode(model, x, graph=False)
            he = he.clone()
            hg, _ = D.encode(model, x, graph=True)
            torch.cuda.synchronize()
            assert torch.equal(he, hg), mode
    model.eval()
