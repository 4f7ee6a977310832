"""Generate golden vectors by running the *reference* (/root/reference, imported through
refshim) in the build container.  Outputs small .npz fixtures next to this script;
those fixtures (data only) are what the tests and the GPU box use.

    python tests/golden/make_golden.py

Fixtures
  relshift.npz    rel_shift (attention.py:99-118) on random score matrices, T = 1..9
  lengths.npz     get_pred_len (u2.py:319-321) and the subsampled-mask length
                  (transformer_encoder.py:117-120) for xlen = 1..1100
  ctc.npz         HybridCTCLoss with ctc_weight=1 (pure CTC, reduction sum / B) on fixed
                  logits: loss + d loss / d logits; repeated labels, L_b = 0, infeasible
  kl.npz          HybridCTCLoss with ctc_weight=0 (label-smoothed KL), loss + grad
  loader/         16-utt synthetic Kaldi data dir (FM ark + CM ark, feats.scp with the
                  placeholder @DIR@, utt2num_frames, text, vocab.txt) written by the
                  reference's kaldiio.save_ark; loader.npz = the reference AudioFileDataset's
                  batch composition and collated (xs, xlens, ys, ylens) for SeqBatch/FrameBatch
                  configs, plus load_mat of every entry (FM and CM)
  u2_step.npz     tiny U2 (d 32, 2 enc / 1 dec, V 20, F 40): seed-42 init state_dict, a
                  batch, h_attn / h_ctc / loss / grads, params after clip(5) + Noam step,
                  BN running stats; plus a chunk-mask (stage 4) forward for config 4
  decode.npz      tiny U2 (d 64, ff 256, 2 enc / 1 dec, V 30, F 40; seed-42 init, CTC / output projections scaled
                  x6 so the posteriors are peaked) in eval mode on 3 single utterances:
                  the reference's CTC log-probs, _ctc_prefix_beam_search n-best (token
                  sequences + scores), ctc_prefix_beam_search / attention_rescore /
                  attention (beam 10) results (u2.py:163-317)
  ctc_large.npz   SURVEY §8(c) F-c sizes: HybridCTCLoss(ctc_weight=1) on seeded logits at
                  (T' 249, B 4, V 4233, L <= 40) and (T' 999, B 2, V 4233, L <= 150): loss,
                  per-utterance loss, and the logits gradient on the blank + label columns
                  (+16 random columns) for every frame; the logits are regenerated from
                  their torch.Generator seed (a checksum is stored to detect drift)
  host_policies.npz  SeqBatch / FrameBatch grouping of synthetic length lists (incl. the
                  oversize-utterance edge), Trigger firing sequences, Vocab lookups
  decode_cache.npz tiny U2 with two decoder layers: the reference's attention beam search
                  step by step (hyps fed to forward_one_step, the log-probs it returned,
                  the best hypothesis): pins its never-reordered decoder cache
  u2_variants.npz the tiny U2 of u2_step with the other encoders the reference builds
                  (transformer layers with absolute / relative PE, conformer with absolute
                  PE or ReLU): init state_dict, outputs, loss and every gradient
  transducer.npz  tiny Transducer (Conformer encoder, LSTM decoder, joint): init state_dict,
                  batch (one empty transcript), encoder / decoder outputs, joint logits and every
                  gradient of the RNN-T loss (oracle/rnnt_ref.py) backpropagated through the
                  reference model
  spec_aug.npz    the reference SpecAugment (utils/transform/spec_augment.py) on seeded
                  inputs: global random/numpy seeds per case, input regenerated from its own
                  PCG64 seed, the augmented output, and one random.random() /
                  numpy.random.rand() draw taken after the case (pins RNG consumption)
"""

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402
from inputs import CTC_LARGE_CASES, ctc_large_inputs  # noqa: E402  (shared with the tests)

refshim.install()

from liteasr.criterions.hybrid_ctc_attn import HybridCTCLoss  # noqa: E402
from liteasr.models.u2 import U2, DecoderArch, EncoderArch  # noqa: E402
from liteasr.nets.attention import RelativeMultiHeadAttention  # noqa: E402
from liteasr.utils.mask import padding_mask, triangle_mask  # noqa: E402


def save(name, **arrs):
    out = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrs.items()}
    np.savez_compressed(os.path.join(HERE, name), **out)
    print("wrote", name, sum(a.nbytes for a in out.values()), "bytes")


def gen_relshift():
    g = torch.Generator().manual_seed(0)
    mha = RelativeMultiHeadAttention(1, 4, 0.0)
    arrs = {}
    for T in range(1, 10):
        x = torch.randn(2, 3, T, T, generator=g)
        arrs[f"in_{T}"] = x
        arrs[f"out_{T}"] = mha.rel_shift(x)
    save("relshift.npz", **arrs)


def gen_lengths():
    xl = torch.arange(1, 1101)
    m = U2.__new__(U2)
    pl = U2.get_pred_len(m, xl)
    sub = []
    for x in xl.tolist():
        T = max(x, 3)
        mask = padding_mask(torch.tensor([x, T]))[:1]  # width max(x, T)
        mm = mask[:, :-2:2][:, :-2:2]
        sub.append(int((~mm).sum()))
    tri = triangle_mask(8, stage=2).to(torch.uint8)
    tri2 = triangle_mask(3, 5, diagonal=2).to(torch.uint8)
    save("lengths.npz", xlen=xl, pred_len=pl, sub_valid=np.array(sub), tri_8_s2=tri, tri_3_5_d2=tri2)


class _FakeModel:
    """Feeds fixed logits into the reference criterion (it only calls these)."""

    def __init__(self, h_attn, h_ctc, V):
        self.h_attn, self.h_ctc = h_attn, h_ctc
        self.ignore, self.eos = -1, V - 1

    def __call__(self, xs, xlens, ys, ylens):
        return self.h_attn, self.h_ctc

    def get_pred_len(self, xlens):
        return U2.get_pred_len(self, xlens)

    def get_target(self, ys, ylens):
        return U2.get_target(self, ys, ylens)


def _crit(V, w, s=0.1):
    return HybridCTCLoss(types.SimpleNamespace(vocab_size=V, padding_idx=-1, smoothing=s,
                                               normalize_length=False, ctc_weight=w))


def gen_ctc_kl():
    g = torch.Generator().manual_seed(1)
    B, Tx, V, L = 4, 210, 30, 12
    T = ((Tx - 1) // 2 - 1) // 2  # 51
    xlens = torch.tensor([210, 190, 150, 40])
    ylens = torch.tensor([12, 7, 0, 11])  # utt 3: 40 frames -> 8 CTC frames < needed: infeasible
    ys = torch.randint(1, V - 1, (B, L), generator=g)
    ys[0, 3] = ys[0, 2]  # repeated label
    ys[0, 4] = ys[0, 2]
    ys = ys.masked_fill(padding_mask(ylens) if ylens.max() == L else torch.zeros(B, L, dtype=torch.bool), -1)
    for b in range(B):
        ys[b, ylens[b]:] = -1
    h_ctc = (torch.randn(B, T, V, generator=g) * 2).requires_grad_()
    h_attn = torch.zeros(B, L + 1, V)
    loss = _crit(V, 1.0)(_FakeModel(h_attn, h_ctc, V), None, xlens, ys, ylens)
    fin = torch.isfinite(loss)
    save("ctc.npz", xlens=xlens, ys=ys, ylens=ylens, h_ctc=h_ctc.detach(), loss=loss.detach(),
         finite=fin)
    # finite subset for gradients
    keep = torch.tensor([0, 1, 2])
    h2 = h_ctc.detach()[keep].clone().requires_grad_()
    l2 = _crit(V, 1.0)(_FakeModel(h_attn[keep], h2, V), None, xlens[keep], ys[keep], ylens[keep])
    l2.backward()
    save("ctc_grad.npz", xlens=xlens[keep], ys=ys[keep], ylens=ylens[keep], h_ctc=h2.detach(),
         loss=l2.detach(), grad=h2.grad)
    # label-smoothed KL (ctc_weight = 0)
    h_attn = (torch.randn(B, L + 1, V, generator=g) * 3).requires_grad_()
    h_ctc0 = torch.zeros(B, T, V)
    l3 = _crit(V, 0.0)(_FakeModel(h_attn, h_ctc0, V), None, xlens.clone().fill_(210), ys, ylens)
    l3.backward()
    save("kl.npz", ys=ys, ylens=ylens, h_attn=h_attn.detach(), loss=l3.detach(), grad=h_attn.grad)


def gen_ctc_large():
    arrs = {}
    for name, Tp, B, V, L, seed in CTC_LARGE_CASES:
        xlens, ys, ylens, h = ctc_large_inputs(Tp, B, V, L, seed)
        hr = h.clone().requires_grad_()
        loss = _crit(V, 1.0)(_FakeModel(torch.zeros(B, L + 1, V), hr, V), None, xlens, ys, ylens)
        loss.backward()
        per = []
        for b in range(B):
            lb = _crit(V, 1.0)(_FakeModel(torch.zeros(1, L + 1, V), h[b:b + 1].clone(), V), None,
                               xlens[b:b + 1], ys[b:b + 1], ylens[b:b + 1])
            per.append(float(lb))
        g = torch.Generator().manual_seed(seed + 1000)
        lab = sorted(set([0] + [int(v) for v in ys[ys >= 0].tolist()]))
        extra = torch.randperm(V, generator=g)[:16].tolist()
        cols = np.array(sorted(set(lab + extra)), dtype=np.int64)
        arrs[f"{name}_dims"] = np.array([Tp, B, V, L, seed])
        arrs[f"{name}_xlens"] = xlens
        arrs[f"{name}_ys"] = ys
        arrs[f"{name}_ylens"] = ylens
        arrs[f"{name}_logit_sum"] = h.double().sum()
        arrs[f"{name}_logit_head"] = h.reshape(-1)[:64]
        arrs[f"{name}_loss"] = loss.detach()
        arrs[f"{name}_loss_per_utt"] = np.array(per)
        arrs[f"{name}_cols"] = cols
        arrs[f"{name}_grad_cols"] = hr.grad[:, :, cols]
    save("ctc_large.npz", **arrs)


def gen_host_policies():
    from liteasr.dataclass.vocab import Vocab
    from liteasr.utils.batchify import FrameBatch, SeqBatch
    from liteasr.utils.trigger import Trigger

    rng = np.random.default_rng(5)
    arrs = {}
    xl = sorted(rng.integers(20, 900, size=40).tolist(), reverse=True)
    xl[3] = 2000  # alone over the frame budgets below -> the oversize edge
    xl = sorted(xl, reverse=True)
    yl = rng.integers(1, 60, size=40).tolist()
    samples = [types.SimpleNamespace(xlen=int(a), ylen=int(b)) for a, b in zip(xl, yl)]
    arrs["xlen"], arrs["ylen"] = np.array(xl), np.array(yl)
    cfgs = [("seq", dict(batch_size=8, min_batch_size=1, max_len_in=400, max_len_out=30)),
            ("seq", dict(batch_size=5, min_batch_size=2, max_len_in=800, max_len_out=100)),
            ("seq", dict(batch_size=3, min_batch_size=3, max_len_in=100, max_len_out=10)),
            ("frame", dict(max_frame_in=1500, max_frame_out=None, max_frame_inout=None)),
            ("frame", dict(max_frame_in=None, max_frame_out=120, max_frame_inout=None)),
            ("frame", dict(max_frame_in=3000, max_frame_out=200, max_frame_inout=2600))]
    for ci, (kind, c) in enumerate(cfgs):
        pol = (SeqBatch if kind == "seq" else FrameBatch)(types.SimpleNamespace(**c))
        pol.batchify(list(range(len(samples))), samples)
        comp = [list(pol[b]) for b in range(len(pol))]
        arrs[f"c{ci}_sizes"] = np.array([len(b) for b in comp])
        arrs[f"c{ci}_idx"] = np.array(sum(comp, []))
    # Trigger: which (counter, unit) pokes fire, for a few interval/unit pairs
    pokes = [(e, i, u) for e in range(0, 4) for i in range(0, 12) for u in ("iteration", "epoch")]
    for ti, (interval, unit) in enumerate([(1, "epoch"), (2, "epoch"), (3, "iteration"), (5, "iteration")]):
        fired = []
        trig = Trigger(interval, unit)
        ev = trig(lambda: fired.append(1))
        for k, (e, i, u) in enumerate(pokes):
            n0 = len(fired)
            ev(types.SimpleNamespace(epoch=e, iter=i), u)
            if len(fired) > n0:
                fired[-1] = k
        arrs[f"trig{ti}_fired"] = np.array(fired, dtype=np.int64)
    arrs["pokes"] = np.array([[e, i, 0 if u == "iteration" else 1] for e, i, u in pokes])
    v = Vocab(os.path.join(HERE, "loader", "vocab.txt"))
    arrs["vocab_conv"] = np.array(list(v.lookup(list(range(len(v))), convert=True)))
    arrs["vocab_tokens"] = np.array(list(v.lookup(list(range(len(v))))))
    save("host_policies.npz", **arrs)


def tiny_cfg(**kw):
    c = dict(enc_arch=EncoderArch.Conformer, use_rel=True, input_dim=40, enc_dim=32, enc_ff_dim=64,
             enc_attn_heads=4, enc_layers=2, activation="swish", dec_arch=DecoderArch.Transformer,
             vocab_size=20, dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=1, dropout_rate=0.0,
             enc_dropout_rate=0.0, enc_pos_dropout_rate=0.0, enc_attn_dropout_rate=0.0,
             enc_ff_dropout_rate=0.0, dec_dropout_rate=0.0, dec_pos_dropout_rate=0.0,
             dec_self_attn_dropout_rate=0.0, dec_src_attn_dropout_rate=0.0, dec_ff_dropout_rate=0.0)
    c.update(kw)
    return types.SimpleNamespace(**c)


def gen_u2_step():
    torch.manual_seed(42)
    model = U2(tiny_cfg())
    model.train()
    init = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
    g = torch.Generator().manual_seed(3)
    B, Tx, L, V = 3, 120, 6, 20
    xlens = torch.tensor([120, 113, 97])
    xs = torch.randn(B, Tx, 40, generator=g).masked_fill(padding_mask(xlens).unsqueeze(-1), 0.0)
    ylens = torch.tensor([6, 4, 2])
    ys = torch.randint(1, V - 1, (B, L), generator=g).masked_fill(padding_mask(ylens), -1)
    crit = _crit(V, 0.3)
    rec = {}

    class _Rec:  # one forward only (BN running stats must be updated exactly once)
        def __call__(self, *a):
            rec["out"] = model(*a)
            return rec["out"]

        def get_pred_len(self, xl):
            return model.get_pred_len(xl)

        def get_target(self, y, yl):
            return model.get_target(y, yl)

    loss = crit(_Rec(), xs, xlens, ys, ylens)
    h_attn, h_ctc = rec["out"]
    loss.backward()
    grads = {"grad." + n: p.grad.clone() for n, p in model.named_parameters()}
    norm = torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0)
    opt = torch.optim.Adam(model.parameters(), lr=1.0, betas=(0.9, 0.98), eps=1e-9)
    step, dim, warm = 1, 32, 25000
    lr = 1.0 * dim ** -0.5 * min(step ** -0.5, step * warm ** -1.5)  # liteasr/optims/noam.py:41-46
    for grp in opt.param_groups:
        grp["lr"] = lr
    opt.step()
    after = {"new." + k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
    # config-4 composition: chunk mask (stage 4) passed straight to the layers
    torch.manual_seed(42)
    m2 = U2(tiny_cfg())
    m2.train()
    enc = m2.encoder
    xmask = padding_mask(xlens)
    x = enc.pe(enc.embed(xs))
    km = xmask[:, :-2:2][:, :-2:2]
    Tp = km.shape[1]
    cm = km[:, None, None, :] | triangle_mask(Tp, stage=4)[None, None]
    for layer in enc.enc_layers:
        x = layer(x, mask=cm)
    h_chunk = enc.after_norm(x[0])
    save("u2_step.npz", xs=xs, xlens=xlens, ys=ys, ylens=ylens, h_attn=h_attn.detach(),
         h_ctc=h_ctc.detach(), loss=loss.detach(), grad_norm=norm, lr=np.array(lr), h_enc_chunk4=h_chunk.detach(),
         **{"init." + k: v for k, v in init.items()}, **grads, **after)


def gen_decode():
    torch.manual_seed(42)
    model = U2(tiny_cfg(enc_dim=64, dec_dim=64, enc_ff_dim=256, dec_ff_dim=256, vocab_size=30))
    with torch.no_grad():
        model.ctc.ctc_lo.weight.mul_(6.0)
        model.decoder.linear_out.weight.mul_(6.0)
    model.eval()
    # u2.py:283-288 hands _preprocess plain lists for xlens / ylens, which it cannot take
    # (mask.py:24 AttributeError, u2.py:356 TypeError); wrap it so the lists become int64
    # tensors -- the only change, the rest of attention_rescore runs as written.
    _pp = model._preprocess
    model._preprocess = lambda xs, xlens, ys, ylens: _pp(
        xs, torch.as_tensor(xlens, dtype=torch.long), ys, torch.as_tensor(ylens, dtype=torch.long))
    state = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
    g = torch.Generator().manual_seed(11)
    arrs = {}
    with torch.no_grad():
        for u, T in enumerate((120, 97, 64)):
            x = torch.randn(1, T, 40, generator=g)
            hyps, h = model._ctc_prefix_beam_search(x)
            logp = model.ctc.log_softmax(h).squeeze(0)
            arrs[f"u{u}.x"] = x[0]
            arrs[f"u{u}.ctc_logp"] = logp
            arrs[f"u{u}.enc"] = h[0]
            n = len(hyps)
            lens = np.array([len(hh[0]) for hh in hyps], dtype=np.int64)
            flat = np.array([t for hh in hyps for t in hh[0]], dtype=np.int64)
            arrs[f"u{u}.nbest_len"] = lens
            arrs[f"u{u}.nbest_tok"] = flat
            arrs[f"u{u}.nbest_score"] = np.array([hh[1] for hh in hyps], dtype=np.float64)
            arrs[f"u{u}.nbest_n"] = np.array(n)
            arrs[f"u{u}.ctc_best"] = np.array(model.ctc_prefix_beam_search(x), dtype=np.int64)
            arrs[f"u{u}.rescore_best"] = np.array(model.attention_rescore(x), dtype=np.int64)
            arrs[f"u{u}.attn_best"] = np.array(model.attention(x), dtype=np.int64)
    save("decode.npz", n_utt=np.array(3), **arrs, **{"init." + k: v for k, v in state.items()})


def gen_loader():
    import shutil
    import tempfile

    from liteasr.dataclass.vocab import Vocab
    from liteasr.dataset.asr_dataset import AudioFileDataset
    from liteasr.utils.kaldiio import load_mat, save_ark

    rng = np.random.default_rng(11)
    out_dir = os.path.join(HERE, "loader")
    shutil.rmtree(out_dir, ignore_errors=True)
    os.makedirs(out_dir)
    chars = [chr(ord("a") + i) for i in range(20)]
    with open(os.path.join(out_dir, "vocab.txt"), "w") as f:
        f.write("<unk> 1\n")
        for i, ch in enumerate(chars):
            f.write(f"{ch} {i + 2}\n")
    F = 20
    utts = {}
    lens = rng.integers(30, 121, size=16)
    lens[5] = lens[9]  # a tie: the length sort must be stable
    for i, T in enumerate(lens):
        utts[f"utt{i:02d}"] = (rng.standard_normal((int(T), F)) * 2 + 0.5).astype(np.float32)
    texts = {}
    for i, k in enumerate(utts):
        L = int(rng.integers(1, 16))
        t = "".join(rng.choice(chars + ["z"], size=L))  # 'z' is out of vocab -> <unk>
        texts[k] = t
    tmp = tempfile.mkdtemp()
    arrs = {}
    for tag, cm in (("fm", None), ("cm", 2)):
        ark = os.path.join(out_dir, f"feats_{tag}.ark")
        scp = os.path.join(tmp, f"{tag}.scp")
        save_ark(ark, utts, scp=scp, compression_method=cm)
        lines = open(scp).read().replace(out_dir, "@DIR@")
        open(os.path.join(out_dir, f"feats_{tag}.scp"), "w").write(lines)
        for line in open(scp):
            k, p = line.split()
            arrs[f"mat_{tag}_{k}"] = load_mat(p)
    with open(os.path.join(out_dir, "utt2num_frames"), "w") as f:
        for k, v in utts.items():
            f.write(f"{k} {v.shape[0]}\n")
    with open(os.path.join(out_dir, "text"), "w") as f:
        for k, t in texts.items():
            f.write(f"{k} {t}\n")
    # run the reference dataset on a resolved copy
    data = os.path.join(tmp, "data")
    os.makedirs(data)
    for fn in ("utt2num_frames", "text"):
        shutil.copy(os.path.join(out_dir, fn), data)
    vocab = Vocab(os.path.join(out_dir, "vocab.txt"))
    cfgs = [dict(batch_count="seq", batch_size=4, min_batch_size=1, max_len_in=60, max_len_out=10),
            dict(batch_count="seq", batch_size=6, min_batch_size=2, max_len_in=100, max_len_out=8),
            dict(batch_count="frame", max_frame_in=300, max_frame_out=None, max_frame_inout=None),
            dict(batch_count="frame", max_frame_in=None, max_frame_out=30, max_frame_inout=350)]
    pp = types.SimpleNamespace(workflow=[], spec_aug=None)
    for tag in ("fm", "cm"):
        lines = open(os.path.join(out_dir, f"feats_{tag}.scp")).read().replace("@DIR@", out_dir)
        open(os.path.join(data, "feats.scp"), "w").write(lines)
        for ci, c in enumerate(cfgs):
            full = dict(batch_count="seq", batch_size=None, min_batch_size=None, max_len_in=None, max_len_out=None,
                        max_frame_in=None, max_frame_out=None, max_frame_inout=None)
            full.update(c)
            ds = AudioFileDataset("train", data, None, types.SimpleNamespace(**full), pp, vocab)
            comp = [list(ds.batchify_policy[b]) for b in range(len(ds))]
            arrs[f"{tag}_c{ci}_batch_sizes"] = np.array([len(b) for b in comp])
            arrs[f"{tag}_c{ci}_batch_idx"] = np.array(sum(comp, []))
            for b in range(len(ds)):
                xs, xl, ys, yl = ds.collator([ds[b]])
                if ci == 0:
                    arrs[f"{tag}_c{ci}_b{b}_xs"] = xs
                else:  # same matrices, other grouping: shape + exact float64 sum suffice
                    arrs[f"{tag}_c{ci}_b{b}_xs_shape"] = np.array(xs.shape)
                    arrs[f"{tag}_c{ci}_b{b}_xs_sum"] = xs.double().sum()
                arrs[f"{tag}_c{ci}_b{b}_xlens"] = xl
                arrs[f"{tag}_c{ci}_b{b}_ys"] = ys
                arrs[f"{tag}_c{ci}_b{b}_ylens"] = yl
    arrs["vocab_len"] = np.array(len(vocab))
    arrs["lookup_all"] = np.array(vocab.lookup("".join(chars) + "z?"))
    shutil.rmtree(tmp)
    save("loader.npz", **arrs)


SPEC_AUG_CASES = [
    # name, cfg overrides, lengths (one call per utterance, in order), F
    ("default_t600", {}, [600], 80),
    ("default_t161", {}, [161], 80),
    ("nowarp_t160", {}, [160], 80),
    ("short_t50", {}, [50], 80),
    ("tiny_t3", {}, [3], 80),
    ("multi_zero", dict(freq_mask_times=2, time_mask_times=3, replace_with_zero=True), [400], 80),
    ("multi_mean", dict(freq_mask_times=3, time_mask_times=2, time_warp=40), [333], 80),
    ("copy_f40", dict(inplace=False, freq_mask=10, time_mask=30, time_warp=5), [97], 40),
    ("batch4", {}, [300, 250, 200, 170], 80),
]


def gen_spec_aug():
    import random

    from liteasr.config import _SpecAugmentConfig
    from liteasr.utils.transform.spec_augment import SpecAugment

    arrs = {}
    for ci, (name, over, lens, F) in enumerate(SPEC_AUG_CASES):
        cfg = _SpecAugmentConfig(**over)
        sa = SpecAugment(cfg)
        random.seed(1000 + ci)
        np.random.seed(2000 + ci)
        for ui, t in enumerate(lens):
            x = np.random.default_rng(3000 + 10 * ci + ui).standard_normal((t, F)).astype(np.float32)
            x[:, :5] += 4.0  # non-zero mean so the mean fill is visible
            arrs[f"{name}_u{ui}_out"] = sa(torch.from_numpy(x.copy())).numpy()
        arrs[f"{name}_cfg"] = np.array([cfg.time_warp, cfg.freq_mask, cfg.freq_mask_times, cfg.time_mask,
                                        cfg.time_mask_times, int(cfg.inplace), int(cfg.replace_with_zero)])
        arrs[f"{name}_lens"] = np.array(lens)
        arrs[f"{name}_F"] = np.array(F)
        arrs[f"{name}_seeds"] = np.array([1000 + ci, 2000 + ci, 3000 + 10 * ci])
        arrs[f"{name}_next_random"] = np.array(random.random())
        arrs[f"{name}_next_numpy"] = np.array(np.random.rand())
    arrs["cases"] = np.array([c[0] for c in SPEC_AUG_CASES])
    save("spec_aug.npz", **arrs)


def gen_paraformer():
    """Tiny Paraformer (d 64, 2 enc / 1 dec, V 20, F 40) through the reference's model and
    ParaformerLoss: seed-42 init state_dict, a batch, python-random seed for the glancing
    sampler, every intermediate the oracle restates (encoder output, alpha, h_cif,
    sum_alpha, first-pass argmax, replace map), hs_attn, loss and every gradient."""
    import random

    from liteasr.criterions.paraformer_loss import ParaformerLoss
    from liteasr.models.paraformer import Paraformer

    cfg = types.SimpleNamespace(dropout_rate=0.0, use_rel=True, input_dim=40, enc_dim=64, enc_ff_dim=128,
                                enc_attn_heads=4, enc_dropout_rate=0.0, enc_pos_dropout_rate=0.0,
                                enc_attn_dropout_rate=0.0, enc_ff_dropout_rate=0.0, enc_layers=2,
                                activation="swish", sample_ratio=0.75, vocab_size=20, dec_dim=64, dec_ff_dim=128,
                                dec_attn_heads=4, dec_dropout_rate=0.0, dec_self_attn_dropout_rate=0.0,
                                dec_src_attn_dropout_rate=0.0, dec_ff_dropout_rate=0.0, dec_layers=1,
                                pos_dropout_rate=0.0)
    arrs = {}
    for case, (seed, xl, yl) in enumerate([(3, [120, 113, 97], [6, 4, 2]), (4, [160, 160, 131, 90], [9, 7, 9, 3])]):
        torch.manual_seed(42)
        model = Paraformer(cfg)
        model.train()
        init = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe") and k != "pe.pe"}
        g = torch.Generator().manual_seed(seed)
        xlens = torch.tensor(xl)
        B, Tx, L, V = len(xl), max(xl), max(yl), 20
        xs = torch.randn(B, Tx, 40, generator=g).masked_fill(padding_mask(xlens).unsqueeze(-1), 0.0)
        ylens = torch.tensor(yl)
        ys = torch.randint(1, V - 1, (B, L), generator=g).masked_fill(padding_mask(ylens), -1)
        rec = {}
        pred_fwd = model.predictor.forward

        def pred_hook(xs_, xlens_=None, ylens_=None):
            rec["h_enc"] = xs_.detach().clone()
            out = pred_fwd(xs_, xlens_, ylens_)
            rec["h_cif"] = out[0].detach().clone()
            return out

        model.predictor.forward = pred_hook
        samp_fwd = model.sampler.forward

        def samp_hook(hs, embed_ys, ys_, ys_hat, ylens_):
            rec["ys_hat"] = ys_hat.clone()
            st = random.getstate()
            out = samp_fwd(hs, embed_ys, ys_, ys_hat, ylens_)
            random.setstate(st)  # replay the same draws to record the replace map
            rep = torch.zeros_like(ys_, dtype=torch.bool)
            dist = (ys_hat != ys_).sum(-1)
            num = torch.ceil(model.sampler.sample_ratio * dist).long()
            for b in range(ys_.size(0)):
                rep[b][random.sample(range(ylens_[b]), num[b])] = True
            rec["replace"] = rep
            return out

        model.sampler.forward = samp_hook
        crit = ParaformerLoss(types.SimpleNamespace(vocab_size=V, gamma=1.0))

        class _Rec:
            def __call__(self, *a):
                rec["out"] = model(*a)
                return rec["out"]

            def get_target(self, y, yl):
                return model.get_target(y, yl)

        random.seed(100 + case)
        loss = crit(_Rec(), xs, xlens, ys, ylens)
        hs_attn, sum_alpha = rec["out"]
        loss.backward()
        pre = f"c{case}."
        arrs.update({pre + "xs": xs, pre + "xlens": xlens, pre + "ys": ys, pre + "ylens": ylens,
                     pre + "random_seed": np.array(100 + case), pre + "hs_attn": hs_attn.detach(),
                     pre + "sum_alpha": sum_alpha.detach(), pre + "loss": loss.detach(),
                     pre + "h_enc": rec["h_enc"], pre + "h_cif": rec["h_cif"], pre + "ys_hat": rec["ys_hat"],
                     pre + "replace": rec["replace"]})
        arrs.update({pre + "grad." + n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
        if case == 0:
            arrs.update({"init." + k: v for k, v in init.items()})
    save("paraformer.npz", **arrs)


def gen_transducer():
    """Tiny Transducer (liteasr/models/transducer.py; Conformer encoder d 64 x 2 with relative
    PE and Swish, LSTM decoder dec_dim 16 / 48 units x 2 layers, joint 24, V 20, F 40), seed-42
    init state_dict, a batch with an empty transcript: the encoder output, the decoder
    output, the joint logits h_jnt (B, T', Lmax+1, V) and every parameter gradient of the
    RNN-T loss backpropagated through the REFERENCE model.  The loss and its logits
    gradient come from oracle/rnnt_ref.py (the reference's loss is the absent warp-transducer
    package, rnnt.py:28,33: that part is unpinned; the model forward / backward is the
    reference's own)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import rnnt_ref
    from liteasr.models.transducer import DecoderArch as TDA
    from liteasr.models.transducer import EncoderArch as TEA
    from liteasr.models.transducer import Transducer

    cfg = types.SimpleNamespace(joint_dim=24, dropout_rate=0.0, enc_arch=TEA.Conformer, use_rel=True, input_dim=40,
                                enc_dim=64, enc_ff_dim=128, enc_attn_heads=4, enc_dropout_rate=0.0,
                                enc_pos_dropout_rate=0.0, enc_attn_dropout_rate=0.0, enc_ff_dropout_rate=0.0,
                                enc_layers=2, activation="swish", dec_arch=TDA.LSTM, vocab_size=20, dec_dim=16,
                                dec_units=48, dec_dropout_rate=0.0, dec_layers=2)
    torch.manual_seed(42)
    model = Transducer(cfg)
    model.train()
    init = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
    g = torch.Generator().manual_seed(5)
    xl, yl = [120, 97, 64], [5, 3, 0]
    xlens, ylens = torch.tensor(xl), torch.tensor(yl)
    B, Tx, L, V = 3, max(xl), max(yl), 20
    xs = torch.randn(B, Tx, 40, generator=g).masked_fill(padding_mask(xlens).unsqueeze(-1), 0.0)
    ys = torch.randint(1, V, (B, L), generator=g).masked_fill(padding_mask(ylens), -1)
    rec = {}
    enc_fwd, dec_fwd = model.encoder.forward, model.decoder.forward
    model.encoder.forward = lambda *a, **k: rec.setdefault("h_enc", enc_fwd(*a, **k))
    model.decoder.forward = lambda *a, **k: rec.setdefault("h_dec", dec_fwd(*a, **k))
    h_jnt = model(xs, xlens, ys, ylens)
    plen = model.get_pred_len(xlens)
    loss, nll, dz = rnnt_ref.rnnt_batch(h_jnt.detach().double().numpy(), ys.clamp(min=0).numpy(), plen.numpy(),
                                        ylens.numpy())
    h_jnt.backward(torch.from_numpy(dz).float())
    arrs = {"xs": xs, "xlens": xlens, "ys": ys, "ylens": ylens, "h_enc": rec["h_enc"].detach(),
            "h_dec": rec["h_dec"].detach(), "h_jnt": h_jnt.detach(), "loss": np.array(loss), "nll": nll}
    arrs.update({"init." + k: v for k, v in init.items()})
    arrs.update({"grad." + n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    save("transducer.npz", **arrs)


def gen_decode_cache():
    """decode_cache.npz: the reference's attention beam search (u2.py:163-216) with TWO
    decoder layers, where its forward_one_step cache matters: the cache is never reordered
    with the hypotheses, so layers >= 1 attend to the previous step's row order.  Per
    utterance: the input, every step's hyps fed to forward_one_step and the log-probs it
    returned, and the best hypothesis."""
    torch.manual_seed(42)
    model = U2(tiny_cfg(enc_dim=64, dec_dim=64, enc_ff_dim=256, dec_ff_dim=256, vocab_size=30, dec_layers=2))
    with torch.no_grad():
        model.decoder.linear_out.weight.mul_(6.0)
    model.eval()
    state = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
    g = torch.Generator().manual_seed(13)
    arrs = {"n_utt": np.array(2)}
    step = model.decoder.forward_one_step
    with torch.no_grad():
        for u, T in enumerate((120, 80)):
            x = torch.randn(1, T, 40, generator=g)
            trace = []

            def rec(y, mask, memory, memory_mask, cache, _step=step, _t=trace):
                logp, new = _step(y, mask, memory, memory_mask, cache)
                _t.append((y.clone(), logp.clone()))
                return logp, new

            model.decoder.forward_one_step = rec
            best = model.attention(x)
            model.decoder.forward_one_step = step
            arrs[f"u{u}.x"] = x[0]
            arrs[f"u{u}.steps"] = np.array(len(trace))
            for i, (y, lp) in enumerate(trace):
                arrs[f"u{u}.hyps{i}"] = y
                arrs[f"u{u}.logp{i}"] = lp
            arrs[f"u{u}.attn_best"] = np.array(best, dtype=np.int64)
    save("decode_cache.npz", **arrs, **{"init." + k: v for k, v in state.items()})


# encoder variants the reference's U2 builds besides the default conformer + relative PE +
# Swish (liteasr/nets/transformer_encoder.py:47-100): name -> U2Config overrides
U2_VARIANTS = {
    "tfm_abs": dict(enc_arch=EncoderArch.Transformer, use_rel=False),
    "tfm_rel": dict(enc_arch=EncoderArch.Transformer, use_rel=True),
    "cfm_abs_relu": dict(enc_arch=EncoderArch.Conformer, use_rel=False, activation="relu"),
    "cfm_rel_relu": dict(enc_arch=EncoderArch.Conformer, use_rel=True, activation="relu"),
}


def gen_u2_variants():
    """u2_variants.npz: per variant <name>.init.* (seed-42 state_dict), outputs, loss and every
    gradient of one hybrid-loss step (w 0.3) on the u2_step batch recipe."""
    arrs = {}
    for name, kw in U2_VARIANTS.items():
        torch.manual_seed(42)
        model = U2(tiny_cfg(**kw))
        model.train()
        init = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith(".pe.pe")}
        g = torch.Generator().manual_seed(3)
        B, Tx, L, V = 3, 120, 6, 20
        xlens = torch.tensor([120, 113, 97])
        xs = torch.randn(B, Tx, 40, generator=g).masked_fill(padding_mask(xlens).unsqueeze(-1), 0.0)
        ylens = torch.tensor([6, 4, 2])
        ys = torch.randint(1, V - 1, (B, L), generator=g).masked_fill(padding_mask(ylens), -1)
        rec = {}

        class _Rec:  # one forward only (BN running stats must be updated exactly once)
            def __call__(self, *a):
                rec["out"] = model(*a)
                return rec["out"]

            def get_pred_len(self, xl):
                return model.get_pred_len(xl)

            def get_target(self, y, yl):
                return model.get_target(y, yl)

        loss = _crit(V, 0.3)(_Rec(), xs, xlens, ys, ylens)
        h_attn, h_ctc = rec["out"]
        loss.backward()
        arrs.update({f"{name}.xs": xs, f"{name}.xlens": xlens, f"{name}.ys": ys, f"{name}.ylens": ylens,
                     f"{name}.h_attn": h_attn.detach(), f"{name}.h_ctc": h_ctc.detach(),
                     f"{name}.loss": loss.detach()})
        arrs.update({f"{name}.init.{k}": v for k, v in init.items()})
        arrs.update({f"{name}.grad.{n}": p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    save("u2_variants.npz", **arrs)


GENERATORS = dict(relshift=gen_relshift, lengths=gen_lengths, ctc_kl=gen_ctc_kl, u2_step=gen_u2_step,
                  decode=gen_decode, loader=gen_loader, spec_aug=gen_spec_aug, ctc_large=gen_ctc_large,
                  host_policies=gen_host_policies, paraformer=gen_paraformer, transducer=gen_transducer,
                  u2_variants=gen_u2_variants, decode_cache=gen_decode_cache)

if __name__ == "__main__":
    # python tests/golden/make_golden.py [name ...]   (default: all)
    torch.set_num_threads(4)
    for name in sys.argv[1:] or list(GENERATORS):
        GENERATORS[name]()
