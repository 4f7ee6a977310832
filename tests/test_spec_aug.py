"""SpecAugment: host plan drawing + the batched HIP kernel
(csrc/specaug.hip) against the reference's SpecAugment
(liteasr/utils/transform/spec_augment.py:14-125).

Pins:
* oracle/spec_augment_ref.resize_rows == Pillow Image.resize(BICUBIC) bit for bit (CPU,
  Pillow imported directly; skipped where Pillow is absent);
* tests/golden/spec_aug.npz: outputs of the reference SpecAugment itself on seeded inputs
  (tests/golden/make_golden.py gen_spec_aug), incl. the RNG state after each case.

Tolerance: warped pixels and untouched pixels are compared bit-exactly; mean-filled
pixels within 1e-6 absolute (the reference fills with numpy's float32 pairwise mean, we
sum in float64), zero-filled pixels exactly.
"""

import os
import random
import types

import numpy as np
import pytest
import torch

from oracle import spec_augment_ref as O
from liteasr_amd.utils.transform.spec_augment import SpecAugment

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spec_aug.npz")


def _cases():
    d = np.load(G)
    out = []
    for name in d["cases"]:
        name = str(name)
        c = d[f"{name}_cfg"]
        cfg = types.SimpleNamespace(time_warp=int(c[0]), freq_mask=int(c[1]), freq_mask_times=int(c[2]),
                                    time_mask=int(c[3]), time_mask_times=int(c[4]), inplace=bool(c[5]),
                                    replace_with_zero=bool(c[6]))
        seeds = d[f"{name}_seeds"]
        lens = [int(t) for t in d[f"{name}_lens"]]
        F = int(d[f"{name}_F"])
        xs = []
        for ui, t in enumerate(lens):
            x = np.random.default_rng(int(seeds[2]) + ui).standard_normal((t, F)).astype(np.float32)
            x[:, :5] += 4.0
            xs.append(x)
        outs = [d[f"{name}_u{ui}_out"] for ui in range(len(lens))]
        out.append(dict(name=name, cfg=cfg, seeds=seeds, xs=xs, outs=outs, F=F,
                        next_random=float(d[f"{name}_next_random"]), next_numpy=float(d[f"{name}_next_numpy"])))
    return out


CASES = _cases()


def _fill_region(row, t, F):
    """Boolean (t, F) map of pixels some mask wrote."""
    m = np.zeros((t, F), bool)
    nf, nt = int(row[2]), int(row[3])
    for k in range(nf + nt):
        lo, hi = int(row[4 + 2 * k]), int(row[5 + 2 * k])
        if k < nf:
            m[:, lo:hi] = True
        else:
            m[lo:hi] = True
    return m


def _check(got, ref, row, what):
    t, F = ref.shape
    assert got.shape == ref.shape, what
    m = _fill_region(row, t, F)
    assert np.array_equal(got[~m].view(np.uint32), ref[~m].view(np.uint32)), \
        f"{what}: unmasked pixels differ (max {np.abs(got[~m] - ref[~m]).max() if (~m).any() else 0})"
    if m.any():
        np.testing.assert_allclose(got[m], ref[m], rtol=0, atol=1e-6, err_msg=what)


def _to_oracle_plan(row):
    nf, nt = int(row[2]), int(row[3])
    warp = (int(row[0]), int(row[1])) if row[1] else None
    pairs = [(int(row[4 + 2 * k]), int(row[5 + 2 * k])) for k in range(nf + nt)]
    return warp, pairs[:nf], pairs[nf:]


def _draw_rows(case):
    sa = SpecAugment(case["cfg"])
    random.seed(int(case["seeds"][0]))
    np.random.seed(int(case["seeds"][1]))
    rows = [sa.plan(x.shape[0], case["F"]) for x in case["xs"]]
    return sa, rows


def test_bicubic_restatement_matches_pillow():
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(7)
    pairs = [(1, 1), (1, 7), (7, 1), (2, 3), (80, 1), (81, 1), (80, 160), (100, 37), (37, 100),
             (919, 999), (999, 919), (5, 5)]
    pairs += [(int(rng.integers(1, 400)), int(rng.integers(1, 400))) for _ in range(20)]
    for n_in, n_out in pairs:
        x = (rng.standard_normal((n_in, 24)) * 10).astype(np.float32)
        ref = np.asarray(Image.fromarray(x).resize((24, n_out), Image.BICUBIC))
        got = O.resize_rows(x, n_out)
        assert np.array_equal(ref.view(np.uint32), got.view(np.uint32)), (n_in, n_out)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_plan_and_oracle_match_reference_golden(case):
    """Host plan drawing consumes the RNG like the reference; the oracle applied to that
    plan reproduces the reference's output."""
    _, rows = _draw_rows(case)
    assert random.random() == case["next_random"]
    assert np.random.rand() == case["next_numpy"]
    # the oracle's own draw (independent restatement) yields the same plan
    random.seed(int(case["seeds"][0]))
    np.random.seed(int(case["seeds"][1]))
    for x, row in zip(case["xs"], rows):
        assert O.draw_plan(x.shape[0], case["F"], case["cfg"]) == _to_oracle_plan(row)
    for ui, (x, row, ref) in enumerate(zip(case["xs"], rows, case["outs"])):
        got = O.apply_plan(x, _to_oracle_plan(row), case["cfg"].replace_with_zero)
        _check(got, ref, row, f"{case['name']} u{ui}")


def test_collator_returns_plan_and_trainer_contract():
    """Device-capable postprocess: the collator draws plans in utterance order."""
    from liteasr_amd.utils.transform import PostProcess

    cfg = types.SimpleNamespace(workflow=["spec_aug"], spec_aug=CASES[-1]["cfg"])
    pp = PostProcess(cfg)
    assert pp.device_capable
    case = CASES[-1]
    random.seed(int(case["seeds"][0]))
    np.random.seed(int(case["seeds"][1]))
    plan = pp.plan_batch([x.shape[0] for x in case["xs"]], case["F"])
    _, rows = _draw_rows(case)
    assert plan.dtype == torch.int32 and np.array_equal(plan.numpy(), np.stack(rows))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_spec_aug_gpu_matches_reference_golden(case):
    sa, rows = _draw_rows(case)
    B = len(case["xs"])
    T = max(x.shape[0] for x in case["xs"]) + 3
    F = case["F"]
    xs = torch.zeros(B, T, F)
    for i, x in enumerate(case["xs"]):
        xs[i, : x.shape[0]] = torch.from_numpy(x)
        xs[i, x.shape[0]:] = 7.0  # padding rows must come back untouched
    xlens = torch.tensor([x.shape[0] for x in case["xs"]], dtype=torch.int64)
    plan = torch.from_numpy(np.stack(rows))
    out = sa.apply_batch(xs.cuda(), xlens.cuda(), plan.cuda()).cpu()
    torch.cuda.synchronize()
    for i, (row, ref) in enumerate(zip(rows, case["outs"])):
        t = ref.shape[0]
        _check(out[i, :t].numpy(), ref, row, f"{case['name']} u{i}")
        assert torch.equal(out[i, t:], xs[i, t:])


@pytest.mark.gpu
def test_spec_aug_gpu_per_utterance_call():
    """Reference interface: SpecAugment(cfg)(x) with x on the GPU, same RNG stream."""
    case = CASES[0]
    sa = SpecAugment(case["cfg"])
    random.seed(int(case["seeds"][0]))
    np.random.seed(int(case["seeds"][1]))
    got = sa(torch.from_numpy(case["xs"][0]).cuda())
    assert got.is_cuda
    assert random.random() == case["next_random"]
    random.seed(int(case["seeds"][0]))
    np.random.seed(int(case["seeds"][1]))
    row = sa.plan(case["xs"][0].shape[0], case["F"])
    _check(got.cpu().numpy(), case["outs"][0], row, "per-utterance")


@pytest.mark.gpu
@pytest.mark.parametrize("zero", [False, True])
def test_spec_aug_gpu_full_batch_vs_oracle(zero):
    """Config-2 sized batch (B 32, T 1000, F 80), several masks: every utterance against the
    oracle; rows past xlen untouched."""
    cfg = types.SimpleNamespace(time_warp=80, freq_mask=27, freq_mask_times=2, time_mask=100,
                                time_mask_times=2, inplace=True, replace_with_zero=zero)
    sa = SpecAugment(cfg)
    g = torch.Generator().manual_seed(5)
    B, T, F = 32, 1000, 80
    xlens = torch.randint(int(0.95 * T), T + 1, (B,), generator=g)
    xlens[0] = T
    xlens[1] = 150  # too short to warp
    xs = torch.randn(B, T, F, generator=g)
    for b in range(B):
        xs[b, int(xlens[b]):] = 0
    random.seed(11)
    np.random.seed(12)
    plan = sa.plan_batch(xlens.tolist(), F)
    out = sa.apply_batch(xs.cuda(), xlens.cuda(), plan.cuda()).cpu()
    for b in range(B):
        t = int(xlens[b])
        row = plan[b].numpy()
        ref = O.apply_plan(xs[b, :t].numpy(), _to_oracle_plan(row), zero)
        _check(out[b, :t].numpy(), ref, row, f"b{b}")
        assert torch.equal(out[b, t:], xs[b, t:])


@pytest.mark.gpu
def test_spec_aug_gpu_extreme_warps():
    """Hand-made plans hitting both tap paths of the warp kernel: LDS taps (<= 32) and the
    per-pixel fallback (segments shrunk > ~8x), equal-size (copy) segments, and t = Tmax."""
    cfg = types.SimpleNamespace(time_warp=80, freq_mask=27, freq_mask_times=1, time_mask=100,
                                time_mask_times=1, inplace=True, replace_with_zero=False)
    sa = SpecAugment(cfg)
    T, F = 800, 80
    warps = [(200, 3), (100, 700), (790, 10), (10, 790), (400, 400), (300, 301), (799, 1), (1, 799)]
    B = len(warps)
    g = torch.Generator().manual_seed(9)
    xs = torch.randn(B, T, F, generator=g) * 3
    xlens = torch.full((B,), T, dtype=torch.int64)
    plan = torch.zeros(B, sa.plan_stride, dtype=torch.int32)
    for b, (c, w) in enumerate(warps):
        plan[b, 0], plan[b, 1] = c, w
    plan[1, 2], plan[1, 4], plan[1, 5] = 1, 3, 20  # one freq mask on one utterance
    out = sa.apply_batch(xs.cuda(), xlens.cuda(), plan.cuda()).cpu()
    for b in range(B):
        row = plan[b].numpy()
        ref = O.apply_plan(xs[b].numpy(), _to_oracle_plan(row), False)
        _check(out[b].numpy(), ref, row, f"warp {warps[b]}")
