"""Data contract against the reference's own outputs (tests/golden/loader.npz,
written by tests/golden/make_golden.py running the reference kaldiio / Vocab / AudioFileDataset
on the committed 16-utterance data dir tests/golden/loader/).  Everything here is bit-exact:
decoded feature values (FM and CM-compressed), vocabulary ids, the length-sorted SeqBatch /
FrameBatch grouping, and the collated (xs, xlens, ys, ylens)."""

import os
import shutil
import types

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
CFGS = [dict(batch_count="seq", batch_size=4, min_batch_size=1, max_len_in=60, max_len_out=10),
        dict(batch_count="seq", batch_size=6, min_batch_size=2, max_len_in=100, max_len_out=8),
        dict(batch_count="frame", max_frame_in=300, max_frame_out=None, max_frame_inout=None),
        dict(batch_count="frame", max_frame_in=None, max_frame_out=30, max_frame_inout=350)]


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "loader.npz"))


def _datadir(tmp, tag):
    src = os.path.join(GOLD, "loader")
    d = os.path.join(tmp, f"data_{tag}")
    os.makedirs(d, exist_ok=True)
    for fn in os.listdir(src):
        shutil.copy(os.path.join(src, fn), d)
    scp = open(os.path.join(d, f"feats_{tag}.scp")).read().replace("@DIR@", d)
    open(os.path.join(d, "feats.scp"), "w").write(scp)
    return d


def _dcfg(c):
    from liteasr_amd.config import DatasetConfig

    return DatasetConfig(**c)


@pytest.mark.parametrize("tag", ["fm", "cm"])
def test_load_mat_bit_exact(tmp_path, gold, tag):
    from liteasr_amd.utils.kaldiio import load_mat, load_scp

    d = _datadir(str(tmp_path), tag)
    scp = load_scp(os.path.join(d, "feats.scp"))
    assert len(scp) == 16
    for k, arr in scp.items():
        ref = gold[f"mat_{tag}_{k}"]
        assert arr.dtype == ref.dtype and arr.shape == ref.shape
        assert np.array_equal(arr.view(np.uint32), ref.view(np.uint32)), k
    # sliced access ("ark:off[a:b]" inclusive ranges, matio.py:291-325)
    first = open(os.path.join(d, "feats.scp")).readline().split()
    assert np.array_equal(load_mat(first[1] + "[2:5,1:3]"), gold[f"mat_{tag}_{first[0]}"][2:6, 1:4])


def test_vocab(gold):
    from liteasr_amd.dataclass.vocab import Vocab

    v = Vocab(os.path.join(GOLD, "loader", "vocab.txt"))
    assert len(v) == int(gold["vocab_len"]) and v.valid
    chars = "".join(chr(ord("a") + i) for i in range(20))
    assert np.array_equal(np.array(v.lookup(chars + "z?")), gold["lookup_all"])
    assert v[0] == "<blank>" and v["<sos/eos>"] == len(v) - 1


@pytest.mark.parametrize("tag", ["fm", "cm"])
@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_dataset_batches_and_collator(tmp_path, gold, tag, ci):
    from liteasr_amd.config import PostProcessConfig
    from liteasr_amd.dataclass.vocab import Vocab
    from liteasr_amd.dataset import AudioFileDataset

    d = _datadir(str(tmp_path), tag)
    vocab = Vocab(os.path.join(d, "vocab.txt"))
    ds = AudioFileDataset("train", d, None, _dcfg(CFGS[ci]), PostProcessConfig(workflow=[]), vocab)
    pre = f"{tag}_c{ci}"
    sizes = [len(ds.batchify_policy[b]) for b in range(len(ds))]
    assert sizes == gold[pre + "_batch_sizes"].tolist()
    assert sum((list(ds.batchify_policy[b]) for b in range(len(ds))), []) == gold[pre + "_batch_idx"].tolist()
    for b in range(len(ds)):
        xs, xl, ys, yl = ds.collator([ds[b]])
        g = f"{pre}_b{b}"
        assert xl.dtype == torch.int64 and ys.dtype == torch.int64 and yl.dtype == torch.int64
        assert torch.equal(xl, torch.from_numpy(gold[g + "_xlens"]))
        assert torch.equal(yl, torch.from_numpy(gold[g + "_ylens"]))
        assert torch.equal(ys, torch.from_numpy(gold[g + "_ys"]))
        if ci == 0:
            ref = torch.from_numpy(gold[g + "_xs"])
            assert xs.shape == ref.shape and torch.equal(xs.view(torch.int32), ref.view(torch.int32))
        else:
            assert list(xs.shape) == gold[g + "_xs_shape"].tolist()
            assert xs.double().sum().item() == float(gold[g + "_xs_sum"])


def test_read_padded_errors(tmp_path):
    from liteasr_amd.utils import kaldiio as K

    d = _datadir(str(tmp_path), "fm")
    ents = [ln.split()[1] for ln in open(os.path.join(d, "feats.scp"))]
    with pytest.raises(IOError, match="frames > tmax"):
        K.read_padded(ents[:2], 10, 20)
    with pytest.raises(IOError, match="columns"):
        K.read_padded(ents[:1], 200, 21)
    with pytest.raises(IOError, match="cannot open"):
        K.read_padded([os.path.join(d, "nope.ark") + ":0"], 10, 20)
    arr, lens = K.read_padded([], 5, 20)
    assert arr.shape == (0, 5, 20) and lens.shape == (0,)


def test_writer_roundtrip_all_formats(tmp_path):
    """Our writer (save_ark) -> native reader, every compression method, both endians."""
    from liteasr_amd.utils import kaldiio as K

    rng = np.random.default_rng(3)
    d = {f"u{i}": (rng.standard_normal((int(rng.integers(2, 40)), 7)) * 3).astype(np.float32) for i in range(5)}
    for endian in ("<", ">"):
        for m in (None, 1, 2, 3, 4, 5, 6, 7):
            ark, scp = str(tmp_path / f"a{m}.ark"), str(tmp_path / f"a{m}.scp")
            K.save_ark(ark, d, scp=scp, compression_method=m, endian=endian)
            got = dict(K.load_ark(ark, endian=endian))
            lazy = K.load_scp(scp, endian=endian)
            for k, v in d.items():
                assert got[k].shape == v.shape and np.array_equal(got[k], lazy[k])
                if m is None:
                    assert np.array_equal(got[k], v)
                elif m in (1, 2, 3, 5):  # lossy but close (auto-ranged methods)
                    assert np.abs(got[k] - v).max() <= (v.max() - v.min()) / 60 + 1e-6


def test_trainer_step_semantics():
    """Trainer.run plumbing (liteasr/trainer.py:130-172) on a CPU stand-in model: gradient
    accumulation, NaN-skip without an iteration count, iteration events, max_iter stop."""
    from liteasr_amd.config import LiteasrConfig
    from liteasr_amd.trainer import Trainer

    class DS(torch.utils.data.Dataset):
        def __init__(self, n):
            self.n = n

        def __len__(self):
            return self.n

        def __getitem__(self, i):
            return [i]

        def collator(self, s):
            i = s[0][0]
            x = torch.full((2, 3), float(i + 1))
            if i == 3:
                x[0, 0] = float("nan")
            return (x,)

    task = types.SimpleNamespace(dataset=lambda split: DS(6))
    model = torch.nn.Linear(3, 1)
    calls = {"step": 0, "events": 0}

    class Opt:
        def __init__(self, params):
            self.inner = torch.optim.SGD(list(params), lr=0.1)

        def step(self):
            calls["step"] += 1
            self.inner.step()

        def zero_grad(self):
            self.inner.zero_grad()

    cfg = LiteasrConfig()
    cfg.distributed.num_workers = 0
    cfg.optimization.accum_grad = 2
    cfg.optimization.max_iter = 2
    cfg.optimization.clip_grad_norm = 5.0
    cfg.common.trigger = [dict(name="count_event", interval=1, unit="iteration")]
    crit = lambda m, x: m(x).sum()  # noqa: E731
    tr = Trainer.__new__(Trainer)

    def count_event():
        calls["events"] += 1

    tr.count_event = count_event
    Trainer.__init__(tr, cfg, task, model, crit, Opt(model.parameters()), device="cpu")
    tr.train_iter.data_loader = torch.utils.data.DataLoader(DS(6), batch_size=1, shuffle=False,
                                                            collate_fn=DS(6).collator)
    tr.run()
    # batches 1,2 -> step (iter 1); 3,4 (contains NaN) -> skipped; 5,6 -> step (iter 2); stop
    assert tr.iter == 2 and tr.skipped == 1 and calls["step"] == 2 and calls["events"] == 2


def test_collator_with_default_spec_aug(tmp_path, gold):
    """PostProcessConfig with its default workflow ["spec_aug"] (config/__init__.py:54-56): the train
    collator returns the un-augmented batch plus one SpecAugment plan row per utterance,
    drawn in batch order; the valid split is not augmented."""
    import random

    from liteasr_amd.config import PostProcessConfig
    from liteasr_amd.dataclass.vocab import Vocab
    from liteasr_amd.dataset import AudioFileDataset
    from liteasr_amd.utils.transform.spec_augment import SpecAugment

    d = _datadir(str(tmp_path), "fm")
    vocab = Vocab(os.path.join(d, "vocab.txt"))
    from liteasr_amd.config import _SpecAugmentConfig

    pp = PostProcessConfig()
    assert pp.workflow == ["spec_aug"]
    # the fixture's features are narrow (F < the default freq_mask 27, which would make the
    # reference's randrange raise too): scale the mask sizes down
    pp.spec_aug = _SpecAugmentConfig(time_warp=5, freq_mask=3, time_mask=6)
    ds = AudioFileDataset("train", d, None, _dcfg(CFGS[0]), pp, vocab)
    random.seed(3)
    np.random.seed(4)
    out = ds.collator([ds[0]])
    assert len(out) == 5
    xs, xl, _, _, plan = out
    ref = torch.from_numpy(gold["fm_c0_b0_xs"])
    assert torch.equal(xs.view(torch.int32), ref.view(torch.int32))
    random.seed(3)
    np.random.seed(4)
    want = SpecAugment(pp.spec_aug).plan_batch(xl.tolist(), xs.shape[-1])
    assert plan.dtype == torch.int32 and torch.equal(plan, want)
    va = AudioFileDataset("valid", d, None, _dcfg(CFGS[0]), pp, vocab)
    assert len(va.collator([va[0]])) == 4
