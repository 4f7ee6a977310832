"""Trainer.run end to end on the GPU through the CLI path (liteasr/train.py:46-101 ->
liteasr/trainer.py:130-172): a user config tree composed and prepared like the CLI does,
the reference-decoded loader fixture (tests/golden/loader/, transcripts cut to 4 characters
so every utterance is CTC-feasible), task/model/optimizer/criterion built by
``build_trainer``, then ``Trainer.run`` with its events.

The loop is checked against the oracle: the batches the criterion saw during the first
iterations are replayed through oracle/u2_oracle.train_step chained from the same initial
weights (fp64, Adam+Noam state carried), and every recorded loss must match; the run must
also leave the CLI's artefacts (train.log with the loss lines, .hydra/, the epoch checkpoint).
"""

import logging
import os
import sys

import pytest
import torch

from cfgtree import user_tree
from oracle import u2_oracle as O

pytestmark = pytest.mark.gpu

TRIGGERS = ["{name: report_loss, interval: 1, unit: iteration}", "{name: valid, interval: 1, unit: epoch}",
            "{name: save_model, interval: 1, unit: epoch}"]


@pytest.mark.parametrize("dtype,tol", [("fp32", 2e-5), ("bf16", 5e-3)])
def test_trainer_run_matches_oracle_chain(tmp_path, monkeypatch, dtype, tol):
    from liteasr_amd import train as T

    conf, data = user_tree(tmp_path, max_iter=6, max_chars=4, triggers=TRIGGERS, compute_dtype=dtype)
    monkeypatch.chdir(tmp_path)
    root = logging.getLogger()
    saved = root.handlers[:], root.level
    try:
        cfg, run_dir = T.prepare(["-cd", str(conf)])
        tr = T.build_trainer(cfg)
        model = tr._model
        p0 = {k: v.detach().double().cpu().clone() for k, v in model.named_parameters()}
        b0 = {k: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()
              for k, v in model.named_buffers() if not k.endswith(".pe.pe")}
        seen = []
        crit = tr.criterion

        def recording(m, xs, xlens, ys, ylens):
            loss = crit(m, xs, xlens, ys, ylens)
            if m.training:
                seen.append((float(loss.detach()), xs.detach().cpu().double(), xlens.cpu(), ys.cpu(), ylens.cpu()))
            return loss

        tr.criterion = recording
        tr.run()
        torch.cuda.synchronize()
        assert tr.iter == 6 and tr.skipped == 0 and len(seen) == 6

        mc = cfg.model
        cfg_o = O.default_cfg(enc_dim=mc.enc_dim, enc_heads=mc.enc_attn_heads, enc_ff=mc.enc_ff_dim,
                              enc_layers=mc.enc_layers, dec_dim=mc.dec_dim, dec_heads=mc.dec_attn_heads,
                              dec_ff=mc.dec_ff_dim, dec_layers=mc.dec_layers, vocab_size=mc.vocab_size,
                              input_dim=mc.input_dim)
        params, bufs, st = p0, b0, None
        for i, (loss, xs, xl, ys, yl) in enumerate(seen):
            loss_o, _, params, st, _ = O.train_step(params, bufs, (xs, xl, ys, yl), cfg_o, ctc_weight=0.3,
                                                    smoothing=0.1, clip=5.0, opt_state=st, model_dim=64)
            assert abs(loss - loss_o.item()) <= tol * abs(loss_o.item()), (i, loss, loss_o.item())

        # the CLI's artefacts: logs (rank 0, Hydra's file handler), run config, checkpoint
        for h in root.handlers:
            h.flush()
        log = open(os.path.join(run_dir, "train.log")).read()
        assert log.count("current loss") == 6 and "valid loss" in log, log[-2000:]
        assert os.path.exists(os.path.join(run_dir, ".hydra", "config.yaml"))
        ck = os.path.join(run_dir, "ckpts", "model.ep.1.pt")
        sd = torch.load(ck, map_location="cpu", weights_only=True)
        assert set(k for k in sd if not k.endswith(".pe.pe")) >= set(p0)
    finally:
        for h in root.handlers[:]:
            if h not in saved[0]:
                root.removeHandler(h)
                h.close()
        root.setLevel(saved[1])


def test_trainer_run_spec_augment_nan_skip_and_log_format(tmp_path, monkeypatch):
    """The train split's collator draws SpecAugment plans on the host (reference RNG order),
    ``lasr_spec_augment`` applies them on the device inside the loop, a NaN loss skips its
    optimizer step without counting an iteration, and the log lines keep the reference's
    format (trainer.py:150-209)."""
    import random
    import re

    import numpy as np

    from liteasr_amd import train as T

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_spec_aug import _check, _to_oracle_plan
    from oracle import spec_augment_ref as SO

    pp = ("{workflow: [spec_aug], spec_aug: {time_warp: 5, freq_mask: 4, freq_mask_times: 2, time_mask: 8, "
          "time_mask_times: 2, inplace: true, replace_with_zero: false}}")
    conf, data = user_tree(tmp_path, max_iter=5, max_chars=4, triggers=TRIGGERS, postprocess=pp)
    monkeypatch.chdir(tmp_path)
    root = logging.getLogger()
    saved = root.handlers[:], root.level
    try:
        cfg, run_dir = T.prepare(["-cd", str(conf)])
        tr = T.build_trainer(cfg)
        post = tr._train_post
        applied = []
        inner_apply = post.apply_batch

        def recording_apply(xs, xlens, plan):
            x_in = xs.detach().cpu().clone()
            out = inner_apply(xs, xlens, plan)
            applied.append((x_in, xlens.cpu(), plan.cpu(), out.detach().cpu().clone()))
            return out

        post.apply_batch = recording_apply
        crit, calls = tr.criterion, []

        def nan_on_third(m, *batch):
            loss = crit(m, *batch)
            if m.training:
                calls.append(1)
                if len(calls) == 3:
                    loss = loss * float("nan")
            return loss

        tr.criterion = nan_on_third
        random.seed(123)
        np.random.seed(456)
        tr.run()
        torch.cuda.synchronize()
        assert tr.iter == 5 and tr.skipped == 1 and len(calls) == 6 and len(applied) == 6

        # plans: the oracle's independent draw from the same seeds, batch by batch, and the
        # device output against the oracle's apply (bit-exact outside the masks)
        random.seed(123)
        np.random.seed(456)
        sa_cfg = cfg.postprocess.spec_aug
        for bi, (x_in, xl, plan, out) in enumerate(applied):
            for u in range(x_in.shape[0]):
                t = int(xl[u])
                row = plan[u].numpy()
                assert SO.draw_plan(t, x_in.shape[2], sa_cfg) == _to_oracle_plan(row), (bi, u)
                ref = SO.apply_plan(x_in[u, :t].numpy(), _to_oracle_plan(row), False)
                _check(out[u, :t].numpy(), ref, row, f"batch {bi} utt {u}")

        for h in root.handlers:
            h.flush()
        log = open(os.path.join(run_dir, "train.log")).read().splitlines()
        loss_re = re.compile(r"^\[INFO\]\[liteasr_amd\.trainer\] - (\d+) / 5 iters, (\d+) / inf epochs - "
                             r"current loss: (\d+\.\d\d)$")
        iters = [int(m.group(1)) for m in map(loss_re.match, log) if m]
        assert iters == [1, 2, 3, 4, 5], log
        assert any("iteration 3 is skipped since gradient is NaN" in ln for ln in log)
        assert any(re.search(r"\] - 3 / 5 iters, 1 / inf epochs - valid loss: \d+\.\d\d$", ln) for ln in log), log
    finally:
        for h in root.handlers[:]:
            if h not in saved[0]:
                root.removeHandler(h)
                h.close()
        root.setLevel(saved[1])
