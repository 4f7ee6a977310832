"""A user config tree in the reference's own layout (liteasr/config/: config.yaml + one
``my_*`` file per plugin group extending the registered option, ``???`` for the values the
task fills), over a copy of the reference-decoded loader fixture (tests/golden/loader/)."""

import os
import shutil
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOADER = os.path.join(ROOT, "tests", "golden", "loader")


def data_dir(tmp_path, max_chars=None):
    """tests/golden/loader copied to tmp_path/data with feats.scp pointing at it.  With
    ``max_chars`` every transcript is cut to its first characters: the fixture's labels are
    longer than its shortest utterances' subsampled frames (CTC infeasible, loss inf), which
    a loader test does not care about and a training test does."""
    data = tmp_path / "data"
    shutil.copytree(LOADER, data)
    scp = (data / "feats_fm.scp").read_text().replace("@DIR@", str(data))
    (data / "feats.scp").write_text(scp)
    if max_chars is not None:
        lines = (data / "text").read_text().splitlines()
        cut = [f"{ln.split()[0]} {ln.split()[1][:max_chars]}" for ln in lines]
        (data / "text").write_text("\n".join(cut) + "\n")
    return data


def user_tree(tmp_path, model=None, max_iter=2, max_chars=None, triggers=None, compute_dtype=None,
              postprocess="{workflow: []}"):
    d = tmp_path / "conf"
    for g in ("model", "criterion", "optimizer", "task"):
        (d / g).mkdir(parents=True)
    trig = triggers or ["{name: report_loss, interval: 1, unit: iteration}"]
    (d / "config.yaml").write_text(textwrap.dedent("""\
        defaults:
          - liteasr_config
          - task: my_task
          - model: my_U2
          - criterion: my_hybrid_ctc
          - optimizer: my_noam
          - _self_
        common:
          seed: 7
          trigger:
        """) + "".join(f"    - {t}\n" for t in trig) + textwrap.dedent(f"""\
        dataset: {{batch_count: seq, batch_size: 4, min_batch_size: 1, max_len_in: 1000, max_len_out: 150}}
        postprocess: {postprocess}
        distributed: {{num_workers: 0}}
        optimization: {{max_epoch: -1, max_iter: {max_iter}, accum_grad: 1, clip_grad_norm: 5.0}}
        hydra:
          run:
            dir: runs/${{task.name}}_${{model.name}}
          job_logging:
            formatters: {{mine: {{format: '[%(levelname)s][%(name)s] - %(message)s'}}}}
            handlers: {{file: {{formatter: mine}}}}
        """))
    m = model or dict(enc_dim=64, enc_ff_dim=128, enc_attn_heads=4, enc_layers=2, dec_dim=64, dec_ff_dim=128,
                      dec_attn_heads=4, dec_layers=1, dropout_rate=0.0)
    if compute_dtype:
        m = dict(m, compute_dtype=compute_dtype)
    (d / "model" / "my_U2.yaml").write_text(
        "defaults:\n  - U2\nname: U2\ninput_dim: ???\nvocab_size: ???\n"
        + "".join(f"{k}: {v}\n" for k, v in m.items()) + "enc_dropout_rate: ${model.dropout_rate}\n")
    (d / "criterion" / "my_hybrid_ctc.yaml").write_text(
        "defaults:\n  - hybrid_ctc\nname: hybrid_ctc\nvocab_size: ???\nsmoothing: 0.1\nctc_weight: 0.3\n")
    (d / "optimizer" / "my_noam.yaml").write_text("defaults:\n  - noam\nname: noam\nmodel_dim: 64\n")
    data = data_dir(tmp_path, max_chars)
    (d / "task" / "my_task.yaml").write_text(
        f"defaults:\n  - asr\nname: asr\nvocab: {data / 'vocab.txt'}\ntrain: {data}\nvalid: {data}\n")
    return d, data
