"""Config composition and the training CLI's host side (liteasr/train.py:21-43, Hydra 1.1
semantics of the reference's config tree liteasr/config/), CPU only."""

import logging
import os
import pickle

import pytest
import yaml

from cfgtree import user_tree
from liteasr_amd.config.compose import (ConfigError, Node, compose, missing_keys, resolve,
                                        save_run_config)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = ["task=asr_kaldi", "model=conformer_small", "criterion=hybrid_ctc_w03", "optimizer=noam_d256"]


def test_presets_compose_schema_then_group_then_self():
    cfg = compose(overrides=GROUPS)
    # schema defaults survive where neither the preset nor config.yaml set them
    assert cfg.common.memory_save is False and cfg.distributed.backend == "NCCL"
    # config.yaml (_self_) over the schema
    assert cfg.common.seed == 42 and cfg.optimization.clip_grad_norm == 5.0
    assert [t.name for t in cfg.common.trigger] == ["report_loss", "valid", "save_model"]
    # the registered node under the preset: name + fields the preset does not mention
    assert cfg.model.name == "U2" and cfg.model.activation == "swish" and cfg.model.compute_dtype == "bf16"
    assert cfg.model.enc_dropout_rate == 0.1 and cfg.model.enc_ff_dropout_rate == 0.1
    assert cfg.criterion.name == "hybrid_ctc" and cfg.criterion.ctc_weight == 0.3
    assert cfg.optimizer.name == "noam" and cfg.optimizer.model_dim == 256
    # schema interpolations resolved (DistributedConfig.world_piece_size, InferenceConfig)
    assert cfg.distributed.world_piece_size == [1]
    assert cfg.inference.ckpt_path == "ckpts"
    assert cfg.run_cfg.dir == cfg.hydra.run.dir and cfg.job_logging_cfg == cfg.hydra.job_logging
    assert cfg.hydra.job_logging.handlers.file.filename == "train.log"


def test_group_option_extends_another_and_overrides():
    cfg = compose(overrides=["task=asr_kaldi", "model=conformer_large", "criterion=ctc_only",
                             "optimizer=noam_d256", "model.dropout_rate=0.2", "+common.extra=3",
                             "~postprocess.spec_aug", "dataset.batch_size=8"])
    m = cfg.model
    assert (m.enc_dim, m.enc_attn_heads, m.chunk_size, m.enc_layers) == (512, 16, 16, 12)
    assert m.dynamic_chunk is True and m.max_chunk == 25
    assert m.enc_dropout_rate == 0.2 and m.dec_pos_dropout_rate == 0.2 and m.enc_attn_dropout_rate == 0.0
    assert cfg.criterion.ctc_weight == 1.0 and cfg.criterion.smoothing == 0.1
    assert cfg.common.extra == 3 and "spec_aug" not in cfg.postprocess and cfg.dataset.batch_size == 8
    assert sorted(missing_keys(cfg)) == ["criterion.vocab_size", "inference.ckpt_name", "model.input_dim",
                                         "model.vocab_size", "task.train", "task.valid", "task.vocab"]


def test_registered_options_without_yaml():
    cfg = compose(overrides=["task=asr", "model=U2", "criterion=hybrid_ctc", "optimizer=adam"])
    assert cfg.model.name == "U2" and cfg.model.enc_layers == 12 and cfg.optimizer.name == "adam"


@pytest.mark.parametrize("ovr,msg", [
    (["model=U2", "criterion=hybrid_ctc", "optimizer=noam"], "You must specify 'task'"),
    (GROUPS[:1] + ["model=nope"] + GROUPS[2:], "registered model 'nope'"),
    (GROUPS + ["model.not_a_field=1"], r"use \+model.not_a_field"),
    (GROUPS + ["common.seed.x=1"], "not a config node"),
    (GROUPS + ["model.enc_dim"], "not key=value"),
    (GROUPS + ["+model.bad=${model.nowhere}"], "not found"),
])
def test_compose_errors(ovr, msg):
    with pytest.raises(ConfigError, match=msg):
        compose(overrides=ovr)


def test_interpolation_rules():
    root = {"a": {"b": 3, "s": "x${a.b}y", "whole": "${a.b}", "chain": "${a.whole}"},
            "l": ["${a.b}", {"k": "${a.chain}"}], "t": "${now:%Y}-${now:%Y}"}
    resolve(root)
    assert root["a"]["whole"] == 3 and root["a"]["s"] == "x3y" and root["a"]["chain"] == 3
    assert root["l"] == [3, {"k": 3}]
    y = root["t"].split("-")
    assert y[0] == y[1] and len(y[0]) == 4
    with pytest.raises(ConfigError, match="cycle"):
        resolve({"a": "${b}", "b": "${a}"})


def test_user_config_tree_in_reference_format(tmp_path):
    d, data = user_tree(tmp_path)
    cfg = compose(str(d), "config", ["optimizer.warmup=10"])
    assert cfg.common.seed == 7 and cfg.optimization.max_iter == 2
    assert cfg.model.enc_dim == 64 and cfg.model.input_dim == "???" and cfg.model.enc_dropout_rate == 0.0
    assert cfg.optimizer.warmup == 10 and cfg.optimizer.model_dim == 64 and cfg.task.vocab.endswith("vocab.txt")
    assert cfg.hydra.run.dir == "runs/asr_U2"
    # the job_logging override merged into Hydra's defaults, not replacing them
    assert cfg.hydra.job_logging.handlers.file.formatter == "mine"
    assert cfg.hydra.job_logging.handlers.file.filename == "train.log"


def test_prepare_writes_run_dir_and_logs(tmp_path, monkeypatch):
    from liteasr_amd import train as T

    d, data = user_tree(tmp_path)
    monkeypatch.chdir(tmp_path)
    root = logging.getLogger()
    saved = root.handlers[:], root.level
    try:
        cfg, run_dir = T.prepare(["-cd", str(d), "model.enc_layers=1"])
        assert run_dir == str(tmp_path / "runs" / "asr_U2") and os.getcwd() == run_dir
        job = yaml.safe_load(open(os.path.join(run_dir, ".hydra", "config.yaml")))
        assert job["model"]["enc_layers"] == 1 and "hydra" not in job
        assert yaml.safe_load(open(os.path.join(run_dir, ".hydra", "overrides.yaml"))) == ["model.enc_layers=1"]
        assert "hydra" not in cfg and cfg.run_cfg.dir == "runs/asr_U2"
        logging.getLogger("liteasr_amd.train").info("hello from the job")
        for h in root.handlers:
            h.flush()
        assert "[INFO][liteasr_amd.train] - hello from the job" in open(os.path.join(run_dir, "train.log")).read()
        # the task side of train(): datasets and model dims from the data, on the host
        from liteasr_amd import tasks

        task = tasks.setup_task(cfg.task)
        task.load_dataset("train", task.cfg.train, cfg.dataset, cfg.postprocess, False)
        model = task.build_model(cfg.model)
        assert cfg.model.input_dim == task.feat_dim == 20 and cfg.model.vocab_size == len(task.vocab)
        assert model.encoder is not None and os.path.isdir(os.path.join(run_dir, "ckpts"))
    finally:
        for h in root.handlers[:]:
            if h not in saved[0]:
                root.removeHandler(h)
                h.close()
        root.setLevel(saved[1])


def test_print_config_and_missing(tmp_path, capsys, monkeypatch):
    from liteasr_amd import train as T

    monkeypatch.chdir(tmp_path)
    assert T.prepare(GROUPS + ["--cfg", "job"]) == (None, None)
    out = yaml.safe_load(capsys.readouterr().out)
    assert out["model"]["enc_dim"] == 256 and "hydra" not in out
    with pytest.raises(ConfigError, match="task.vocab"):
        T.prepare(GROUPS)
    assert not os.path.exists(tmp_path / "outputs")


def test_node_roundtrip_and_call_func_without_gpu(caplog):
    from liteasr_amd.distributed import utils as du

    cfg = compose(overrides=GROUPS)
    back = pickle.loads(pickle.dumps(cfg))  # what mp.spawn ships to every rank
    assert back == cfg and back.model.enc_dim == 256
    save_dir = Node.wrap({"a": [{"b": 1}]})
    assert save_dir.a[0].b == 1 and save_dir.to_container() == {"a": [{"b": 1}]}
    assert du.get_rank() == -1 and du.get_world_size() == -1 and du.is_master()
    calls = []
    with caplog.at_level(logging.WARNING):
        du.call_func(calls.append, cfg)
    assert calls == [] and "no GPU" in caplog.text


def test_save_run_config(tmp_path):
    cfg = compose(overrides=GROUPS)
    save_run_config(cfg, str(tmp_path), GROUPS)
    job = yaml.safe_load(open(tmp_path / ".hydra" / "config.yaml"))
    assert job["criterion"]["ctc_weight"] == 0.3 and job["run_cfg"]["dir"] == cfg.hydra.run.dir
