"""ASR task (liteasr/tasks/asr.py:23-98): vocabulary, feature datasets, model saving."""

import logging
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Union

from ..config import MISSING, LiteasrDataclass
from ..dataclass.vocab import Vocab
from ..dataset import AudioFileDataset
from . import LiteasrTask, register_task

logger = logging.getLogger(__name__)


@dataclass
class ASRConfig(LiteasrDataclass):
    vocab: str = field(default=MISSING)
    train: str = field(default=MISSING)
    valid: str = field(default=MISSING)
    test: List[str] = field(default_factory=list)
    delimiter: Optional[str] = field(default=None)
    save_dir: str = field(default="ckpts")


@register_task("asr", dataclass=ASRConfig)
class ASRTask(LiteasrTask):
    def __init__(self, cfg: ASRConfig):
        super().__init__(cfg)
        self.vocab = Vocab(cfg.vocab)
        self.save_dir = cfg.save_dir
        Path(self.save_dir).mkdir(parents=True, exist_ok=True)
        self.vocab_size = len(self.vocab)
        self.feat_dim = 0

    def load_dataset(self, split: str, data_dir: Union[str, list], dataset_cfg=None, postprocess_cfg=None,
                     memory_save: bool = False):
        assert split in ["train", "valid", "test"]

        def one(d):
            logger.info("loading {} data from {}".format(split, d))
            return AudioFileDataset(split=split, data_dir=d, delimiter=self.cfg.delimiter, dataset_cfg=dataset_cfg,
                                    postprocess_cfg=postprocess_cfg, vocab=self.vocab, keep_raw=split == "test",
                                    memory_save=memory_save)

        if isinstance(data_dir, str):
            self.datasets[split] = one(data_dir)
            self.feat_dim = self.datasets[split].feat_dim
        elif isinstance(data_dir, (list, tuple)):
            self.datasets[split] = [one(d) for d in data_dir]
            self.feat_dim = self.datasets[split][0].feat_dim
        else:
            raise TypeError("data_dir with type {} cannot be parsed".format(type(data_dir)))

    def inference(self, x, model):
        tokens = self.vocab.lookupi(model.inference(x), convert=True)
        return "".join(tokens) if self.cfg.delimiter is None else self.cfg.delimiter.join(tokens)

    def save_model(self, model_name: str, model):
        model.save(os.sep.join((self.save_dir, model_name)))
