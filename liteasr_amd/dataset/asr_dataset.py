"""Feature dataset with length-sorted minibatches (liteasr/dataset/asr_dataset.py:24-155).

Behaviour kept from the reference: utterances are read from feats.scp / utt2num_frames /
text in file order; ``batchify`` sorts indices by frame count (descending, stable) and
groups them with SeqBatch/FrameBatch; ``dataset[i]`` is the i-th minibatch (a list of
Audio records); ``collator`` pads xs with 0 and ys with -1 and returns int64 lengths.

MI355X-side difference: the collator decodes the whole minibatch with one native call
(lasr_ark_read_padded) straight into the padded float32 batch instead of loading and
padding utterance by utterance.  With a device-capable postprocess (SpecAugment) the
collator only draws the augmentation plan and returns it as a fifth element; the trainer
applies it to the batch on the GPU.  (The reference's ``memory_save`` pickle dump of
batches is not carried over: it serialises Python objects to disk and is not on the step
path.)
"""

import logging
from typing import List, Optional

import numpy as np
import torch

from ..dataclass.audio_data import Audio
from ..dataclass.sheet import AudioSheet, TextSheet
from ..utils.batchify import FrameBatch, SeqBatch
from ..utils.kaldiio import read_padded
from ..utils.transform import PostProcess
from .liteasr_dataset import LiteasrDataset

logger = logging.getLogger(__name__)


class AudioFileDataset(LiteasrDataset):
    def __init__(self, split: str, data_dir: str, delimiter: Optional[str], dataset_cfg, postprocess_cfg, vocab,
                 keep_raw=False, memory_save=False):
        super().__init__()
        if memory_save:
            raise NotImplementedError("memory_save (pickled batch dumps) is not supported")
        self.split = split
        self.data: List[Audio] = []
        self.batchify_policy = None
        self.postprocess = None
        if postprocess_cfg is not None:
            self.set_postprocess(postprocess_cfg)
        audios = AudioSheet(data_dir)
        texts = TextSheet(data_dir, vocab=vocab, delimiter=delimiter)
        assert len(audios) == len(texts)
        for (uttid, fd, start, shape), (uttid_t, ids, text) in zip(audios, texts):
            assert uttid_t == uttid
            self.data.append(Audio(fd, start, shape, ids, text if keep_raw else None))
        self.feat_dim = self.data[0].x.shape[-1]
        if dataset_cfg is not None:
            self.batchify(dataset_cfg)

    def batchify(self, dataset_cfg):
        if dataset_cfg.batch_count == "seq":
            policy = SeqBatch
        elif dataset_cfg.batch_count == "frame":
            policy = FrameBatch
        else:
            logger.error(f"unsupport strategy {dataset_cfg.batch_count}")
            raise ValueError
        self.batchify_policy = policy(dataset_cfg)
        order = sorted(range(len(self.data)), key=lambda i: self.data[i].xlen, reverse=True)
        self.batchify_policy.batchify(order, self.data)

    def set_postprocess(self, postprocess_cfg):
        self.postprocess = PostProcess(postprocess_cfg)

    @property
    def train(self):
        return self.split == "train"

    def collator(self, samples: List[List[Audio]]):
        batch = samples[0]
        B = len(batch)
        xlens = torch.tensor([s.xlen for s in batch], dtype=torch.long)
        ylens = torch.tensor([s.ylen for s in batch], dtype=torch.long)
        post = self.postprocess if (self.train and self.postprocess is not None and len(self.postprocess)) else None
        plan = None
        if post is not None and post.device_capable:
            # draw the augmentation here (same RNG order as the reference's per-utterance
            # calls); the pixels are produced on the GPU by the trainer (apply_batch)
            plan = post.plan_batch(xlens.tolist(), self.feat_dim)
            post = None
        if post is None and all(s.start is None for s in batch):
            tmax = int(xlens.max()) if B else 0
            xs = torch.empty(B, tmax, self.feat_dim, dtype=torch.float32)
            _, lens = read_padded([s.fd for s in batch], tmax, self.feat_dim, out=xs.numpy())
            if not np.array_equal(lens, xlens.numpy()):
                raise ValueError("feature frame counts disagree with utt2num_frames")
        else:
            xs = [post(s.x) if post is not None else s.x for s in batch]
            xs = torch.nn.utils.rnn.pad_sequence(xs, batch_first=True, padding_value=0)
        lmax = int(ylens.max()) if B else 0
        ys = torch.full((B, lmax), -1, dtype=torch.long)
        for i, s in enumerate(batch):
            if s.ylen:
                ys[i, : s.ylen] = torch.tensor(s.tokenids, dtype=torch.long)
        if plan is not None:
            return xs, xlens, ys, ylens, plan
        return xs, xlens, ys, ylens

    def __getitem__(self, index):
        if self.batchify_policy is not None:
            return [self.data[i] for i in self.batchify_policy[index]]
        return self.data[index]

    def __len__(self):
        return len(self.batchify_policy) if self.batchify_policy is not None else len(self.data)
