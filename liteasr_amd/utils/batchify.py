"""Minibatch policies over length-sorted utterances (liteasr/utils/batchify.py:12-159).

SeqBatch: the batch size of a minibatch is fixed by its FIRST (longest) utterance:
max(min_batch_size, int(batch_size / (1 + max(int(xlen / max_len_in), int(ylen / max_len_out))))).
FrameBatch: a minibatch closes when (utterances + 1) * max length would exceed
max_frame_in / max_frame_out / max_frame_inout."""

from typing import List, Sequence


class BatchifyPolicy(object):
    def __init__(self, dataset_cfg):
        self._num = 0
        self.data: List[List[int]] = []
        self.minibatch: List[int] = []
        self.dataset_cfg = dataset_cfg
        self.sample = None

    @property
    def empty(self) -> bool:
        return len(self.minibatch) == 0

    @property
    def full(self) -> bool:
        raise NotImplementedError

    def push(self, idx):
        raise NotImplementedError

    def refresh(self):
        raise NotImplementedError

    def pop(self):
        self.data.append(self.minibatch)
        self._num += len(self.minibatch)
        self.minibatch = []

    def batchify(self, indices: Sequence[int], samples):
        assert len(indices) == len(samples), f"{len(samples)}"
        self.refresh()
        for idx in indices:
            self.sample = samples[idx]
            if self.full:
                self.pop()
                self.refresh()
            self.push(idx)
        if not self.empty:
            self.pop()
            self.refresh()

    def __getitem__(self, index):
        return self.data[index]

    def __len__(self):
        return len(self.data)


class SeqBatch(BatchifyPolicy):
    @property
    def full(self):
        return len(self.minibatch) == self.dynamic_batch_size

    def push(self, idx):
        first = self.empty
        self.minibatch.append(idx)
        if first:
            self.refresh()

    def refresh(self):
        c = self.dataset_cfg
        if self.empty:
            self.factor, self.dynamic_batch_size, self.max_ilen, self.max_olen = 0, c.batch_size, 0, 0
        else:
            self.max_ilen, self.max_olen = self.sample.xlen, self.sample.ylen
            self.factor = max(int(self.max_ilen / c.max_len_in), int(self.max_olen / c.max_len_out))
            self.dynamic_batch_size = max(c.min_batch_size, int(c.batch_size / (1 + self.factor)))


class FrameBatch(BatchifyPolicy):
    @property
    def full(self):
        c = self.dataset_cfg
        mi = max(self.max_ilen, self.sample.xlen)
        mo = max(self.max_olen, self.sample.ylen)
        n = len(self.minibatch) + 1
        if c.max_frame_in and mi * n > c.max_frame_in:
            return True
        if c.max_frame_out and mo * n > c.max_frame_out:
            return True
        return bool(c.max_frame_inout and (mi + mo) * n > c.max_frame_inout)

    def push(self, idx):
        self.minibatch.append(idx)
        self.refresh()

    def refresh(self):
        if self.empty:
            self.max_ilen = self.max_olen = 0
        else:
            self.max_ilen = max(self.max_ilen, self.sample.xlen)
            self.max_olen = max(self.max_olen, self.sample.ylen)
