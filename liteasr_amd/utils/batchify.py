"""Minibatch planning over length-sorted utterances (policies of liteasr/utils/batchify.py).

Utterances arrive longest first.  A planner walks them once and decides, before adding
each one, whether the open minibatch is closed first:

* ``SeqBatch``  -- the minibatch's capacity is fixed when it is opened, from its first
  (longest) utterance:  max(min_batch_size,
  int(batch_size / (1 + max(int(xlen / max_len_in), int(ylen / max_len_out))))).
* ``FrameBatch`` -- it closes when (size + 1) x max length would exceed any of the
  enabled frame budgets max_frame_in / max_frame_out / max_frame_inout.

Both keep the reference's edge behaviour: the "closes first?" test also runs on an empty
minibatch, so an utterance that alone exceeds a frame budget emits an empty minibatch
before it (it still gets a minibatch of its own).  ``policy.data[i]`` / ``policy[i]`` is
the i-th minibatch as a list of utterance indices.
"""

from typing import List, Sequence


class BatchifyPolicy(object):
    def __init__(self, dataset_cfg):
        self.dataset_cfg = dataset_cfg
        self.data: List[List[int]] = []

    # subclasses: does the open minibatch (its indices, its samples) close before `nxt`?
    def _closes_before(self, members, nxt) -> bool:
        raise NotImplementedError

    def batchify(self, indices: Sequence[int], samples):
        assert len(indices) == len(samples), f"{len(samples)}"
        members, open_samples = [], []
        for idx in indices:
            nxt = samples[idx]
            if self._closes_before(open_samples, nxt):
                self.data.append(members)
                members, open_samples = [], []
            members.append(idx)
            open_samples.append(nxt)
        if members:
            self.data.append(members)
        return self

    def __getitem__(self, index):
        return self.data[index]

    def __len__(self):
        return len(self.data)


class SeqBatch(BatchifyPolicy):
    def capacity(self, head) -> int:
        c = self.dataset_cfg
        factor = max(int(head.xlen / c.max_len_in), int(head.ylen / c.max_len_out))
        return max(c.min_batch_size, int(c.batch_size / (1 + factor)))

    def _closes_before(self, open_samples, nxt) -> bool:
        cap = self.capacity(open_samples[0]) if open_samples else self.dataset_cfg.batch_size
        return len(open_samples) == cap


class FrameBatch(BatchifyPolicy):
    def _closes_before(self, open_samples, nxt) -> bool:
        c = self.dataset_cfg
        n = len(open_samples) + 1
        xmax = max([s.xlen for s in open_samples] + [nxt.xlen])
        ymax = max([s.ylen for s in open_samples] + [nxt.ylen])
        budgets = ((c.max_frame_in, xmax), (c.max_frame_out, ymax), (c.max_frame_inout, xmax + ymax))
        return any(limit and length * n > limit for limit, length in budgets)
