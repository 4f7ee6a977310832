"""Never-ending minibatch stream with an epoch counter (the reference's EpochDataLoader,
liteasr/utils/data_loader.py:6-29, as the Trainer consumes it).

The Trainer iterates ``for i, batch in enumerate(loader)`` forever and decides itself when
to stop; each time the underlying torch DataLoader is exhausted, ``epoch`` advances and a
new pass starts.  A DistributedSampler is re-seeded per pass through ``set_epoch`` so
every rank reshuffles consistently.  Re-entering ``iter()`` resumes the current pass.
"""

from torch.utils.data.dataloader import DataLoader

_EXHAUSTED = object()


class EpochDataLoader(object):
    def __init__(self, **loader_kwargs):
        self.data_loader = DataLoader(**loader_kwargs)
        self.epoch = 0
        self._pass = None  # iterator over the current epoch

    def __len__(self):
        return len(self.data_loader)

    def _start_pass(self):
        set_epoch = getattr(self.data_loader.sampler, "set_epoch", None)
        if callable(set_epoch):
            set_epoch(self.epoch)
        self._pass = iter(self.data_loader)

    def __iter__(self):
        if self._pass is None:
            self._start_pass()
        while True:
            item = next(self._pass, _EXHAUSTED)
            if item is _EXHAUSTED:
                self.epoch += 1
                self._start_pass()
                item = next(self._pass)  # an empty dataset ends the stream here
            yield item
