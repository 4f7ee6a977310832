"""One utterance record (liteasr/dataclass/audio_data.py:10-48): where its features live,
its frame count and token ids.  Feature matrices decode through the native reader."""

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ..utils.kaldiio import load_mat


@dataclass
class Audio(object):
    __slots__ = ["fd", "start", "shape", "tokenids", "text"]

    fd: str
    start: Optional[int]
    shape: int
    tokenids: Optional[Tuple[int]]
    text: Optional[str]

    @property
    def x(self):
        if self.start is None:  # feature matrix ("ark:offset")
            return torch.from_numpy(load_mat(self.fd))
        raise NotImplementedError("raw-waveform input (wav.scp) is outside the feature training path")

    @property
    def xlen(self):
        return self.shape

    @property
    def y(self):
        return torch.tensor(self.tokenids) if self.tokenids is not None else None

    @property
    def ylen(self):
        return len(self.tokenids) if self.tokenids is not None else 0
