"""Per-utterance record of a dataset (the Audio record of liteasr/dataclass/audio_data.py).

Holds where the utterance's feature matrix lives (``fd``: a Kaldi "ark:offset" path,
decoded lazily by the native reader), its frame count and its token ids.  Positional
construction order (fd, start, shape, tokenids, text) is the reference's.  Raw-waveform
entries (``start`` not None, from wav.scp/segments) are outside the feature training path
and raise.
"""

from typing import Optional, Tuple

import torch

from ..utils.kaldiio import load_mat


class Audio(object):
    __slots__ = ("fd", "start", "shape", "tokenids", "text")

    def __init__(self, fd: str, start: Optional[int], shape: int, tokenids: Optional[Tuple[int]],
                 text: Optional[str]):
        self.fd, self.start, self.shape, self.tokenids, self.text = fd, start, shape, tokenids, text

    def __repr__(self):
        return f"Audio(fd={self.fd!r}, start={self.start}, shape={self.shape}, ylen={self.ylen})"

    def __eq__(self, other):
        return isinstance(other, Audio) and all(getattr(self, k) == getattr(other, k) for k in self.__slots__)

    @property
    def x(self) -> torch.Tensor:
        if self.start is not None:
            raise NotImplementedError("raw-waveform input (wav.scp) is outside the feature training path")
        return torch.from_numpy(load_mat(self.fd))

    @property
    def xlen(self) -> int:
        return self.shape

    @property
    def y(self):
        return None if self.tokenids is None else torch.tensor(self.tokenids)

    @property
    def ylen(self) -> int:
        return 0 if self.tokenids is None else len(self.tokenids)
