"""Kaldi data-directory sheets (liteasr/dataclass/sheet.py:19-123): feats.scp +
utt2num_frames (AudioSheet) and text (TextSheet), iterated line by line in step."""

import os
from typing import Optional

from .vocab import Vocab


def _lines(path: Optional[str]) -> int:
    if path is None:
        return 0
    n = 0
    with open(path, "r") as f:
        for n, _ in enumerate(f, 1):
            pass
    return n


class AudioSheet(object):
    def __init__(self, data_dir):
        files = os.listdir(data_dir)
        if "feats.scp" in files:
            self.scp = f"{data_dir}/feats.scp"
            assert "utt2num_frames" in files
            self.shape = f"{data_dir}/utt2num_frames"
            self.segments = None
            self.lines = _lines(self.scp)
        elif "wav.scp" in files:
            raise NotImplementedError("wav.scp input is outside the feature training path (feats.scp only)")
        else:
            raise FileNotFoundError(f"wav.scp not found in {data_dir}")

    def __iter__(self):
        with open(self.scp, "r") as fscp, open(self.shape, "r") as fshp:
            while True:
                a, b = fscp.readline(), fshp.readline()
                if not a or not b:
                    break
                e1, e2 = a.strip().split(None, 1), b.strip().split(None, 1)
                if len(e1) != 2 or len(e2) != 2:
                    raise ValueError(f"Invalid line found:\n>\t{a}\n>\t{b}")
                assert e1[0] == e2[0]
                yield e1[0], e1[1], None, int(e2[1])

    def __len__(self):
        return self.lines


class TextSheet(object):
    def __init__(self, data_dir, vocab: Vocab, delimiter: Optional[str] = None):
        self.text = f"{data_dir}/text"
        self.vocab = vocab
        self.delimiter = delimiter
        self.lines = _lines(self.text)

    def __iter__(self):
        with open(self.text, "r") as f:
            for line in f:
                uttid, text = line.strip().split(maxsplit=1)
                tokens = text.split(self.delimiter)
                # delimiter None: the text is one token string looked up character-wise
                ids = self.vocab.lookup(tokens[0]) if self.delimiter is None else self.vocab.lookup(tokens)
                yield uttid, ids, text

    def __len__(self):
        return self.lines
