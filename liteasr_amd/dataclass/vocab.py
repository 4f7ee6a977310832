"""Token vocabulary with the id layout of liteasr/dataclass/vocab.py:20-85.

File format: one ``<token> <id>`` pair per line with ids 1, 2, ... in order.  Id 0 is
``<blank>`` (CTC blank), the file supplies 1..N and ``<sos/eos>`` is appended as N + 1.
Lookups: a token string maps to its id (unknown strings to the id of ``<unk>``), an int
id maps back to its token.
"""

from typing import Any, Iterable, List

BLANK, SOS_EOS, UNK, SPACE = "<blank>", "<sos/eos>", "<unk>", "<space>"


def _read_table(path: str) -> List[str]:
    tokens = [BLANK]
    with open(path, "r") as fh:
        for lineno, raw in enumerate(fh, start=1):
            fields = raw.split()
            if len(fields) != 2:
                raise ValueError(f"{path}:{lineno}: expected '<token> <id>', got {raw!r}")
            token, tid = fields[0], int(fields[1])
            if tid != len(tokens):
                raise ValueError(f"{path}:{lineno}: token id {tid} out of sequence (expected {len(tokens)})")
            tokens.append(token)
    tokens.append(SOS_EOS)
    return tokens


class Vocab(object):
    def __init__(self, vocab_path: str) -> None:
        self.id2token = _read_table(vocab_path)
        self.token2id = {tok: i for i, tok in enumerate(self.id2token)}

    @property
    def valid(self) -> bool:
        """Token <-> id maps are mutual inverses (no duplicate tokens in the file)."""
        return all(self.id2token[i] == tok for tok, i in self.token2id.items())

    def __getitem__(self, key):
        if isinstance(key, str):
            tid = self.token2id.get(key)
            return self.token2id[UNK] if tid is None else tid
        if isinstance(key, int):
            if key >= len(self.id2token):
                raise IndexError(f"token id {key} >= vocabulary size {len(self.id2token)}")
            return self.id2token[key]
        raise KeyError(f"vocabulary keys are token strings or int ids, not {type(key).__name__}")

    def convert(self, index):
        """Id -> text piece: blank / sos-eos vanish, <space> becomes ' '."""
        assert isinstance(index, int)
        tok = self.id2token[index]
        return {BLANK: "", SOS_EOS: "", SPACE: " "}.get(tok, tok)

    def __len__(self) -> int:
        return len(self.id2token)

    def lookupi(self, seq: Iterable[Any], convert=False):
        fn = self.convert if convert else self.__getitem__
        return map(fn, seq)

    def lookup(self, seq: Iterable[Any], convert=False):
        return tuple(self.lookupi(seq, convert=convert))
