"""Token vocabulary (liteasr/dataclass/vocab.py:4-85): id 0 is <blank>, ids 1..N come from
the vocab file ("<token> <id>", consecutive), and <sos/eos> is appended as N+1."""

from typing import Any, Iterable


class Vocab(object):
    def __init__(self, vocab_path: str) -> None:
        self.token2id = {"<blank>": 0}
        self.id2token = ["<blank>"]
        with open(vocab_path, "r") as f:
            for line in f.readlines():
                entry = line.strip().split()
                if len(entry) != 2:
                    raise ValueError(f"Invalid line is found:\n>    {line}")
                token, tid = entry[0], int(entry[1])
                if tid != len(self.id2token):
                    raise ValueError(f"Missing token id: {len(self.id2token)}")
                self.token2id[token] = tid
                self.id2token.append(token)
        self.token2id["<sos/eos>"] = len(self.id2token)
        self.id2token.append("<sos/eos>")

    @property
    def valid(self) -> bool:
        return all(self.id2token[self.token2id[t]] == t for t in self.token2id)

    def __getitem__(self, index):
        if isinstance(index, str):
            return self.token2id[index] if index in self.token2id else self.token2id["<unk>"]
        if isinstance(index, int):
            if index < len(self.id2token):
                return self.id2token[index]
            raise IndexError("Index out of range of vocabulary")
        raise KeyError(f"Key {index} is not valid")

    def convert(self, index):
        assert isinstance(index, int)
        tok = self.id2token[index]
        if tok in ("<blank>", "<sos/eos>"):
            return ""
        if tok == "<space>":
            return " "
        return tok

    def __len__(self) -> int:
        return len(self.id2token)

    def lookupi(self, seq: Iterable[Any], convert=False):
        return map(self.convert, seq) if convert else map(lambda t: self[t], seq)

    def lookup(self, seq: Iterable[Any], convert=False):
        return tuple(self.lookupi(seq, convert=convert))
