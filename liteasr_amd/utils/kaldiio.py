"""Kaldi feature I/O (the subset of liteasr/utils/kaldiio the training path uses).

Reading goes through the native reader ``libliteasr_io.so`` (include/liteasr_io.h):
``load_mat`` / ``load_scp`` keep the reference's names and semantics
(liteasr/utils/kaldiio/matio.py:62-92, 225-338): ``"<ark>:<offset>[slices]"`` paths, FM / FV /
DM / DV / CM / CM2 / CM3 objects, float64 for D*, float32 otherwise.  ``read_padded`` is the
batched form the collator uses (one call per minibatch into a pinned buffer).

Writing (``save_ark`` / ``save_mat``, matio.py:643-903, compression_header.py:58-233) is plain
numpy; it exists so datasets and tests can be produced, and its byte layout is Kaldi's.
"""

from __future__ import annotations

import ctypes as C
import os
import struct
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libliteasr_io.so")

KIND_NAMES = {1: "FM", 2: "FV", 3: "DM", 4: "DV", 5: "CM", 6: "CM2", 7: "CM3"}

# compression methods (liteasr/utils/kaldiio/compression_header.py:8-14, Kaldi's enum)
kAutomaticMethod = 1
kSpeechFeature = 2
kTwoByteAuto = 3
kTwoByteSignedInteger = 4
kOneByteAuto = 5
kOneByteUnsignedInteger = 6
kOneByteZeroOne = 7


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        L = C.CDLL(_LIB_PATH)
        i64p = C.POINTER(C.c_int64)
        L.lasr_io_last_error.restype = C.c_char_p
        L.lasr_ark_probe.argtypes = [C.c_char_p, C.c_int64, C.c_int, i64p, i64p, C.POINTER(C.c_int)]
        L.lasr_ark_read.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_int64,
                                    i64p, i64p]
        L.lasr_ark_read_padded.argtypes = [C.c_int, C.POINTER(C.c_char_p), i64p, C.c_int, C.c_void_p, C.c_int64,
                                           C.c_int64, i64p, C.c_int]
        _LIB = L
    return _LIB


def _check(rc):
    if rc != 0:
        msg = lib().lasr_io_last_error()
        raise IOError(msg.decode() if msg else f"liteasr_io error {rc}")


# ------------------------------------------------------------------- ark paths ---
def parse_arkpath(ark_name: str) -> Tuple[str, Optional[int], Optional[tuple]]:
    """``'a.ark:12[3:4]'`` -> ('a.ark', 12, (slice(3, 5),)) (matio.py:244-325 semantics:
    ranges are inclusive, ``'|'`` pipes are returned unparsed)."""
    s = ark_name.strip()
    if s.endswith("|") or s.startswith("|"):
        return ark_name, None, None
    slices = None
    if "[" in ark_name and "]" in ark_name:
        base, rng = ark_name.split("[")
        try:
            slices = _to_slices(rng.replace("]", "").strip())
        except Exception:
            slices = None
        else:
            ark_name = base
    if ":" in ark_name:
        fname, off = ark_name.rsplit(":", 1)
        try:
            return fname, int(off), slices
        except ValueError:
            return ark_name, None, slices
    return ark_name, None, slices


def _to_slices(spec: str) -> tuple:
    out = []
    for ele in spec.split(","):
        if ele in ("", ":"):
            out.append(slice(None))
            continue
        try:
            v = [int(x) for x in ele.split(":")]
        except ValueError:
            raise ValueError(f"Format error: {spec}") from None
        if len(v) == 1:
            out.append(slice(v[0], v[0] + 1))
        elif len(v) == 2:
            out.append(slice(v[0], v[1] + 1))
        elif len(v) == 3:
            out.append(slice(v[0], v[1] + 1, v[2]))
        else:
            raise RuntimeError(f"Too many : {spec}")
    return tuple(out)


# ----------------------------------------------------------------------- reading ---
def probe(path: str, offset: Optional[int] = None, endian: str = "<"):
    r, c, k = C.c_int64(), C.c_int64(), C.c_int()
    _check(lib().lasr_ark_probe(path.encode(), -1 if offset is None else offset, int(endian == ">"),
                                C.byref(r), C.byref(c), C.byref(k)))
    return r.value, c.value, KIND_NAMES[k.value]


def load_mat(ark_name: str, endian: str = "<", fd_dict=None) -> np.ndarray:
    """The matrix/vector at ``ark_name`` (reference load_mat, matio.py:225-241)."""
    assert endian in ("<", ">"), endian
    path, offset, slices = parse_arkpath(ark_name)
    if path.strip().endswith("|") or path.strip().startswith("|"):
        raise NotImplementedError("pipe arks are not supported by the native reader")
    rows, cols, kind = probe(path, offset, endian)
    f64 = kind in ("DM", "DV")
    vec = kind in ("FV", "DV")
    shape = (rows,) if vec else (rows, cols)
    arr = np.empty(shape, dtype=np.float64 if f64 else np.float32)
    ld = rows if vec else cols
    _check(lib().lasr_ark_read(path.encode(), -1 if offset is None else offset, int(endian == ">"),
                               arr.ctypes.data_as(C.c_void_p), 1 if f64 else 0, rows, max(ld, 1), None, None))
    if slices is not None:
        arr = arr[slices]
    return arr


def read_padded(entries: Iterable[str], tmax: int, feat_dim: int, out: Optional[np.ndarray] = None,
                nthreads: int = 0, endian: str = "<"):
    """Decode feature matrices ``entries`` (``ark:offset`` strings) into a zero-padded
    float32 [n, tmax, feat_dim] array (``out`` may be a view of a pinned torch buffer).
    Returns (array, lengths int64[n])."""
    entries = list(entries)
    n = len(entries)
    paths, offs = [], []
    for e in entries:
        p, o, sl = parse_arkpath(e)
        if sl is not None:
            raise ValueError("read_padded: sliced ark paths are not supported; use load_mat")
        paths.append(p.encode())
        offs.append(-1 if o is None else o)
    if out is None:
        out = np.empty((n, tmax, feat_dim), dtype=np.float32)
    assert out.dtype == np.float32 and out.flags.c_contiguous and out.shape == (n, tmax, feat_dim)
    lens = np.zeros(n, dtype=np.int64)
    parr = (C.c_char_p * max(n, 1))(*paths)
    oarr = (C.c_int64 * max(n, 1))(*offs)
    _check(lib().lasr_ark_read_padded(n, parr, oarr, int(endian == ">"), out.ctypes.data_as(C.c_void_p), tmax,
                                      feat_dim, lens.ctypes.data_as(C.POINTER(C.c_int64)), nthreads))
    return out, lens


class _LazyScp(dict):
    """uttid -> matrix, loaded on access (reference load_scp's LazyLoader)."""

    def __getitem__(self, key):
        return load_mat(dict.__getitem__(self, key), endian=self.endian)

    def items(self):
        for k in self.keys():
            yield k, self[k]

    def values(self):
        for k in self.keys():
            yield self[k]


def load_scp(fname: str, endian: str = "<", separator: Optional[str] = None) -> Dict[str, np.ndarray]:
    d = _LazyScp()
    d.endian = endian
    with open(fname, "r") as f:
        for line in f:
            seps = line.split(separator, 1)
            if len(seps) != 2:
                raise ValueError(f"Invalid line is found:\n>   {line}")
            dict.__setitem__(d, seps[0], seps[1].rstrip())
    return d


def load_ark(fname: str, endian: str = "<"):
    """Iterate (key, matrix) over a whole binary ark."""
    size = os.path.getsize(fname)
    with open(fname, "rb") as f:
        pos = 0
        while pos < size:
            f.seek(pos)
            key = bytearray()
            while True:
                ch = f.read(1)
                if ch in (b" ", b""):
                    break
                key += ch
            if not key:
                return
            start = pos + len(key) + 1
            yield key.decode(), load_mat(f"{fname}:{start}", endian)
            pos = start + _object_size(fname, start, endian)


def _object_size(fname, offset, endian):
    rows, cols, kind = probe(fname, offset, endian)
    head = 2 + len(kind) + 1
    if kind in ("CM", "CM2", "CM3"):
        head += 16
        per = {"CM": 1, "CM2": 2, "CM3": 1}[kind]
        return head + (8 * cols if kind == "CM" else 0) + per * rows * cols
    if kind in ("FV", "DV"):
        return head + 5 + rows * (4 if kind == "FV" else 8)
    return head + 10 + rows * cols * (4 if kind == "FM" else 8)


# ----------------------------------------------------------------------- writing ---
def _quant(x, minv, rng, c, dtype):
    # GlobalHeader.float_to_uint: (x - min) / range * c + 0.499, truncated
    return ((x - minv) / rng * c + 0.499).astype(dtype)


def _dequant(u, minv, rng, c):
    return minv + u.astype(np.float32) * rng / c


def _write_compressed(fd, a: np.ndarray, method: int, endian: str) -> int:
    if method == kAutomaticMethod:
        method = kSpeechFeature if a.shape[0] > 8 else kTwoByteAuto
    typ = {kSpeechFeature: "CM", kTwoByteAuto: "CM2", kTwoByteSignedInteger: "CM2", kOneByteAuto: "CM3",
           kOneByteUnsignedInteger: "CM3", kOneByteZeroOne: "CM3"}.get(method)
    if typ is None:
        raise ValueError(f"Unknown compression_method: {method}")
    if method in (kSpeechFeature, kTwoByteAuto, kOneByteAuto):
        minv, maxv = a.min(), a.max()
        if minv == maxv:
            maxv = minv + (1.0 + abs(minv))
        rng = maxv - minv
    else:
        minv, rng = {kTwoByteSignedInteger: (-32768.0, 65535.0), kOneByteUnsignedInteger: (0.0, 255.0),
                     kOneByteZeroOne: (0.0, 1.0)}[method]
    c = 255.0 if typ == "CM3" else 65535.0
    rows, cols = a.shape
    fd.write(typ.encode() + b" " + struct.pack(endian + "ffii", minv, rng, rows, cols))
    n = len(typ) + 17
    if typ == "CM":
        # per-column 0/25/75/100 percentiles, 16-bit quantised, kept strictly increasing
        q = rows // 4
        if rows >= 5:
            s = np.partition(a, [0, q, 3 * q, rows - 1], axis=0)
            p = [s[0], s[q], s[3 * q], s[rows - 1]]
        else:
            s = np.sort(a, axis=0)
            p0 = s[0]
            p25 = s[1] if rows > 1 else p0 + 1
            p75 = s[2] if rows > 2 else p25 + 1
            p100 = s[3] if rows > 3 else p75 + 1
            p = [p0, p25, p75, p100]
        u = [_quant(v, minv, rng, c, np.dtype(endian + "u2")) for v in p]
        u[0] = np.minimum(u[0], 65532)
        u[1] = np.minimum(np.maximum(u[1], u[0] + 1), 65533)
        u[2] = np.minimum(np.maximum(u[2], u[1] + 1), 65534)
        u[3] = np.maximum(u[3], u[2] + 1)
        f = [_dequant(v, minv, rng, c)[:, None] for v in u]
        hdr = np.concatenate(f, axis=1)
        hb = _quant(hdr, minv, rng, c, np.dtype(endian + "u2")).astype(np.dtype(endian + "u2")).tobytes()
        fd.write(hb)
        n += len(hb)
        x = a.T
        t1 = np.clip((x - f[0]) / (f[1] - f[0]) * 64.0 + 0.5, 0.0, 64.0)
        t2 = np.clip((x - f[1]) / (f[2] - f[1]) * 128.0 + 64.5, 64.0, 192.0)
        t3 = np.clip((x - f[2]) / (f[3] - f[2]) * 63.0 + 192.5, 192.0, 255.0)
        lo, hi = x < f[1], x >= f[2]
        data = np.where(lo, t1, np.where(~lo & ~hi, t2, t3)).astype(np.dtype(endian + "u1")).tobytes()
    else:
        data = _quant(a, minv, rng, c, np.dtype(endian + ("u2" if c == 65535.0 else "u1"))).tobytes()
    fd.write(data)
    return n + len(data)


def write_array(fd, array: np.ndarray, endian: str = "<", compression_method: Optional[int] = None) -> int:
    """One Kaldi binary object (\\0B header + payload); returns bytes written."""
    assert isinstance(array, np.ndarray), type(array)
    fd.write(b"\0B")
    if compression_method is not None:
        if array.ndim != 2:
            raise ValueError("array must be matrix if compression_method is not None")
        return 2 + _write_compressed(fd, array, compression_method, endian)
    if array.dtype == np.int32:
        assert array.ndim == 1
        fd.write(b"\4" + struct.pack(endian + "i", len(array)))
        for v in array:
            fd.write(b"\4" + struct.pack(endian + "i", int(v)))
        return 2 + (len(array) + 1) * 5
    if array.dtype not in (np.float32, np.float64) or array.ndim not in (1, 2):
        raise ValueError(f"Unsupported array type: {array.dtype}")
    tag = {(np.dtype(np.float32), 1): b"FV ", (np.dtype(np.float64), 1): b"DV ",
           (np.dtype(np.float32), 2): b"FM ", (np.dtype(np.float64), 2): b"DM "}[(array.dtype, array.ndim)]
    fd.write(tag + b"\4" + struct.pack(endian + "i", array.shape[0]))
    n = 2 + 3 + 5
    if array.ndim == 2:
        fd.write(b"\4" + struct.pack(endian + "i", array.shape[1]))
        n += 5
    data = array.astype(array.dtype.newbyteorder(endian)).tobytes()
    fd.write(data)
    return n + len(data)


def save_ark(ark: str, array_dict: Dict[str, np.ndarray], scp: Optional[str] = None, append: bool = False,
             endian: str = "<", compression_method: Optional[int] = None):
    """Write ``{key: array}`` to a binary ark (+ ``key ark:offset`` scp lines)."""
    pos = []
    with open(ark, "ab" if append else "wb") as fd:
        base = fd.tell()
        size = 0
        for key, arr in array_dict.items():
            kb = (key + " ").encode()
            fd.write(kb)
            size += len(kb)
            pos.append(size)
            size += write_array(fd, arr, endian, compression_method)
    if scp is not None:
        with open(scp, "a" if append else "w") as f:
            for key, p in zip(array_dict, pos):
                f.write(f"{key} {ark}:{p + base}\n")


def save_mat(fname: str, array: np.ndarray, endian: str = "<", compression_method: Optional[int] = None):
    with open(fname, "wb") as fd:
        return write_array(fd, array, endian, compression_method)
