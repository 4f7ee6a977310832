"""Synthetic fbank batches for throughput runs (SURVEY.md §8(d) input recipe).

xs ~ N(0, 1) of shape (B, T, F) zeroed past each length, xlens ~ U[0.95 T, T] with
xlens[0] = T (the collator's descending sort puts the longest utterance first,
liteasr/dataset/asr_dataset.py:107-110), ys ~ U{1 .. V-2} (never blank 0 nor sos/eos
V-1) padded with -1, ylens ~ U[L/2, L] with ylens[0] = L.  Drawn on the host from one
seeded torch.Generator, in that order, so every rank/run gets reproducible inputs.
"""

from __future__ import annotations

import torch


def synthetic_batch(B: int, T: int, L: int, V: int, F_: int = 80, seed: int = 0):
    gen = torch.Generator().manual_seed(seed)
    xlens = torch.randint(int(0.95 * T), T + 1, (B,), generator=gen)
    xlens[0] = T
    xs = torch.randn(B, T, F_, generator=gen)
    frame = torch.arange(T)
    xs[frame[None, :] >= xlens[:, None]] = 0.0
    ylens = torch.randint(max(1, L // 2), L + 1, (B,), generator=gen)
    ylens[0] = L
    ys = torch.randint(1, V - 1, (B, L), generator=gen)
    ys[torch.arange(L)[None, :] >= ylens[:, None]] = -1
    return xs, xlens, ys, ylens
