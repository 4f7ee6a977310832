"""Seeded golden-case inputs shared by tests/golden/make_golden.py (which runs the reference
on them in the build container) and the tests (which regenerate the same inputs on the
GPU box, where only the .npz outputs travel).  Data recipes only; no reference code."""

import torch


CTC_LARGE_CASES = [
    # name, T' (frames after subsampling of utterance 0), B, V, Lmax, seed
    ("t249", 249, 4, 4233, 40, 31),
    ("t999", 999, 2, 4233, 150, 32),
]


def ctc_large_inputs(Tp, B, V, L, seed):
    """Seeded CTC inputs (shared with the tests, which regenerate the logits): xlens give
    pred_len Tp for utterance 0 and shorter ones after; labels with repeats; logits*2."""
    g = torch.Generator().manual_seed(seed)
    Tx = 4 * Tp + 3  # ((Tx - 1) // 2 - 1) // 2 == Tp
    xlens = torch.tensor([Tx] + [Tx - 4 * (7 + 5 * b) for b in range(1, B)])
    ylens = torch.tensor([L] + [max(1, L - 3 * b) for b in range(1, B)])
    ys = torch.randint(1, V - 1, (B, L), generator=g)
    ys[:, 5] = ys[:, 4]  # repeated labels (the skip rule's exception)
    ys[:, 6] = ys[:, 4]
    for b in range(B):
        ys[b, ylens[b]:] = -1
    h_ctc = torch.randn(B, Tp, V, generator=g) * 2
    return xlens, ys, ylens, h_ctc
