"""Float64 CTC restatement (numpy), TEST INFRASTRUCTURE ONLY.

The reference's CTC lives in a third-party dependency: PyTorch aten's ctc_loss /
_ctc_loss_backward (torch version unpinned by the reference, README.md:32; 2.10.0 here),
called from liteasr/criterions/hybrid_ctc_attn.py:67-75 with blank=0, reduction="sum".
This module restates the published algorithm (Graves et al., 2006, the alpha/beta
recursion over the blank-interleaved label sequence) in float64, independently of
torch, and is pinned against the reference call site's outputs by
tests/test_oracle_golden.py::test_ctc_numpy_restatement_matches_reference.

Gradient returned is w.r.t. the *logits* (through log_softmax): softmax - gamma,
which is what the reference's autograd produces for log_softmax -> ctc_loss.
"""

import numpy as np


def ctc_nll_and_grad(lp: np.ndarray, labels: np.ndarray, blank: int = 0):
    """lp: [T, V] log-probabilities (rows already log_softmax'ed); labels: [L] ints.
    Returns (nll, grad [T, V] of nll w.r.t. the logits that produced lp).

    alpha_t(s) = lp_t(l'_s) + logsumexp(alpha_{t-1}(s), alpha_{t-1}(s-1),
    [alpha_{t-1}(s-2) if l'_s != blank and l'_s != l'_{s-2}]), and beta mirrored; the
    recursion is vectorised over the extended-label positions s (one numpy step per
    frame), exact in float64."""
    lp = np.asarray(lp, dtype=np.float64)
    T, V = lp.shape
    L = len(labels)
    ext = np.full(2 * L + 1, blank, dtype=np.int64)
    ext[1::2] = labels
    S = len(ext)
    # skip transitions s-2 -> s allowed where the label differs from the one two back
    skip = np.zeros(S, dtype=bool)
    if S > 2:
        skip[2:] = (ext[2:] != blank) & (ext[2:] != ext[:-2])
    skip_b = np.zeros(S, dtype=bool)  # s+2 -> s in the backward pass
    if S > 2:
        skip_b[:-2] = (ext[:-2] != blank) & (ext[:-2] != ext[2:])
    ninf = -np.inf
    a = np.full((T, S), ninf)
    b = np.full((T, S), ninf)
    emit = lp[:, ext]  # [T, S]
    a[0, 0] = emit[0, 0]
    if S > 1:
        a[0, 1] = emit[0, 1]
    with np.errstate(invalid="ignore"):
        for t in range(1, T):
            prev = a[t - 1]
            acc = prev.copy()
            acc[1:] = np.logaddexp(acc[1:], prev[:-1])
            sk = np.full(S, ninf)
            sk[2:] = np.where(skip[2:], prev[:-2], ninf)
            acc = np.logaddexp(acc, sk)
            a[t] = acc + emit[t]
        b[T - 1, S - 1] = emit[T - 1, S - 1]
        if S > 1:
            b[T - 1, S - 2] = emit[T - 1, S - 2]
        for t in range(T - 2, -1, -1):
            nxt = b[t + 1]
            acc = nxt.copy()
            acc[:-1] = np.logaddexp(acc[:-1], nxt[1:])
            sk = np.full(S, ninf)
            sk[:-2] = np.where(skip_b[:-2], nxt[2:], ninf)
            acc = np.logaddexp(acc, sk)
            b[t] = acc + emit[t]
    ll = np.logaddexp(a[T - 1, S - 1], a[T - 1, S - 2]) if S > 1 else a[T - 1, 0]
    nll = -ll
    grad = np.exp(lp)
    if np.isfinite(nll):
        occ = np.exp(a + b - emit + nll)  # [T, S] posterior occupancy of each lattice node
        for s in range(S):
            grad[:, ext[s]] -= occ[:, s]
    return nll, grad
