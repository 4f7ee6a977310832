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


def _lse(*xs):
    m = max(xs)
    if m == -np.inf:
        return -np.inf
    return m + np.log(sum(np.exp(x - m) for x in xs))


def ctc_nll_and_grad(lp: np.ndarray, labels: np.ndarray, blank: int = 0):
    """lp: [T, V] log-probabilities (rows already log_softmax'ed); labels: [L] ints.
    Returns (nll, grad [T, V] of nll w.r.t. the logits that produced lp)."""
    T, V = lp.shape
    L = len(labels)
    ext = np.full(2 * L + 1, blank, dtype=np.int64)
    ext[1::2] = labels
    S = len(ext)
    a = np.full((T, S), -np.inf)
    b = np.full((T, S), -np.inf)
    a[0, 0] = lp[0, ext[0]]
    if S > 1:
        a[0, 1] = lp[0, ext[1]]
    for t in range(1, T):
        for s in range(S):
            terms = [a[t - 1, s]]
            if s >= 1:
                terms.append(a[t - 1, s - 1])
            if s >= 2 and ext[s] != blank and ext[s] != ext[s - 2]:
                terms.append(a[t - 1, s - 2])
            a[t, s] = _lse(*terms) + lp[t, ext[s]]
    b[T - 1, S - 1] = lp[T - 1, ext[S - 1]]
    if S > 1:
        b[T - 1, S - 2] = lp[T - 1, ext[S - 2]]
    for t in range(T - 2, -1, -1):
        for s in range(S):
            terms = [b[t + 1, s]]
            if s + 1 < S:
                terms.append(b[t + 1, s + 1])
            if s + 2 < S and ext[s] != blank and ext[s] != ext[s + 2]:
                terms.append(b[t + 1, s + 2])
            b[t, s] = _lse(*terms) + lp[t, ext[s]]
    ll = _lse(a[T - 1, S - 1], a[T - 1, S - 2]) if S > 1 else a[T - 1, 0]
    nll = -ll
    grad = np.exp(lp).copy()
    if np.isfinite(nll):
        for t in range(T):
            for s in range(S):
                grad[t, ext[s]] -= np.exp(a[t, s] + b[t, s] - lp[t, ext[s]] + nll)
    return nll, grad
