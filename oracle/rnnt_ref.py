"""RNN-T (transducer) loss: float64 numpy restatement.

TEST INFRASTRUCTURE ONLY.  Only tests/ (and the golden generator) may import this module,
as the checker -- never as the thing measured or shipped.

The reference computes this loss in a third-party package that is NOT in /root/reference
and not importable here: liteasr/criterions/rnnt.py:28 imports `warprnnt_pytorch.RNNTLoss`
(warp-transducer, HawkAaron, unpinned: requirements.txt does not list it) and :33
`warp_rnnt.rnnt_loss` (warp-rnnt, 1ytic, unpinned).  Both implement the published
algorithm of Graves, "Sequence Transduction with Recurrent Neural Networks" (2012), §2.3-2.5,
with blank = 0 and the batch mean, on raw joint logits (warp-transducer applies the
log-softmax itself, rnnt.py:64; the warp-rnnt branch applies it first, rnnt.py:50).  This is
a direct restatement of that algorithm; with neither package available its agreement with
the reference is UNPINNED.  It is pinned instead by tests/test_rnnt.py: exhaustive
enumeration of every alignment path on small lattices, and central finite differences of the
loss for the gradient.

Lattice (one utterance): T frames x (U+1) label positions; node (t, u) emits blank
(-> (t+1, u)) or label y[u] (-> (t, u+1)); the path ends with the blank emitted at
(T-1, U).
  alpha(0,0) = 0
  alpha(t,u) = logaddexp(alpha(t-1,u) + lp(t-1,u,blank), alpha(t,u-1) + lp(t,u-1,y[u-1]))
  beta(T-1,U) = lp(T-1,U,blank)
  beta(t,u)  = logaddexp(beta(t+1,u) + lp(t,u,blank), beta(t,u+1) + lp(t,u,y[u]))
  nll = -beta(0,0) = -(alpha(T-1,U) + lp(T-1,U,blank))
Gradient w.r.t. the log-probs (occupancies, Graves eq. 16-17):
  d nll / d lp(t,u,blank) = -exp(alpha(t,u) + lp(t,u,blank) + beta(t+1,u) + nll)
  d nll / d lp(t,u,y[u])  = -exp(alpha(t,u) + lp(t,u,y[u]) + beta(t,u+1) + nll)
(beta(T, U) := 0, beta(T, u < U) := -inf, beta(t, U+1) := -inf), and through the
log-softmax, d nll / d z(t,u,k) = softmax_k * occ(t,u) - c_k(t,u) with occ = sum_k c_k =
exp(alpha(t,u) + beta(t,u) + nll).
"""

from __future__ import annotations

import numpy as np


def log_softmax(z):
    m = z.max(-1, keepdims=True)
    return z - (m + np.log(np.exp(z - m).sum(-1, keepdims=True)))


def rnnt_nll_and_grad(z: np.ndarray, y, blank: int = 0):
    """z: logits (T, U+1, V) of one utterance (already cut to its lengths); y: U labels.
    Returns (nll, d nll / d z)."""
    z = np.asarray(z, dtype=np.float64)
    T, U1, V = z.shape
    U = U1 - 1
    y = np.asarray(y, dtype=np.int64)
    assert len(y) == U
    lp = log_softmax(z)
    lpb = lp[:, :, blank]
    lpy = np.full((T, U1), -np.inf)
    for u in range(U):
        lpy[:, u] = lp[:, u, y[u]]
    alpha = np.full((T, U1), -np.inf)
    alpha[0, 0] = 0.0
    for t in range(T):
        for u in range(U1):
            if t == 0 and u == 0:
                continue
            a = alpha[t - 1, u] + lpb[t - 1, u] if t > 0 else -np.inf
            b = alpha[t, u - 1] + lpy[t, u - 1] if u > 0 else -np.inf
            alpha[t, u] = np.logaddexp(a, b)
    beta = np.full((T + 1, U1 + 1), -np.inf)
    beta[T, U] = 0.0
    for t in range(T - 1, -1, -1):
        for u in range(U, -1, -1):
            beta[t, u] = np.logaddexp(beta[t + 1, u] + lpb[t, u], beta[t, u + 1] + lpy[t, u])
    nll = -beta[0, 0]
    cb = np.exp(alpha + lpb + beta[1:, :U1] + nll)
    cy = np.exp(alpha + lpy + beta[:T, 1:U1 + 1] + nll)
    cy[:, U] = 0.0
    occ = cb + cy
    g = np.exp(lp) * occ[:, :, None]
    g[:, :, blank] -= cb
    for u in range(U):
        g[:, u, y[u]] -= cy[:, u]
    return float(nll), g


def rnnt_batch(z: np.ndarray, ys, xl, yl, blank: int = 0):
    """Batch mean (warp-transducer / warp-rnnt reduction='mean'): z (B, Tmax, Umax+1, V),
    ys (B, Umax) padded, xl / yl lengths.  Returns (loss, per-utterance nll, dloss/dz with
    zeros outside each utterance's (xl, yl+1) block)."""
    B = z.shape[0]
    g = np.zeros_like(np.asarray(z, dtype=np.float64))
    nll = np.zeros(B)
    for b in range(B):
        T, U = int(xl[b]), int(yl[b])
        nll[b], gb = rnnt_nll_and_grad(z[b, :T, :U + 1], np.asarray(ys[b][:U]), blank)
        g[b, :T, :U + 1] = gb / B
    return float(nll.mean()), nll, g


def rnnt_brute_force(z: np.ndarray, y, blank: int = 0) -> float:
    """-log of the sum over every alignment path (exhaustive; tiny lattices only)."""
    lp = log_softmax(np.asarray(z, dtype=np.float64))
    T, U1, _ = lp.shape
    U = U1 - 1
    tot = []

    def walk(t, u, acc):
        if t == T - 1 and u == U:
            tot.append(acc + lp[t, u, blank])
            return
        if t < T - 1:
            walk(t + 1, u, acc + lp[t, u, blank])
        if u < U:
            walk(t, u + 1, acc + lp[t, u, y[u]])

    walk(0, 0, 0.0)
    return -float(np.logaddexp.reduce(np.array(tot)))
