"""RNN-T loss restatement (oracle/rnnt_ref.py) pinned without the reference's third-party
package (warp-transducer / warp-rnnt, liteasr/criterions/rnnt.py:28,33 -- absent, parity
against it UNPINNED): the forward-backward recursion equals the exhaustive sum over every
alignment path, and its analytic gradient equals central finite differences."""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import rnnt_ref as R  # noqa: E402


@pytest.mark.parametrize("T,U,V,seed", [(1, 0, 3, 0), (1, 2, 4, 1), (3, 0, 5, 2), (4, 3, 6, 3), (5, 2, 4, 4),
                                        (3, 3, 3, 5)])
def test_rnnt_recursion_equals_path_enumeration(T, U, V, seed):
    rng = np.random.default_rng(seed)
    z = rng.normal(size=(T, U + 1, V)) * 2
    y = rng.integers(1, V, size=U)
    nll, _ = R.rnnt_nll_and_grad(z, y)
    assert abs(nll - R.rnnt_brute_force(z, y)) <= 1e-12 * max(1.0, abs(nll))


@pytest.mark.parametrize("T,U,V,seed", [(4, 3, 5, 7), (6, 1, 7, 8), (2, 4, 3, 9)])
def test_rnnt_gradient_equals_finite_differences(T, U, V, seed):
    rng = np.random.default_rng(seed)
    z = rng.normal(size=(T, U + 1, V))
    y = rng.integers(1, V, size=U)
    _, g = R.rnnt_nll_and_grad(z, y)
    eps = 1e-6
    num = np.zeros_like(z)
    for idx in np.ndindex(*z.shape):
        zp, zm = z.copy(), z.copy()
        zp[idx] += eps
        zm[idx] -= eps
        num[idx] = (R.rnnt_nll_and_grad(zp, y)[0] - R.rnnt_nll_and_grad(zm, y)[0]) / (2 * eps)
    assert np.abs(g - num).max() <= 1e-7 * max(1.0, np.abs(num).max())
    # through the log-softmax the gradient of every (t, u) row sums to zero
    assert np.abs(g.sum(-1)).max() < 1e-12


def test_rnnt_batch_mean_and_padding():
    rng = np.random.default_rng(11)
    B, Tm, Um, V = 3, 6, 4, 5
    z = rng.normal(size=(B, Tm, Um + 1, V))
    xl, yl = np.array([6, 4, 1]), np.array([4, 0, 2])
    ys = rng.integers(1, V, size=(B, Um))
    loss, nll, g = R.rnnt_batch(z, ys, xl, yl)
    assert abs(loss - nll.mean()) < 1e-12
    for b in range(B):
        n1, g1 = R.rnnt_nll_and_grad(z[b, :xl[b], :yl[b] + 1], ys[b, :yl[b]])
        assert abs(n1 - nll[b]) < 1e-12 and np.abs(g1 / B - g[b, :xl[b], :yl[b] + 1]).max() < 1e-15
        assert not g[b, xl[b]:].any() and not g[b, :, yl[b] + 1:].any()
