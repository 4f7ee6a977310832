"""Decoding restatement (pure Python), TEST INFRASTRUCTURE ONLY.

Restates the reference's inference search algorithms so the native decoder can be
checked on the same inputs:
  * ctc_prefix_beam_search  -- liteasr/models/u2.py:218-263 (per-frame topk(beam), the
    blank / repeat / extend rules, defaultdict insertion order, stable descending sort)
    with log_add from u2.py:367-375;
  * rescore_pick           -- u2.py:300-315 (sum of attention log-probs at the hypothesis
    tokens + eos, plus 0.5 * CTC score, first strict maximum wins).
Pinned against the reference itself through tests/golden/decode.npz (made by
tests/golden/make_golden.py::gen_decode from /root/reference) in
tests/test_decode.py.  Never imported by the product path.
"""

import math
from collections import defaultdict

import numpy as np


def log_add(args):
    """u2.py:367-375."""
    if all(a == -float("inf") for a in args):
        return -float("inf")
    a_max = max(args)
    return a_max + math.log(sum(math.exp(a - a_max) for a in args))


def topk_desc(logp, k):
    """Descending top-k of a float32 row, ties to the smaller index."""
    idx = np.argsort(-logp.astype(np.float64), kind="stable")[:k]
    return logp[idx], idx


def ctc_prefix_beam_search(logp, beam=10, blank=0, topk=None):
    """logp: (T, V) float32 CTC log-probs.  topk: optional precomputed (vals, idx) [T, k]."""
    cur = [(tuple(), (0.0, -float("inf")))]
    for t in range(logp.shape[0] if topk is None else topk[0].shape[0]):
        if topk is None:
            vals, idx = topk_desc(logp[t], beam)
        else:
            vals, idx = topk[0][t], topk[1][t]
        nxt = defaultdict(lambda: (-float("inf"), -float("inf")))
        for ps, s in zip(vals, idx):
            s, ps = int(s), float(ps)
            for prefix, (pb, pnb) in cur:
                last = prefix[-1] if len(prefix) > 0 else None
                if s == blank:
                    n_pb, n_pnb = nxt[prefix]
                    nxt[prefix] = (log_add([n_pb, pb + ps, pnb + ps]), n_pnb)
                elif s == last:
                    n_pb, n_pnb = nxt[prefix]
                    nxt[prefix] = (n_pb, log_add([n_pnb, pnb + ps]))
                    n_prefix = prefix + (s,)
                    n_pb, n_pnb = nxt[n_prefix]
                    nxt[n_prefix] = (n_pb, log_add([n_pnb, pb + ps]))
                else:
                    n_prefix = prefix + (s,)
                    n_pb, n_pnb = nxt[n_prefix]
                    nxt[n_prefix] = (n_pb, log_add([n_pnb, pb + ps, pnb + ps]))
        cur = sorted(nxt.items(), key=lambda x: log_add(list(x[1])), reverse=True)[:beam]
    return [(list(p), log_add([pb, pnb])) for p, (pb, pnb) in cur]


def rescore_pick(hyps, attn_logp, eos, ctc_weight=0.5):
    """hyps: [(tokens, ctc_score)]; attn_logp: (n, L+1, V) log-probs.  u2.py:300-315.
    The reference's `score` becomes a 0-d fp32 tensor at its first `+=`, so the sum
    (python-float CTC term included) is carried in float32."""
    f32 = np.float32
    best, best_i = -float("inf"), 0
    for i, (toks, sc) in enumerate(hyps):
        s = f32(0.0)
        for j, w in enumerate(toks):
            s = f32(s + f32(attn_logp[i][j][w]))
        s = f32(s + f32(attn_logp[i][len(toks)][eos]))
        s = f32(s + f32(sc * ctc_weight))
        if s > best:
            best, best_i = s, i
    return best_i
