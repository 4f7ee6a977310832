"""Inference searches of U2 (liteasr/models/u2.py:160-317), SURVEY §8 f3.

Device side: the encoder / decoder run through the same HIP kernels as training
(nets/functional.py: encoder_out, ctc_logits, decoder_logits); per-frame log_softmax +
top-k and the rescoring gathers are one HIP kernel (lasr_logsoftmax_topk).  Host side:
the CTC prefix beam search is native C++ (libliteasr_decode.so, csrc/decode/), fed
with the [T', beam] candidates; the attention beam's (beam x beam) bookkeeping is a few
float32 numpy operations mirroring the reference's torch ops.  No CPU fallback: both
libraries must be present.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import kernels as K
from .nets import functional as FN

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libliteasr_decode.so")
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        L = C.CDLL(_LIB_PATH)
        L.lasr_ctc_prefix_beam_search.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                  C.c_int, C.c_void_p, C.c_int64, C.c_void_p,
                                                  C.c_void_p]
        L.lasr_ctc_prefix_beam_search.restype = C.c_int
        L.lasr_decode_last_error.restype = C.c_char_p
        _LIB = L
    return _LIB


def prefix_beam_search(topk_val: np.ndarray, topk_idx: np.ndarray, beam: int, blank: int = 0):
    """Native CTC prefix beam search over per-frame candidates [T, k] (float32 log-probs,
    int32 ids, descending).  Returns [(tokens list, score float)], best first."""
    v = np.ascontiguousarray(topk_val, dtype=np.float32)
    i = np.ascontiguousarray(topk_idx, dtype=np.int32)
    T, k = v.shape
    cap = max(1, beam * T)
    tok = np.empty(cap, dtype=np.int32)
    lens = np.empty(beam, dtype=np.int32)
    score = np.empty(beam, dtype=np.float64)
    n = _lib().lasr_ctc_prefix_beam_search(v.ctypes.data, i.ctypes.data, T, k, blank, beam,
                                           tok.ctypes.data, cap, lens.ctypes.data, score.ctypes.data)
    if n < 0:
        raise RuntimeError("lasr_ctc_prefix_beam_search: " + _lib().lasr_decode_last_error().decode())
    out, o = [], 0
    for j in range(n):
        out.append((tok[o:o + lens[j]].tolist(), float(score[j])))
        o += int(lens[j])
    return out


def _mem_mask(B, T, dev):
    return torch.zeros(B, T, dtype=torch.uint8, device=dev)


def encode(model, x, graph=True):
    """`self.encoder(x)` for one utterance x [1, T, F] (no padding mask) -> (h [T', d], T').

    With ``graph`` the ~250 encoder launches of a batch-1 utterance (launch-latency-bound)
    are captured once per input shape into a hipGraph and replayed; the returned h is that
    graph's static output, valid until the next encode of the same shape.  The cache is
    keyed on the flat parameter version, so a weight update re-captures (the working-copy
    cast is host-conditional and must not be skipped by a stale graph), and on the
    train/eval mode.  (The fused Adam kernel rewrites flat and its working copy in place,
    without a version bump: the graph reads them through the same pointers, so replays
    after optimizer steps see the new weights.)"""
    if x.device.type != "cuda":
        raise RuntimeError("liteasr_amd decoding runs on the HIP device only")
    if not graph:
        return _encode_eager(model, x)
    st = model.store
    # model.training too: dropout and BatchNorm (batch vs running statistics) are baked
    # into the captured launches, so a train()/eval() switch must re-capture
    key = (tuple(x.shape), x.dtype, st.flat._version, st.generation, bool(model.training))
    cache = model.__dict__.setdefault("_encode_graphs", {})
    e = cache.get(key)
    if e is None:
        cache.clear()
        static = x.clone()
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):  # warm-up: workspaces, working copies, allocator pools
            _encode_eager(model, static)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            h, T = _encode_eager(model, static)
        # keep the workspace the graph was captured against alive even if it is regrown
        e = cache[key] = (g, static, h, T, K.WS.buf.get(x.device.index))
    g, static, h, T, _ = e
    static.copy_(x)
    g.replay()
    return h, T


def _encode_eager(model, x):
    B, Tx = x.shape[0], x.shape[1]
    xlens = torch.full((B,), Tx, dtype=torch.int64, device=x.device)
    ys = torch.full((B, 1), -1, dtype=torch.int64, device=x.device)
    ylens = torch.zeros(B, dtype=torch.int64, device=x.device)
    xe, prep, _ = model._run_encoder(x, xlens, ys, ylens)
    return FN.encoder_out(xe, model, model.compute_dtype), prep.T


def ctc_prefix_beam_search_nbest(model, x, beam=10):
    """u2.py:218-263: (n-best [(tokens, score)], h [T', d], T')."""
    h, T = encode(model, x)
    logits = FN.ctc_logits(h, model)
    vals, idx, _ = K.logsoftmax_topk(logits, min(beam, logits.shape[1]))
    hyps = prefix_beam_search(vals.cpu().numpy(), idx.cpu().numpy(), beam, model.blank)
    return hyps, h, T


def rescore(model, hyps, h, T, ctc_weight=0.5):
    """u2.py:268-317: decoder over the n-best (memory = h repeated, no memory mask),
    score = sum of attention log-probs at the tokens + eos (fp32, as the reference's
    0-d tensor sum) + ctc_weight * CTC score; first strict maximum wins."""
    dev = h.device
    n = len(hyps)
    Lmax = max(1, max(len(t) for t, _ in hyps))
    L1 = Lmax + 1
    ys = torch.full((n, Lmax), -1, dtype=torch.int64)
    for i, (t, _) in enumerate(hyps):
        ys[i, :len(t)] = torch.tensor(t, dtype=torch.int64)
    ylens = torch.tensor([len(t) for t, _ in hyps], dtype=torch.int64)
    Tx = 4 * T + 3  # any Tx with ((Tx-1)//2-1)//2 == T; all frames valid
    prep = model._prep_targets(ys.to(dev), ylens.to(dev), n, Tx)
    mem = h.view(1, T, -1).expand(n, T, h.shape[1]).reshape(n * T, h.shape[1])
    h_attn = FN.decoder_logits(model, mem, prep.ys_in, prep.dec_mask, _mem_mask(n, T, dev), n, L1, T)
    gidx = torch.full((n, L1), -1, dtype=torch.int32)
    for i, (t, _) in enumerate(hyps):
        gidx[i, :len(t)] = torch.tensor(t, dtype=torch.int32)
        gidx[i, len(t)] = model.eos
    _, _, g = K.logsoftmax_topk(h_attn, 0, gather_idx=gidx.view(-1).to(dev))
    return pick_best(hyps, g.view(n, L1).cpu().numpy(), ctc_weight)


def pick_best(hyps, g, ctc_weight=0.5):
    """Host half of rescoring (u2.py:300-315): g[i, j] = attention log-prob of hypothesis
    i's j-th token (j = len: eos).  float32 running sum like the reference's 0-d tensor,
    python-float CTC term cast to float32, first strict maximum wins."""
    f32 = np.float32
    best, best_i = -float("inf"), 0
    for i, (t, sc) in enumerate(hyps):
        s = f32(0.0)
        for j in range(len(t) + 1):  # tokens, then eos at position len(t)
            s = f32(s + g[i, j])
        s = f32(s + f32(sc * ctc_weight))
        if s > best:
            best, best_i = s, i
    return best_i


def attention_beam_search(model, x, beam=10, trace=None):
    """u2.py:163-216: left-to-right attention beam search (memory h repeated, no memory
    mask), max T' steps, the decoder advanced one position per step through its key/value
    cache (FN.DecoderStepCache: the reference's forward_one_step cache semantics, incl. its
    never-reordered cache of layers >= 1), per-step log_softmax + topk(beam) on the device,
    the (beam x beam) score bookkeeping in float32 on the host.  trace (a list): per step
    (hyps fed to the step [beam, i], log-prob top-k values [beam, beam]) for tests."""
    h, T = encode(model, x)
    dev = h.device
    sos, eos = model.sos, model.eos
    init = np.array([0.0] + [-np.inf] * (beam - 1), dtype=np.float32)
    hyps = np.full((beam, 1), sos, dtype=np.int64)
    scores = init.reshape(beam, 1).copy()
    end = np.zeros(beam, dtype=bool)
    dec = FN.DecoderStepCache(model, h, beam, T, T + 1)
    sel_d = None
    for i in range(1, T + 1):
        if end.sum() == beam:
            break
        ids = torch.from_numpy(np.ascontiguousarray(hyps[:, -1]).astype(np.int32)).to(dev)
        logits = dec.step(ids, i, sel_d)
        vals, idx, _ = K.logsoftmax_topk(logits, beam)
        st = vals.cpu().numpy()
        it = idx.cpu().numpy().astype(np.int64)
        if trace is not None:
            trace.append((hyps.copy(), st.copy()))
        st[end] = init
        it[end] = eos
        cand = (scores + st).reshape(-1).astype(np.float32)
        order = np.argsort(-cand.astype(np.float64), kind="stable")[:beam]
        scores = cand[order].reshape(beam, 1)
        sel, off = order // beam, order % beam
        hyps = np.concatenate([hyps[sel], it[sel, off][:, None]], axis=1)
        sel_d = torch.from_numpy(sel.astype(np.int64)).to(dev)
        end = hyps[:, -1] == eos
    best = int(np.argmax(scores.reshape(-1)))
    return hyps[best].tolist()
