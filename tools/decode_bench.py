"""Inference timing on one MI355X: U2-Conformer-small (bf16, random init),
one utterance of T=1000 frames, beam 10.

  python tools/decode_bench.py [--iters N]

Prints one JSON line: per-utterance wall time of ctc_prefix_beam_search, attention_rescore
and attention; the lasr_logsoftmax_topk launch (HIP events, 249 x 4233 logits, k 10) with
its algorithmic bytes; and the reference's pure-Python prefix beam search (restated in
oracle/decode_ref.py, checked bit-exact against the reference in tests/test_decode.py)
timed on the same log-probs on one host core, beside the native C++ search.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    from liteasr_amd import decoding as D
    from liteasr_amd import kernels as K
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.nets import functional as FN
    from liteasr_amd.utils.cfg import resolve_self
    from oracle import decode_ref as R

    torch.manual_seed(42)
    c = U2Config(input_dim=80, vocab_size=4233, enc_dim=256, enc_ff_dim=2048, enc_layers=12, dec_dim=256,
                 dec_ff_dim=2048, dec_layers=6, compute_dtype="bf16")
    resolve_self(c)
    model = U2(c).cuda().eval()
    x = torch.randn(1, a.T, 80, generator=torch.Generator().manual_seed(0)).cuda()
    out = {"workload": f"U2-Conformer-small bf16, 1 utt T={a.T}, beam 10", "iters": a.iters}

    def timed(fn):
        for _ in range(3):  # graph capture, clocks
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.iters * 1e3

    with torch.no_grad():
        out["ctc_prefix_beam_search_ms"] = timed(lambda: model.ctc_prefix_beam_search(x))
        out["attention_rescore_ms"] = timed(lambda: model.attention_rescore(x))
        out["encoder_ms"] = timed(lambda: D.encode(model, x))
        h, T = D.encode(model, x)
        logits = FN.ctc_logits(h, model)
        V = logits.shape[1]
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K.logsoftmax_topk(logits, 10)
        n = 50
        e0.record(s)
        for _ in range(n):
            K.logsoftmax_topk(logits, 10)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        byts = T * V * logits.element_size() + T * 10 * 8
        out["topk_kernel"] = {"rows": T, "V": V, "k": 10, "avg_launch_us": us,
                              "algorithmic_bytes": byts, "GBps": byts / us / 1e3}
        vals, idx, _ = K.logsoftmax_topk(logits, 10)
        v, i = vals.cpu().numpy(), idx.cpu().numpy()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            nat = D.prefix_beam_search(v, i, beam=10)
        out["native_prefix_search_ms"] = (time.perf_counter() - t0) / a.iters * 1e3
        t0 = time.perf_counter()
        ref = R.ctc_prefix_beam_search(None, beam=10, topk=(v, i))
        out["python_prefix_search_ms_1core"] = (time.perf_counter() - t0) * 1e3
        out["native_equals_python"] = nat == ref
        out["attention_ms"] = timed(lambda: model.attention(x)) if a.T <= 400 else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
