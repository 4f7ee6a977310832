"""Measure the bf16 build's per-tensor gradient errors against the fp64 oracle run on the
same bf16-rounded weights and features (for setting tests/test_model_gpu.py bounds)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_model_gpu as T  # noqa: E402
from oracle import u2_oracle as O  # noqa: E402

cases = {
    "tiny": (T.TINY, 3, 130, 8, 0),
    "small2": (T.SMALL, 2, 210, 12, 0),
    "dk32_chunk": (T.LARGE_HEADS, 2, 150, 6, 8),
    "d512_h16_chunk": (O.default_cfg(enc_dim=512, enc_heads=16, enc_ff=2048, enc_layers=2, dec_dim=512, dec_heads=16,
                                     dec_ff=2048, dec_layers=1, vocab_size=4233), 2, 200, 10, 16),
}
out = {}
for name, (cfg, B, Tx, L, chunk) in cases.items():
    for rnd in (False, True):
        r = T.run_case(cfg, B, Tx, L, "bf16", chunk=chunk, round_bf16=rnd)
        g, go = r["grads"]
        errs, floor = T.grad_errs(g, go)
        worst = sorted(((v, k) for k, v in errs.items()), reverse=True)[:4]
        coss = min((T.cos(g[k], go[k]), k) for k in go if go[k].abs().max().item() > floor)
        lg, lo = r["loss"]
        out[f"{name}_round{int(rnd)}"] = dict(loss_rel=abs(lg - lo) / abs(lo), h_attn=T.rel(*r["h_attn"]),
                                              h_ctc=T.rel(*r["h_ctc"]), worst=worst, min_cos=coss)
        print(name, rnd, json.dumps(out[f"{name}_round{int(rnd)}"]), flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "bf16_errs.json"), "w"), indent=1)
