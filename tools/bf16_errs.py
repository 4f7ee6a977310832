"""Measured per-tensor errors of the bf16 build against the bf16-emulating oracle
(oracle/u2_bf16.py) and, for comparison, against the plain fp64 oracle on the same
bf16-rounded weights and features (tests/test_model_gpu.py bars).
    python tools/bf16_errs.py [case ...]   -> gpurun_out/bf16_errs.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_model_gpu as T  # noqa: E402

cases = {
    "tiny": (T.TINY, 3, 130, 8, 0, 0.3),
    "small2": (T.SMALL, 2, 210, 12, 0, 0.3),
    "d512_h16_chunk": (T.LARGE, 2, 200, 10, 16, 0.3),
    "config2_full": (T.CONFIG2, 2, 1000, 40, 0, 0.3),
    "config5_long": (T.CONFIG2, 2, 4000, 150, 0, 1.0),
}
sel = sys.argv[1:] or list(cases)
out = {}
for name in sel:
    cfg, B, Tx, L, chunk, w = cases[name]
    for emu in (True, False):
        r = T.run_case(cfg, B, Tx, L, "bf16", chunk=chunk, ctc_weight=w, round_bf16=True, emulate=emu)
        g, go = r["grads"]
        errs, floor = T.grad_errs(g, go)
        errs = {k: v for k, v in errs.items() if not k.endswith(T.NOISE)}
        noise = T.emu_errors(r)[3] if emu else None
        worst = sorted(((v, k) for k, v in errs.items()), reverse=True)[:5]
        gated = max((v, k) for k, v in errs.items() if T.relu_gated(k))
        lg, lo = r["loss"]
        key = f"{name}_{'emulated' if emu else 'fp64'}"
        out[key] = dict(loss_rel=abs(lg - lo) / abs(lo), h_attn=T.rel(*r["h_attn"]), h_ctc=T.rel(*r["h_ctc"]),
                        worst=worst, worst_relu_gated=gated, worst_incl_zero_grad_tensors=noise)
        print(key, json.dumps(out[key]), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "bf16_errs.json"), "w"), indent=1)
