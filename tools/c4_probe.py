"""Probe: config-4 decoder logits error (fp32 build vs the fp64 oracle) across variants."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import u2_oracle as O  # noqa: E402
import test_model_gpu as TM  # noqa: E402

base = dict(enc_dim=512, enc_heads=16, enc_ff=2048, enc_layers=12, dec_dim=512, dec_heads=16, dec_ff=2048,
            dec_layers=6, vocab_size=4233)
variants = [
    ("config4", {}, 1000, 40, 16),
    ("chunk0", {}, 1000, 40, 0),
    ("enc2", dict(enc_layers=2), 1000, 40, 16),
    ("dec1", dict(dec_layers=1), 1000, 40, 16),
    ("dec2", dict(dec_layers=2), 1000, 40, 16),
    ("L10", {}, 1000, 10, 16),
    ("T200", {}, 200, 40, 16),
    ("H4", dict(enc_heads=4, dec_heads=4), 1000, 40, 16),
    ("d256H16", dict(enc_dim=256, dec_dim=256), 1000, 40, 16),
]
sel = sys.argv[1:]
for name, kw, T, L, chunk in variants:
    if sel and name not in sel:
        continue
    cfg = O.default_cfg(**{**base, **kw})
    r = TM.run_case(cfg, 2, T, L, "fp32", chunk=chunk)
    lg, lo = r["loss"]
    g, go = r["grads"]
    errs, _ = TM.grad_errs(g, go)
    worst = max((v, k) for k, v in errs.items() if not k.startswith("encoder.embed.conv."))
    print(f"{name}: loss {abs(lg - lo) / abs(lo):.2e} h_attn {TM.rel(*r['h_attn']):.2e} h_ctc {TM.rel(*r['h_ctc']):.2e} "
          f"worst {worst[0]:.2e} {worst[1]}", flush=True)
