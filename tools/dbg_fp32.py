"""Locate fp32-build parity failures: per-tensor gradient errors vs the fp64 oracle for a
few shapes (B, T, layers)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_model_gpu as T  # noqa: E402
from oracle import u2_oracle as O  # noqa: E402

for name, cfg, B, Tx, L in [("l1_T1000", O.default_cfg(enc_layers=1, dec_layers=1), 2, 1000, 40),
                            ("l1_T600", O.default_cfg(enc_layers=1, dec_layers=1), 2, 600, 40),
                            ("l1_T1000_B1", O.default_cfg(enc_layers=1, dec_layers=1), 1, 1000, 40),
                            ("l2_T1000", O.default_cfg(enc_layers=2, dec_layers=1), 2, 1000, 40)]:
    r = T.run_case(cfg, B, Tx, L, "fp32")
    g, go = r["grads"]
    errs, _ = T.grad_errs(g, go)
    lg, lo = r["loss"]
    print(name, "loss", abs(lg - lo) / abs(lo), "h_attn", T.rel(*r["h_attn"]), "h_ctc", T.rel(*r["h_ctc"]), flush=True)
    for v, k in sorted(((v, k) for k, v in errs.items()), reverse=True)[:8]:
        print("   %.3g %s" % (v, k), flush=True)
