"""Times the three CTC kernels (row lse + gather, alpha/beta lattice, gradient) at the small
and long configs through bench.ctc_roofline; one JSON line per config, with a hash of the
kernels' outputs on the same inputs so that library builds compare bit for bit.
LITEASR_HIP_LIB selects the library (ablation builds from tools/gemm_exp.sh, EXP_FILES=ctc)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402
from liteasr_amd.utils.synthetic import synthetic_batch  # noqa: E402


def outputs_hash(cfgd, dev):
    B, L, V = cfgd["B"], cfgd["L"], bench.V
    Tp = ((cfgd["T"] - 3) // 2 + 1 - 3) // 2 + 1
    _, xlens, ys, ylens = synthetic_batch(B, cfgd["T"], L, V, seed=99)
    ilen = (((xlens - 1) // 2 - 1) // 2).to(torch.int32).to(dev)
    tlen, tgt = ylens.to(torch.int32).to(dev), ys.clamp(min=0).to(torch.int32).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    logits = K.padded_rows(B * Tp, V, torch.bfloat16, dev).view(B, Tp, V)
    logits.copy_(torch.randn(B, Tp, V, device=dev, generator=g))
    f32 = dict(dtype=torch.float32, device=dev)
    S = 2 * L + 1
    lse, lp = torch.empty(B * Tp, **f32), torch.empty(B * Tp * (L + 1), **f32)
    alpha, beta, nll = torch.empty(B * Tp * S, **f32), torch.empty(B * Tp * S, **f32), torch.empty(B, **f32)
    grad = K.padded_rows(B * Tp, V, torch.bfloat16, dev).view(B, Tp, V)
    K.ctc_fwd(logits, tgt, ilen, tlen, lse, lp, alpha, nll, beta=beta)
    K.ctc_bwd(logits, tgt, ilen, tlen, lse, lp, alpha, nll, beta, grad, 1.0 / B, beta_ready=True)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (lse, lp, alpha, beta, nll, grad.view(torch.int16)):
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()[:16]


dev = torch.device("cuda:0")
for name in (sys.argv[1:] or ["small", "long"]):
    r = bench.ctc_roofline(bench.CONFIGS[name], dev, iters=50)
    print(json.dumps({"cfg": name, "gather_us": r["gather_us"], "lattice_us": r["lattice_us"],
                      "grad_us": r["grad_us"], "hash": outputs_hash(bench.CONFIGS[name], dev)}), flush=True)
