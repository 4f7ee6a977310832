"""Transducer head + RNN-T loss on the GPU (csrc/rnnt.hip, nets/functional.py
TransducerHeadsFn / RNNTLossFn) against the oracles:

* the RNN-T kernels vs oracle/rnnt_ref.py (float64 restatement of the published algorithm,
  pinned by path enumeration and finite differences in tests/test_rnnt.py; the reference's
  own loss is the absent warp-transducer package, so parity against it is UNPINNED):
  loss 1e-5 relative, logits gradient 2e-3 of max (fp32 lattice arithmetic, like the CTC
  kernel's bar) / 2^-7 (bf16 gradient; the oracle is fed the same bf16-rounded logits);
* the whole Transducer step (Conformer encoder, LSTM prediction network, joint, loss) vs
  the reference's own run (tests/golden/transducer.npz, liteasr/models/transducer.py with
  the loss gradient from oracle/rnnt_ref.py): fp32 build h_jnt 2e-4 of max, loss 1e-5
  relative, every parameter gradient 2e-4 of max; bf16 build loss 1e-2 relative, logits
  2e-2 of max, every gradient cosine >= 0.99."""

import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import rnnt_ref  # noqa: E402


def _lattice_case(B, T, U, V, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    xl = torch.randint(max(1, T // 2), T + 1, (B,), generator=g)
    xl[0] = T
    yl = torch.randint(0, U + 1, (B,), generator=g)
    yl[0] = U
    if B > 2:
        yl[1] = 0  # an empty transcript
        xl[2] = 1  # a single frame
    ys = torch.randint(1, V, (B, max(U, 1)), generator=g)
    z = torch.randn(B, T, U + 1, V, generator=g) * 2
    return z, ys, xl, yl


@pytest.mark.parametrize("B,T,U,V,dtype", [(3, 7, 4, 11, torch.float32), (4, 40, 12, 300, torch.float32),
                                           (4, 249, 40, 4233, torch.bfloat16), (2, 60, 150, 97, torch.float32)])
def test_rnnt_kernels_match_restatement(B, T, U, V, dtype):
    from liteasr_amd import kernels as K
    from liteasr_amd.nets.functional import RNNTLossFn

    z, ys, xl, yl = _lattice_case(B, T, U, V, dtype, seed=T + U)
    buf = K.padded_rows(B * T * (U + 1), V, dtype, "cuda").view(B, T, U + 1, V)
    buf.copy_(z.to(dtype))
    zr = buf.double().cpu()  # the values the kernel sees
    logits = buf.requires_grad_()
    loss = RNNTLossFn.apply(logits, ys.int().cuda(), xl.int().cuda(), yl.int().cuda(), 0)
    loss.backward()
    torch.cuda.synchronize()
    lo, nll, go = rnnt_ref.rnnt_batch(zr.numpy(), ys.numpy(), xl.numpy(), yl.numpy())
    assert abs(loss.item() - lo) <= 1e-5 * abs(lo), (loss.item(), lo)
    g = logits.grad.double().cpu().numpy()
    # fp32 lattice: occupancies are exp(alpha + beta - log P) of sums of hundreds of log-probs,
    # so fp32 carries ~|alpha| * 6e-8 relative error into each (measured <= 3e-4 of max at
    # T 60 x U 150); bf16 logits: one bf16 rounding of the gradient on top
    bar = 2e-3 if dtype == torch.float32 else 2 ** -7
    assert np.abs(g - go).max() <= bar * np.abs(go).max(), np.abs(g - go).max() / np.abs(go).max()


def _golden():
    d = np.load(os.path.join(ROOT, "tests", "golden", "transducer.npz"))
    return {k: torch.from_numpy(d[k]) for k in d.files}


def _build(dtype):
    from liteasr_amd.models.transducer import Transducer, TransducerConfig
    from liteasr_amd.utils.cfg import resolve_self

    c = TransducerConfig(input_dim=40, vocab_size=20, enc_dim=64, enc_ff_dim=128, enc_attn_heads=4, enc_layers=2,
                         activation="swish", enc_arch="conformer", dec_dim=16, dec_units=48, dec_layers=2,
                         joint_dim=24, compute_dtype=dtype)
    resolve_self(c)
    return Transducer(c)


def _run(dtype, round_bf16=False):
    from liteasr_amd.criterions.rnnt import RNNTLoss, RNNTLossConfig

    d = _golden()
    init = {k[5:]: v for k, v in d.items() if k.startswith("init.")}
    if round_bf16:
        init = {k: (v.bfloat16().float() if v.is_floating_point() else v) for k, v in init.items()}
    m = _build(dtype)
    missing, unexpected = m.load_state_dict(init, strict=False)
    assert not unexpected and all(k.endswith(".pe") for k in missing), (missing, unexpected)
    m = m.cuda().train()
    xs = d["xs"]
    if round_bf16:
        xs = xs.bfloat16().float()
    crit = RNNTLoss(RNNTLossConfig())
    rec = {}

    class _Rec(torch.nn.Module):
        def forward(self, *a):
            rec["h"] = m(*a)
            return rec["h"]

        def get_target(self, *a):
            return m.get_target(*a)

        def get_pred_len(self, *a):
            return m.get_pred_len(*a)

        def get_target_len(self, *a):
            return m.get_target_len(*a)

    loss = crit(_Rec(), xs.cuda(), d["xlens"].cuda(), d["ys"].cuda(), d["ylens"].cuda())
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}
    return d, loss.item(), rec["h"].detach().double().cpu(), grads


def test_transducer_step_matches_reference_fp32():
    d, loss, h, grads = _run("fp32")
    ref = d["h_jnt"].double()
    assert (h - ref).abs().max().item() <= 2e-4 * ref.abs().max().item()
    assert abs(loss - d["loss"].item()) <= 1e-5 * abs(d["loss"].item()), (loss, d["loss"].item())
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, g in grads.items():
        r = d["grad." + k].double() if "grad." + k in d else torch.zeros_like(g)
        err = (g - r).abs().max().item() / max(r.abs().max().item(), 1e-3 * gmax)
        assert err < 2e-4, (k, err)


def test_transducer_step_matches_reference_bf16():
    d, loss, h, grads = _run("bf16", round_bf16=True)
    ref = d["h_jnt"].double()
    assert (h - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert abs(loss - d["loss"].item()) <= 1e-2 * abs(d["loss"].item()), (loss, d["loss"].item())
    gmax = max(v.abs().max().item() for k, v in d.items() if k.startswith("grad."))
    for k, g in grads.items():
        r = d["grad." + k].double() if "grad." + k in d else torch.zeros_like(g)
        if r.abs().max().item() < 1e-3 * gmax:
            continue
        c = (g.flatten() @ r.flatten()) / (g.norm() * r.norm())
        assert c.item() >= 0.99, (k, c.item())
