"""Full-row GEMM + LayerNorm kernels (gemm_row.hip: lasr_linear_res_ln,
lasr_linear_dx_ln_bwd) against the two-launch path they replace (lasr_gemm with its
residual epilogue + lasr_layernorm_fwd / lasr_layernorm2_fwd; lasr_gemm to a bf16 dln +
lasr_layernorm_bwd).  The row kernels keep each output's k order and the norms' lane
layout and summation order, so every output must be BIT-IDENTICAL, incl. the dgamma / dbeta
partial rows and their reduction.  Shapes: the small config's rows (B*T' = 7968) and ragged
row counts, d 256 and 512, K 256 / 512 / 768 / 2048, dropout on and off, with and without
bias, the chained second norm, dres and the branch gradient."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
EPS = 1e-12


def K():
    from liteasr_amd import kernels

    return kernels


def _rn(g, *shape, scale=1.0, dtype=torch.float32):
    return (torch.randn(*shape, generator=g) * scale).to(DEV).to(dtype)


_CTR = []


def _counter():
    """The dropout masks read the registered device step counter: register one that lives as
    long as the process (a freed one would leave the library a dangling pointer)."""
    if not _CTR:
        _CTR.append(torch.full((1,), 3, dtype=torch.int64, device=DEV))
    K().set_dropout_counter(_CTR[0])
    return _CTR[0]


@pytest.mark.parametrize("M,D,Kd,drop,bias,ydt,chain", [
    (7968, 256, 2048, 0.1, True, torch.bfloat16, False),   # FFN fc2 (+ res 0.5) -> next norm
    (7968, 256, 256, 0.1, True, torch.bfloat16, False),    # linear_out / pointwise_conv2
    (7968, 256, 2048, 0.1, True, torch.float32, True),     # last FFN -> final norm + next layer's norm
    (1001, 256, 512, 0.0, False, torch.float32, False),    # ragged rows, no dropout / bias
    (37, 256, 64, 0.3, True, torch.bfloat16, False),       # one partial tile
    (2000, 512, 2048, 0.1, True, torch.bfloat16, False),   # large config width
    (999, 512, 512, 0.1, True, torch.float32, True),
])
def test_linear_res_ln_bit_exact(M, D, Kd, drop, bias, ydt, chain):
    kn = K()
    _counter()
    g = torch.Generator().manual_seed(M + D + Kd)
    x = _rn(g, M, Kd, dtype=torch.bfloat16)
    w = _rn(g, D, Kd, scale=Kd ** -0.5, dtype=torch.bfloat16)
    b = _rn(g, D, scale=0.1) if bias else None
    res = _rn(g, M, D, scale=2.0)
    g1, b1, g2, b2 = (_rn(g, D) for _ in range(4))
    scale = 0.5
    # two-launch reference path
    out0 = torch.empty(M, D, device=DEV)
    kn.linear(x, w, out0, bias=b, res=res, res_scale=scale, drop_p=drop, drop_seed=77)
    y0 = torch.empty(M, D, device=DEV, dtype=ydt)
    m0, r0 = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    z0 = m0b = r0b = None
    if chain:
        z0 = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
        m0b, r0b = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
        kn.layernorm2_fwd(out0, g1, b1, g2, b2, EPS, y0, m0, r0, z0, m0b, r0b)
    else:
        kn.layernorm_fwd(out0, g1, b1, EPS, y0, m0, r0)
    # one launch
    out1, y1 = torch.empty_like(out0), torch.empty_like(y0)
    m1, r1 = torch.empty_like(m0), torch.empty_like(r0)
    kw = {}
    if chain:
        z1, m1b, r1b = torch.empty_like(z0), torch.empty_like(m0b), torch.empty_like(r0b)
        kw = dict(g2=g2, b2=b2, y2=z1, mean2=m1b, rstd2=r1b)
    kn.linear_res_ln(x, w, out1, y1, m1, r1, g1, b1, EPS, bias=b, res=res, res_scale=scale, drop_p=drop,
                     drop_seed=77, **kw)
    pairs = [("out", out0, out1), ("y1", y0, y1), ("mean1", m0, m1), ("rstd1", r0, r1)]
    if chain:
        pairs += [("y2", z0, z1), ("mean2", m0b, m1b), ("rstd2", r0b, r1b)]
    for name, a, c in pairs:
        assert torch.equal(a, c), f"{name}: max diff {(a.float() - c.float()).abs().max().item():.3e}"
    # and the float64 meaning of the first output (the two paths could share a bug)
    ref = x.double() @ w.double().t() + (b.double() if bias else 0.0)
    if drop == 0.0:
        ref = res.double() + scale * ref
        err = (out1.double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-5, err


@pytest.mark.parametrize("M,D,Kd,dres,gb,drop,defer", [
    (7968, 256, 2048, True, True, 0.1, True),    # FFN fc1 dX -> ln_d backward (+dres, branch grad)
    (7968, 256, 768, True, True, 0.1, True),     # q/k/v dX -> ln_b backward
    (7968, 256, 512, True, False, 0.0, False),   # pw1 dX; immediate dgamma / dbeta reduction
    (1001, 256, 256, False, True, 0.2, True),    # ragged rows, no dres
    (21, 256, 64, True, True, 0.1, False),       # one partial 16-row block
    (2000, 512, 2048, True, True, 0.1, True),
    (999, 512, 768, False, False, 0.0, False),
])
def test_linear_dx_ln_bwd_bit_exact(M, D, Kd, dres, gb, drop, defer):
    kn = K()
    _counter()
    g = torch.Generator().manual_seed(M * 3 + D + Kd)
    dy = _rn(g, M, Kd, dtype=torch.bfloat16)
    w = _rn(g, Kd, D, scale=Kd ** -0.5, dtype=torch.bfloat16)
    x = _rn(g, M, D, scale=3.0) + 0.5
    gamma, beta = _rn(g, D), _rn(g, D)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    kn.layernorm_fwd(x, gamma, beta, EPS, torch.empty(M, D, device=DEV), mean, rstd)
    dr = _rn(g, M, D) if dres else None

    def run(fused):
        dx = torch.empty(M, D, device=DEV)
        gbo = torch.empty(M, D, device=DEV, dtype=torch.bfloat16) if gb else None
        dgam, dbet = torch.full((D,), 0.25, device=DEV), torch.full((D,), -0.5, device=DEV)
        kw = dict(dres=dr, gb=gbo, bscale=0.5, bp=drop, bseed=91)
        ctx = kn.deferred_reductions() if defer else _null()
        with ctx:
            if fused:
                kn.linear_dx_ln_bwd(dy, w, x, gamma, mean, rstd, dx, dgam, dbet, **kw)
            else:
                dln = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
                kn.gemm(dy, w, dln)
                kn.layernorm_bwd(x, dln, gamma, mean, rstd, dx, dgam, dbet, **kw)
        return dx, gbo, dgam, dbet

    ref, got = run(False), run(True)
    for name, a, c in zip(("dx", "gb", "dgamma", "dbeta"), ref, got):
        if a is None:
            continue
        assert torch.equal(a, c), f"{name}: max diff {(a.float() - c.float()).abs().max().item():.3e}"


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_row_ln_refuses_bad_shapes():
    """K % 64 != 0 and widths other than 256 / 512 are refused with an error, not computed."""
    from liteasr_amd._native import NativeError

    kn = K()
    x = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(256, 96, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(64, 256, device=DEV)
    st = torch.empty(64, device=DEV)
    gam = torch.ones(256, device=DEV)
    assert not kn.row_ln_ok(x, w, 256)
    with pytest.raises(NativeError, match="multiple of 64"):
        kn.linear_res_ln(x, w, o, o, st, st, gam, gam, EPS, res=o)
    x2 = torch.zeros(64, 128, device=DEV, dtype=torch.bfloat16)
    w2 = torch.zeros(384, 128, device=DEV, dtype=torch.bfloat16)
    assert not kn.row_ln_ok(x2, w2, 384)
