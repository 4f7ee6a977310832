"""Op-level parity of every HIP kernel against a plain PyTorch fp32/fp64 reference of
the same op (run on the GPU box).  Tolerances: fp32 storage 1e-4 relative to the
tensor's max-abs; bf16 storage 2e-2 (bf16 has an 8-bit mantissa)."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def K():
    from liteasr_amd import kernels

    return kernels


def close(got, ref, tol, what=""):
    got = got.float().cpu()
    ref = ref.float().cpu()
    scale = ref.abs().max().item() + 1e-12
    err = (got - ref).abs().max().item() / scale
    assert err <= tol, f"{what}: max err {err:.3e} > {tol:.1e} (scale {scale:.3e})"


# ------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,Kd", [(1, 1, 1), (37, 53, 29), (130, 70, 257), (300, 260, 96), (64, 128, 2304)])
def test_gemm_layouts(dtype, ta, tb, M, N, Kd):
    g = torch.Generator(device="cpu").manual_seed(M * 1000 + N + Kd)
    A = torch.randn(M, Kd, generator=g)
    B = torch.randn(Kd, N, generator=g)
    a = (A.t().contiguous().t() if ta else A).to(DEV, dtype)
    b = (B.t().contiguous().t() if tb else B).to(DEV, dtype)
    c = torch.empty(M, N, device=DEV, dtype=torch.float32)
    K().gemm(a, b, c)
    ref = a.double() @ b.double()
    close(c, ref, 1e-5 if dtype == torch.float32 else 1e-2, "gemm")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    kn = K()
    from liteasr_amd import _native as Nn

    M, N, Kd = 200, 96, 64
    x = torch.randn(M, Kd, device=DEV).to(dtype)
    w = torch.randn(N, Kd, device=DEV).to(dtype)
    bias = torch.randn(N, device=DEV)
    base = x.double() @ w.double().t()
    # bias + swish with pre-activation out
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    z = torch.empty(M, N, device=DEV, dtype=dtype)
    kn.linear(x, w, out, bias=bias, act=Nn.ACT_SWISH, zout=z)
    zr = base + bias.double()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    close(z, zr, tol, "zout")
    close(out, zr * torch.sigmoid(zr), tol, "swish")
    # relu
    kn.linear(x, w, out, bias=bias, act=Nn.ACT_RELU)
    close(out, torch.relu(zr), tol, "relu")
    # residual add with scale (fp32 residual), alpha
    res = torch.randn(M, N, device=DEV)
    o32 = torch.empty(M, N, device=DEV)
    kn.linear(x, w, o32, bias=bias, res=res, res_scale=0.5, alpha=2.0)
    close(o32, res.double() + 0.5 * (2 * base + bias.double()), tol, "residual")
    # aux swish-grad multiply
    aux = torch.randn(M, N, device=DEV).to(dtype)
    kn.linear(x, w, o32, aux=aux, aux_act=Nn.ACT_SWISH)
    s = torch.sigmoid(aux.double())
    close(o32, base * s * (1 + aux.double() * (1 - s)), tol, "aux swish")
    kn.linear(x, w, o32, aux=aux, aux_act=Nn.ACT_RELU)
    close(o32, base * (aux.double() > 0), tol, "aux relu")
    # gate output (zout_mode 1): act'(pre-activation) * dropout keep flag, and its use as
    # an aux multiplier (aux_act GATE) with the dropout scale as alpha
    for act, dact in ((Nn.ACT_SWISH, lambda t: torch.sigmoid(t) * (1 + t * (1 - torch.sigmoid(t)))),
                      (Nn.ACT_RELU, lambda t: (t > 0).double())):
        kn.linear(x, w, out, bias=bias, act=act, zout=z, zout_mode=1)
        close(z, dact(zr), tol, "gate")
        kn.linear(x, w, out, bias=bias, act=act, zout=z, zout_mode=1, drop_p=0.2, drop_seed=77)
        keep = torch.empty(M, N, device=DEV)
        kn.branch_grad(torch.ones(M, N, device=DEV), keep, 1.0, 0.2, 77)
        keep = (keep > 0).double()
        close(z, dact(zr) * keep, tol, "gate with dropout")
        act_fn = (lambda t: t * torch.sigmoid(t)) if act == Nn.ACT_SWISH else torch.relu
        close(out, act_fn(zr) * keep * kn.dropout_scale(0.2), tol, "activation with dropout")
    kn.linear(x, w, o32, aux=aux, aux_act=Nn.ACT_GATE, alpha=1.25)
    close(o32, 1.25 * base * aux.double(), tol, "aux gate")
    # beta accumulate + alpha_dev
    acc = torch.randn(M, N, device=DEV)
    acc0 = acc.clone()
    ad = torch.tensor([3.0], device=DEV)
    kn.linear(x, w, acc, beta=1.0, alpha_dev=ad)
    close(acc, acc0.double() + 3 * base, tol, "beta/alpha_dev")


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_large_tiles_bf16(ta, tb):
    """Shapes that select the 128x128 tile (>= 512 workgroups): K-contiguous and
    transposed-read (ds_read_b64_tr_b16) LDS images on both operands, ragged M."""
    M, N, Kd = 4100, 2048, 96
    g = torch.Generator(device="cpu").manual_seed(7)
    A = torch.randn(M, Kd, generator=g)
    B = torch.randn(Kd, N, generator=g)
    a = (A.t().contiguous().t() if ta else A).to(DEV, torch.bfloat16)
    b = (B.t().contiguous().t() if tb else B).to(DEV, torch.bfloat16)
    c = torch.empty(M, N, device=DEV, dtype=torch.float32)
    K().gemm(a, b, c)
    close(c, a.cpu().double() @ b.cpu().double(), 1e-2, "gemm128")


def test_gemm_large_tile_epilogues_bf16():
    """Register-prefetched epilogue (bias once per thread, one aux/res source prefetched)
    on 128x128 tiles with a ragged last row tile."""
    kn = K()
    from liteasr_amd import _native as Nn

    M, N, Kd = 4100, 2048, 64
    x = torch.randn(M, Kd, device=DEV).bfloat16()
    w = torch.randn(N, Kd, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV)
    base = (x.double() @ w.double().t()).cpu()
    zr = base + bias.double().cpu()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    z = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    kn.linear(x, w, out, bias=bias, act=Nn.ACT_SWISH, zout=z)
    close(z, zr, 2e-2, "zout128")
    close(out, zr * torch.sigmoid(zr), 2e-2, "swish128")
    res = torch.randn(M, N, device=DEV)
    o32 = torch.empty(M, N, device=DEV)
    kn.linear(x, w, o32, bias=bias, res=res, res_scale=0.5)
    close(o32, res.double().cpu() + 0.5 * zr, 2e-2, "res128")
    aux = torch.randn(M, N, device=DEV).bfloat16()
    kn.linear(x, w, o32, aux=aux, aux_act=Nn.ACT_SWISH)
    s = torch.sigmoid(aux.double().cpu())
    close(o32, base * s * (1 + aux.double().cpu() * (1 - s)), 2e-2, "aux128")


def test_gemm_padded_vocab_bf16():
    """Vocab GEMMs on [rows, V] views of [rows, roundup8(V)] buffers: ragged-N fast epilogue
    (bias), dX with a padded K-contiguous A, and the dW product whose M-contiguous A
    (g^T) is LDS-DMA loaded through the padding columns."""
    kn = K()
    rows, V, d = 3000, 4233, 256
    g = torch.Generator().manual_seed(5)
    hd = torch.randn(rows, d, generator=g).to(DEV, torch.bfloat16)
    W = torch.randn(V, d, generator=g).to(DEV, torch.bfloat16)
    b = torch.randn(V, generator=g).to(DEV)
    logits = kn.padded_rows(rows, V, torch.bfloat16, DEV)
    kn.linear(hd, W, logits, bias=b)
    ref = hd.cpu().double() @ W.cpu().double().t() + b.cpu().double()
    close(logits, ref, 2e-2, "padded logits")
    gl = torch.full((rows, 4240), float("nan"), dtype=torch.bfloat16, device=DEV)[:, :V]
    gl.copy_(torch.randn(rows, V, generator=g))  # padding columns stay NaN: must not leak
    dx = torch.empty(rows, d, device=DEV)
    kn.gemm(gl, W, dx)
    close(dx, gl.cpu().double() @ W.cpu().double(), 1e-2, "padded dX")
    dW = torch.zeros(V, d, device=DEV)
    kn.gemm(gl.t(), hd, dW, beta=1.0, split_k=0)
    close(dW, gl.cpu().double().t() @ hd.cpu().double(), 1e-2, "padded dW")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_splitk_and_batched(dtype):
    kn = K()
    # dW-style TN gemm with split-K accumulate
    R, N1, K1 = 3001, 96, 160
    dy = torch.randn(R, N1, device=DEV).to(dtype)
    x = torch.randn(R, K1, device=DEV).to(dtype)
    dw = torch.randn(N1, K1, device=DEV)
    dw0 = dw.clone()
    kn.gemm(dy.t(), x, dw, beta=1.0, split_k=0)
    ref = dw0.double() + dy.double().t() @ x.double()
    close(dw, ref, 1e-5 if dtype == torch.float32 else 1e-2, "splitk")
    # 2-level batched with head-strided views (attention layout)
    B, T, H, dk = 3, 41, 4, 16
    qkv = torch.randn(B, T, 3, H, dk, device=DEV).to(dtype)
    q = qkv[:, :, 0].permute(0, 2, 1, 3)  # (B,H,T,dk) strided
    k = qkv[:, :, 1].permute(0, 2, 1, 3)
    S = torch.empty(B, H, T, 48, device=DEV)
    kn.gemm(q, k.transpose(-1, -2), S[..., :T], alpha=0.25)
    ref = 0.25 * (q.double() @ k.double().transpose(-1, -2))
    close(S[..., :T], ref, 1e-5 if dtype == torch.float32 else 1e-2, "batched")
    # broadcast operand (stride-0 batch) like the shared positional projection
    p = torch.randn(T, H, dk, device=DEV).to(dtype).permute(1, 0, 2).unsqueeze(0).expand(B, H, T, dk)
    kn.gemm(q, p.transpose(-1, -2), S[..., :T])
    close(S[..., :T], q.double() @ p.double().transpose(-1, -2), 1e-5 if dtype == torch.float32 else 1e-2, "bcast")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,M,N,split", [(7968, 256, 2048, 0), (7968, 2048, 256, 0), (3001, 96, 160, 0),
                                         (517, 64, 80, 1), (20000, 768, 256, 0), (333, 130, 40, 1)])
def test_gemm_fused_rowsum(dtype, R, M, N, split):
    """dW GEMM with the fused bias gradient: rowsum[m] += sum_k dY^T[m, k] (split-K
    partials summed by the reduce kernel, or written directly without split; fallback
    column sum on the non-LDS-DMA paths)."""
    kn = K()
    g = torch.Generator().manual_seed(R + M + N)
    dy = torch.randn(R, M, generator=g).to(DEV, dtype)
    x = torch.randn(R, N, generator=g).to(DEV, dtype)
    dw = torch.randn(M, N, generator=g).to(DEV)
    db = torch.randn(M, generator=g).to(DEV)
    dw0, db0 = dw.double().cpu(), db.double().cpu()
    kn.gemm(dy.t(), x, dw, beta=1.0, split_k=split, rowsum=db)
    close(dw, dw0 + dy.double().cpu().t() @ x.double().cpu(), 1e-5 if dtype == torch.float32 else 1e-2, "dW")
    ref_b = db0 + dy.double().cpu().sum(0)
    close(db, ref_b, 1e-5, "db")
    # padded-vocab view (row stride 4240 > M = 4233)
    if R == 3001:
        V = 4233
        gl = torch.full((R, 4240), float("nan"), dtype=dtype, device=DEV)[:, :V]
        gl.copy_(torch.randn(R, V, generator=g))
        dW = torch.zeros(V, N, device=DEV)
        bv = torch.zeros(V, device=DEV)
        kn.gemm(gl.t(), x, dW, beta=1.0, split_k=0, rowsum=bv)
        close(bv, gl.double().cpu().sum(0), 1e-5, "padded db")


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("M,N,Kd,tile", [(4100, 2048, 256, (0, 0)), (1000, 256, 96, (64, 64)),
                                         (1000, 256, 100, (128, 64)), (999, 384, 160, (64, 128)),
                                         (700, 512, 224, (128, 128)), (700, 512, 2048, (128, 256))])
def test_gemm_ksub2_bit_identical(ta, tb, M, N, Kd, tile):
    """64-deep ring stages (two 32-deep sub-tiles per wait + barrier, per-call ksub = 2)
    accumulate in the same k order as 32-deep stages: outputs bit-identical, including a
    leftover 32-deep sub-tile (K % 64 = 32), a ragged tail (K % 32 != 0), epilogues, and
    split-K weight gradients with the fused bias rowsum."""
    kn = K()
    from liteasr_amd import _native as Nn

    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randn(M, Kd, generator=g)
    B = torch.randn(Kd, N, generator=g)
    a = (A.t().contiguous().t() if ta else A).to(DEV, torch.bfloat16)
    b = (B.t().contiguous().t() if tb else B).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    dy = torch.randn(3001, M, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(3001, N, generator=g).to(DEV, torch.bfloat16)
    outs = []
    tl = tile if tile != (0, 0) else None
    for ks in (1, 2):
        c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        z = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        kn.gemm(a, b, c, bias=bias, act=Nn.ACT_SWISH, zout=z, tile=tl, ksub=ks)
        o32 = torch.empty(M, N, device=DEV)
        kn.gemm(a, b, o32, bias=bias, res=res, res_scale=0.5, tile=tl, ksub=ks)
        dw = torch.ones(M, N, device=DEV)
        db = torch.ones(M, device=DEV)
        kn.gemm(dy.t(), x, dw, beta=1.0, split_k=0, rowsum=db, tile=tl, ksub=ks)
        torch.cuda.synchronize()
        outs.append((c, z, o32, dw, db))
    for name, u, v in zip(("out", "zout", "res", "dW", "db"), outs[0], outs[1]):
        assert torch.equal(u, v), f"ksub 2 differs from ksub 1: {name}"
    ref = (a.double() @ b.double()).cpu() + bias.double().cpu()
    close(outs[1][1], ref, 1e-2, "zout")


@pytest.mark.parametrize("R", [3001, 7968])
def test_gemm_dw_group_bit_identical(R, monkeypatch):
    """Grouped split-K weight gradients (lasr_gemm_dw_group: the dW GEMMs of a backward node
    queued with group=True and launched together at the end of deferred_reductions) give
    the same dW bits as one lasr_gemm launch per problem at the same K slicing, with and
    without the fused bias rowsum, accumulating (beta 1) and overwriting (beta 0); with the
    default fewer slices they match float64 at the bf16 bar."""
    kn = K()
    g = torch.Generator().manual_seed(R)
    probs = [(2048, 256, True, 1.0), (256, 2048, True, 1.0), (256, 256, True, 1.0), (768, 256, True, 0.0),
             (512, 256, False, 1.0), (2048, 256, True, 1.0), (256, 256, False, 1.0)]
    ins = [(torch.randn(R, M, generator=g).to(DEV, torch.bfloat16), torch.randn(R, N, generator=g).to(DEV, torch.bfloat16),
            torch.randn(M, N, generator=g).to(DEV), torch.randn(M, generator=g).to(DEV) if rs else None, beta)
           for M, N, rs, beta in probs]
    outs = {}
    default_div = kn.DW_GROUP_SPLIT_DIV
    monkeypatch.setattr(kn, "DW_GROUP_SPLIT_DIV", 1)  # same K slices as the lone launches: same bits
    for grouped in (False, True, "fewer-slices"):
        if grouped == "fewer-slices":
            monkeypatch.setattr(kn, "DW_GROUP_SPLIT_DIV", default_div)
        res = []
        with kn.deferred_reductions():
            for dy, x, dw0, db0, beta in ins:
                dw = dw0.clone()
                db = db0.clone() if db0 is not None else None
                kn.gemm(dy.t(), x, dw, beta=beta, split_k=0, rowsum=db, group=grouped)
                res.append((dw, db))
            assert (len(kn._DEFER.gemms) > 0) == (bool(grouped) and kn.DW_GROUP)
        torch.cuda.synchronize()
        outs[grouped] = res
    for (a, ab), (b, bb) in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
        if ab is not None:
            # FFN-sized plans run on 128 x 128 group tiles: their rowsum partials group the k
            # rows per thread differently (rowsum_tile<BM>), so they agree to fp32 rounding
            assert torch.allclose(ab, bb, rtol=1e-6, atol=1e-4)
    for (dy, x, dw0, db0, beta), (dw, db) in zip(ins, outs["fewer-slices"]):
        ref = beta * dw0.double() + dy.double().t() @ x.double()
        close(dw, ref, 1e-2, "grouped dW")
        if db0 is not None:
            close(db, db0.double() + dy.double().sum(0), 1e-5, "grouped db")


@pytest.mark.parametrize("R", [7968, 1312])
def test_gemm_dw_group_direct(R, monkeypatch):
    """Direct problems of the grouped weight-gradient launch (the d 512 FFN weights: >=
    DW_DIRECT_MIN_TILES 128 x 128 tiles each): full-K tiles write the gradient itself (beta 1 or 0)
    and add the bias rowsum, no partial slab.  dW is bit-identical to one lasr_gemm launch per
    problem with no K split (a tile's shape never changes an output's k order); the rowsum agrees
    to fp32 rounding (k rows grouped per thread by tile height) and both match float64."""
    kn = K()
    monkeypatch.setattr(kn, "DW_DIRECT_MIN_TILES", 64)  # (off in the product: slower)
    g = torch.Generator().manual_seed(R + 1)
    probs = [(2048, 512, True, 1.0), (512, 2048, True, 1.0), (2048, 512, False, 0.0), (512, 2048, True, 0.0)]
    ins = [(torch.randn(R, M, generator=g).to(DEV, torch.bfloat16), torch.randn(R, N, generator=g).to(DEV, torch.bfloat16),
            torch.randn(M, N, generator=g).to(DEV), torch.randn(M, generator=g).to(DEV) if rs else None, beta)
           for M, N, rs, beta in probs]
    outs = {}
    for grouped in (False, True):
        res = []
        with kn.deferred_reductions():
            for dy, x, dw0, db0, beta in ins:
                dw = dw0.clone()
                db = db0.clone() if db0 is not None else None
                kn.gemm(dy.t(), x, dw, beta=beta, split_k=0 if grouped else 1, rowsum=db, group=grouped)
                res.append((dw, db))
            if grouped:
                keys = {k for k, _, _ in kn._DEFER.gemms}
                assert keys == {(128, 128, "direct")}, keys
            assert not kn._DEFER.segs  # no partial slab to reduce
        torch.cuda.synchronize()
        outs[grouped] = res
    for (a, ab), (b, bb), (dy, x, dw0, db0, beta) in zip(outs[False], outs[True], ins):
        assert torch.equal(a, b)
        ref = beta * dw0.double() + dy.double().t() @ x.double()
        close(b, ref, 1e-2, "direct dW")
        if ab is not None:
            assert torch.allclose(ab, bb, rtol=1e-6, atol=1e-4)
            close(bb, db0.double() + dy.double().sum(0), 1e-5, "direct db")


@pytest.mark.parametrize("B,H,Tq,Tk,dk,qmask,splits", [(8, 4, 151, 999, 64, False, (2, 3, 4, 5)),
                                                      (3, 2, 70, 300, 32, True, (2, 5)),
                                                      (2, 4, 41, 249, 64, False, (4,))])
def test_attn_key_split(B, H, Tq, Tk, dk, qmask, splits):
    """lasr_attn_fwd_split / lasr_attn_bwd_split (keys split over workgroups, combined in
    a second launch) against the one-pass entries on the same inputs: the decoder's source
    attention at the long config (T' 999, the split the heuristic picks: 4), uneven splits
    (3, 5 of 16 key blocks), a query-dependent mask with a fully masked utterance, d_k 32 and
    one key block per split.  Same values up to fp32 summation order: the row maxima
    exactly, ctx / D / dq / dk / dv within a bf16 ulp of the largest value."""
    kn = K()
    g = torch.Generator().manual_seed(Tk + dk)
    bf = torch.bfloat16
    D = H * dk
    q = (torch.randn(B * Tq, D, generator=g) * 0.5).to(DEV, bf)
    kv = (torch.randn(B * Tk, 2 * D, generator=g) * 0.5).to(DEV, bf)
    k, v = kv[:, :D], kv[:, D:]
    if qmask:
        m = torch.rand(B, Tq, Tk, generator=g) < 0.3
        m[1] = True  # one utterance fully masked: uniform attention rows
        mask, msb, msq = kn.pad_mask16(m.to(torch.uint8).to(DEV), B, Tq, Tk)
    else:
        lens = torch.randint(Tk // 2, Tk + 1, (B,), generator=g)
        lens[0] = Tk
        mask = (torch.arange(Tk)[None, :] >= lens[:, None]).to(torch.uint8).to(DEV)
        msb, msq = Tk, 0
    scale = dk ** -0.5
    dctx = (torch.randn(B * Tq, D, generator=g) * 0.5).to(DEV, bf)

    def run(ns):
        stats = torch.empty(B * H * Tq * 2, device=DEV)
        ctx = torch.empty(B * Tq, D, device=DEV, dtype=bf)
        kn.attn_fwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, nsplit=ns)
        Dbuf = torch.empty(B * H * Tq, device=DEV)
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        kn.attn_bwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dq, dkv[:, :D], dkv[:, D:],
                    nsplit=ns)
        torch.cuda.synchronize()
        return stats.view(-1, 2), ctx, Dbuf, dq, dkv

    if not qmask and (B, H, Tq, Tk) == (8, 4, 151, 999):
        assert kn.attn_split(B, H, Tq, Tk) == 4
    base = run(1)
    for ns in splits:
        st, ctx, Db, dq, dkv = run(ns)
        assert torch.equal(st[:, 0], base[0][:, 0]), f"row maxima differ (nsplit {ns})"
        close(st[:, 1], base[0][:, 1], 1e-5, f"1/sum nsplit {ns}")
        close(ctx, base[1], 8e-3, f"ctx nsplit {ns}")
        close(Db, base[2], 8e-3, f"D nsplit {ns}")  # rowsum(dO * O): O is the (re-rounded) ctx
        close(dq, base[3], 8e-3, f"dq nsplit {ns}")
        close(dkv, base[4], 8e-3, f"dk/dv nsplit {ns}")
        assert torch.isfinite(ctx.float()).all() and torch.isfinite(dq.float()).all()


@pytest.mark.parametrize("kind", ["self-masked", "self-nomask", "source"])
def test_decoder_attention_fused_matches_materialised(kind, monkeypatch):
    """Decoder attention on the fused kernels without the positional term (lasr_attn_fwd /
    lasr_attn_bwd through functional.mha_forward / mha_backward, LASR_FUSED_DEC_ATTN)
    against the materialised-score path on the same inputs: self attention with the causal +
    key-padding mask (U2) or none (Paraformer's parallel decoder), and source attention over
    an encoder output (Tq 41 != Tk 249, key padding); B 32, d 256, 4 heads, bf16."""
    from types import SimpleNamespace as NS

    from liteasr_amd.nets import functional as Fn

    g = torch.Generator().manual_seed(len(kind))
    B, Tq, d, H = 32, 41, 256, 4
    Tk = Tq if kind != "source" else 249
    R = B * Tq
    sc = lambda *shape, f=0.08: (torch.randn(*shape, generator=g) * f)  # noqa: E731
    ln = torch.randn(R, d, generator=g).to(DEV, torch.bfloat16)
    x_in = torch.randn(R, d, generator=g).to(DEV)
    gb = torch.randn(R, d, generator=g).to(DEV, torch.bfloat16)
    w = NS(Wo=sc(d, d).to(DEV, torch.bfloat16), bo=sc(d, f=0.1).to(DEV))
    if kind == "source":
        mem = torch.randn(B * Tk, d, generator=g).to(DEV, torch.bfloat16)
        w.Wq, w.bq = sc(d, d).to(DEV, torch.bfloat16), sc(d, f=0.1).to(DEV)
        w.Wkv, w.bkv = sc(2 * d, d).to(DEV, torch.bfloat16), sc(2 * d, f=0.1).to(DEV)
        lens = torch.randint(150, Tk + 1, (B,), generator=g)
        m = torch.arange(Tk)[None, :] >= lens[:, None]
        mask, msb, msq = m.to(torch.uint8).to(DEV), Tk, 0
    else:
        mem = None
        w.Wqkv, w.bqkv = sc(3 * d, d).to(DEV, torch.bfloat16), sc(3 * d, f=0.1).to(DEV)
        if kind == "self-masked":
            lens = torch.randint(5, Tq + 1, (B,), generator=g)
            j = torch.arange(Tq)
            m = (j[None, None, :] > j[None, :, None]) | (j[None, None, :] >= lens[:, None, None])
            mask, msb, msq = m.to(torch.uint8).to(DEV), Tq * Tq, Tq
        else:
            mask, msb, msq = None, 0, 0
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(Fn, "FUSED_DEC_ATTN", fused)
        grads = NS(**{k: torch.zeros_like(v, dtype=torch.float32) for k, v in vars(w).items()})
        dmem = torch.zeros(B * Tk, d, device=DEV) if mem is not None else None
        out, sv = Fn.mha_forward(ln, mem, w, B, Tq, Tk, H, mask, msb, msq, x_in, 0.0, 0, 0.0, 0)
        assert (sv.stats is not None) == fused
        dln = Fn.mha_backward(gb, ln, mem, sv, w, grads, B, Tq, Tk, H, mask, msb, msq, 0.0, 0, dmem)
        torch.cuda.synchronize()
        res[fused] = (out.float(), dln.float(), dmem, grads)
    (o0, d0, m0, g0), (o1, d1, m1, g1) = res[False], res[True]
    close(o1, o0, 1e-2, "out")
    close(d1, d0, 2e-2, "dln")
    if m0 is not None:
        close(m1, m0, 2e-2, "dmem")
    for k in vars(g0):
        close(getattr(g1, k), getattr(g0, k), 2e-2, k)


def test_gemm_dropout_matches_branch_grad():
    kn = K()
    M, N, Kd = 128, 256, 64
    x = torch.randn(M, Kd, device=DEV)
    w = torch.randn(N, Kd, device=DEV)
    out = torch.empty(M, N, device=DEV)
    kn.linear(x, w, out, drop_p=0.1, drop_seed=1234)
    ref = x @ w.t()
    mask = torch.empty(M, N, device=DEV)
    kn.branch_grad(torch.ones(M, N, device=DEV), mask, 1.0, 0.1, 1234)
    close(out, ref * mask, 1e-5, "dropout consistency")
    keep = (mask > 0).float().mean().item()
    assert abs(keep - 0.9) < 0.01, keep
    sc = kn.dropout_scale(0.1)
    assert sc == pytest.approx(65536 / (65536 - 6554), rel=1e-7)
    assert torch.equal(mask[mask > 0], torch.full_like(mask[mask > 0], sc))
    # pairs of elements share one draw (16-bit halves): check both halves are used, i.e.
    # the two elements of a pair are not copies of one decision
    kp = (mask > 0).view(-1, 2)
    assert (kp[:, 0] != kp[:, 1]).float().mean().item() > 0.1


# ------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [64, 256, 512])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm(D, dtype):
    kn = K()
    rows = 333
    x = (torch.randn(rows, D, device=DEV) * 3 + 1)
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    y = torch.empty(rows, D, device=DEV, dtype=dtype)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    kn.layernorm_fwd(x, g, b, 1e-12, y, mean, rstd)
    xr = x.double().requires_grad_()
    yr = F.layer_norm(xr, (D,), g.double(), b.double(), 1e-12)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(y, yr, tol, "ln fwd")
    dy = torch.randn(rows, D, device=DEV)
    dres = torch.randn(rows, D, device=DEV)
    dx = torch.empty(rows, D, device=DEV)
    dg = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    gb = torch.empty(rows, D, device=DEV, dtype=dtype)
    kn.layernorm_bwd(x, dy, g, mean, rstd, dx, dg, db, dres=dres, gb=gb, bscale=0.5)
    gr = torch.autograd.grad(yr, xr, dy.double())[0]
    close(dx, gr + dres.double(), 1e-5, "ln dx")
    close(gb, 0.5 * (gr + dres.double()), tol, "ln gb")
    xh = (x.double() - x.double().mean(-1, keepdim=True)) / x.double().var(-1, unbiased=False, keepdim=True).add(1e-12).sqrt()
    close(dg, (dy.double() * xh).sum(0), 1e-5, "ln dgamma")
    close(db, dy.double().sum(0), 1e-5, "ln dbeta")


@pytest.mark.parametrize("D", [256, 512])
def test_layernorm2_chained_bit_exact(D):
    """lasr_layernorm2_fwd (a layer's final norm chained with the next layer's first norm)
    gives the same bits as two lasr_layernorm_fwd launches: y fp32 + stats, z bf16 + stats."""
    kn = K()
    rows = 1001
    g = torch.Generator().manual_seed(D)
    x = (torch.randn(rows, D, generator=g) * 3 + 0.5).to(DEV)
    g1, b1, g2, b2 = (torch.randn(D, generator=g).to(DEV) for _ in range(4))
    y0, m0, r0 = torch.empty(rows, D, device=DEV), torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    z0 = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    m0b, r0b = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    kn.layernorm_fwd(x, g1, b1, 1e-12, y0, m0, r0)
    kn.layernorm_fwd(y0, g2, b2, 1e-12, z0, m0b, r0b)
    y1, m1, r1 = torch.empty_like(y0), torch.empty_like(m0), torch.empty_like(r0)
    z1, m1b, r1b = torch.empty_like(z0), torch.empty_like(m0b), torch.empty_like(r0b)
    kn.layernorm2_fwd(x, g1, b1, g2, b2, 1e-12, y1, m1, r1, z1, m1b, r1b)
    for a, b in ((y0, y1), (m0, m1), (r0, r1), (z0, z1), (m0b, m1b), (r0b, r1b)):
        assert torch.equal(a, b)


def test_colsum():
    kn = K()
    x = torch.randn(1000, 300, device=DEV).bfloat16()
    out = torch.ones(300, device=DEV)
    kn.colsum(x, out, accumulate=True)
    close(out, 1 + x.double().sum(0), 1e-5, "colsum")


# ------------------------------------------------------------------------- CTC
def _ctc_case(B, T, V, L, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, T, V, generator=g) * 2
    ilen = torch.randint(max(1, T // 2), T + 1, (B,), generator=g)
    ilen[0] = T
    tlen = torch.randint(0, L + 1, (B,), generator=g)
    tlen[0] = L
    tg = torch.randint(1, V, (B, L), generator=g)
    if L >= 3:
        tg[0, 1] = tg[0, 0]  # repeated label
    for b in range(B):
        tg[b, tlen[b]:] = -1
    return logits.to(dtype), tg, ilen, tlen


@pytest.mark.parametrize("B,T,V,L", [(4, 50, 30, 12), (3, 249, 4233, 40), (2, 120, 200, 70),
                                     (2, 999, 4233, 150)])  # SURVEY §8c F-c sizes, long config
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ctc(B, T, V, L, dtype):
    kn = K()
    logits, tg, ilen, tlen = _ctc_case(B, T, V, L, B * T + L, dtype)
    if L == 70:
        ilen[1] = 30  # infeasible: 2*L_b+... > T_b when tlen[1] large
        tlen[1] = 60
        tg[1, :60] = torch.randint(1, V, (60,))
        tg[1, 60:] = -1
    # reference: fp64 CPU log_softmax -> ctc_loss(sum) and autograd
    lr = logits.double().requires_grad_()
    lp = lr.log_softmax(-1).transpose(0, 1)
    nll_ref = F.ctc_loss(lp, tg.clamp(min=0), ilen, tlen, blank=0, reduction="none", zero_infinity=False)
    gref = torch.autograd.grad(nll_ref[torch.isfinite(nll_ref)].sum(), lr)[0]
    d_log = logits.to(DEV)
    tg32 = tg.to(DEV, torch.int32)
    il = ilen.to(DEV, torch.int32)
    tl = tlen.to(DEV, torch.int32)
    S = 2 * L + 1
    lse = torch.empty(B * T, device=DEV)
    lpb = torch.empty(B * T * (L + 1), device=DEV)
    alpha = torch.empty(B * T * S, device=DEV)
    beta = torch.empty(B * T * S, device=DEV)
    nll = torch.empty(B, device=DEV)
    kn.ctc_fwd(d_log, tg32, il, tl, lse, lpb, alpha, nll)
    fin = torch.isfinite(nll_ref)
    tol = 1e-5 if dtype == torch.float32 else 1e-5
    got = nll.cpu().double()
    assert torch.equal(torch.isfinite(got), fin), (got, nll_ref)
    assert ((got[fin] - nll_ref[fin].detach()).abs() <= tol * nll_ref[fin].detach().abs().clamp(min=1)).all(), (got, nll_ref)
    grad = torch.empty(B, T, V, device=DEV, dtype=torch.float32)
    kn.ctc_bwd(d_log, tg32, il, tl, lse, lpb, alpha, nll, beta, grad, 1.0)
    gg = grad.cpu().double()
    # The bar is the reference's own fp32 path (aten fp32 ctc_loss, what LiteASR runs):
    # its max-abs gradient error vs fp64 is 5.8e-4 at 249x4233 and 1.1e-2 at the long
    # 999x4233, L 150 case (the lattice sums thousands of nats in fp32).  Allow
    # max(2e-3, 1.25 x that error), measured here on the same logits.
    l32 = logits.float().requires_grad_()
    n32 = F.ctc_loss(l32.log_softmax(-1).transpose(0, 1), tg.clamp(min=0), ilen, tlen, blank=0,
                     reduction="none", zero_infinity=False)
    g32 = torch.autograd.grad(n32[torch.isfinite(n32)].sum(), l32)[0].double()
    err32 = (g32[fin] - gref[fin]).abs().max().item()
    close(gg[fin], gref[fin], max(2e-3, 1.25 * err32), "ctc grad")
    # beta computed in the forward launch (alongside alpha): identical results
    alpha2, beta2, nll2 = torch.empty_like(alpha), torch.empty_like(beta), torch.empty_like(nll)
    kn.ctc_fwd(d_log, tg32, il, tl, lse, lpb, alpha2, nll2, beta=beta2)
    grad2 = torch.empty_like(grad)
    kn.ctc_bwd(d_log, tg32, il, tl, lse, lpb, alpha2, nll2, beta2, grad2, 1.0, beta_ready=True)
    assert torch.equal(nll2.isfinite(), nll.isfinite()) and torch.equal(nll2[nll.isfinite()], nll[nll.isfinite()])
    torch.testing.assert_close(grad2, grad, rtol=0, atol=0, equal_nan=True)  # infeasible rows: nan


@pytest.mark.parametrize("B,T,V,L,kind", [(2, 200, 5, 60, "few labels"), (2, 150, 3, 40, "one label"),
                                          (2, 700, 50, 300, "long list")])
def test_ctc_label_repeats_and_long_lists(B, T, V, L, kind):
    """Edge cases of the CTC gradient's per-label gamma (ctc_grad_kernel: first position by an
    LDS atomicMin, then one claim round per repeat, summed in position order) and of the
    register lattice: a 4-label vocabulary (every label repeated ~15 times), one label repeated
    through the whole list (40 rounds), and a 300-label list (positions past the 256-thread
    block, a 13-wave lattice).  Loss and gradient against fp64 autograd through aten's CTC,
    the bar of test_ctc (fp32 logits)."""
    kn = K()
    g = torch.Generator().manual_seed(11 + L)
    logits = torch.randn(B, T, V, generator=g) * 2
    ilen = torch.tensor([T] + [T - 7] * (B - 1))
    tlen = torch.tensor([L] + [L - 3] * (B - 1))
    tg = torch.randint(1, V, (B, L), generator=g)
    if kind == "one label":
        tg.fill_(1)
    for b in range(B):
        tg[b, tlen[b]:] = -1
    lr = logits.double().requires_grad_()
    nll_ref = F.ctc_loss(lr.log_softmax(-1).transpose(0, 1), tg.clamp(min=0), ilen, tlen, blank=0,
                         reduction="none", zero_infinity=False)
    fin = torch.isfinite(nll_ref)
    assert fin.all()
    gref = torch.autograd.grad(nll_ref.sum(), lr)[0]
    l32 = logits.float().requires_grad_()
    n32 = F.ctc_loss(l32.log_softmax(-1).transpose(0, 1), tg.clamp(min=0), ilen, tlen, blank=0,
                     reduction="none", zero_infinity=False)
    g32 = torch.autograd.grad(n32.sum(), l32)[0].double()
    err32 = (g32 - gref).abs().max().item()
    d_log = logits.to(DEV)
    tg32, il, tl = tg.to(DEV, torch.int32), ilen.to(DEV, torch.int32), tlen.to(DEV, torch.int32)
    S = 2 * L + 1
    lse, lpb = torch.empty(B * T, device=DEV), torch.empty(B * T * (L + 1), device=DEV)
    alpha, beta = torch.empty(B * T * S, device=DEV), torch.empty(B * T * S, device=DEV)
    nll = torch.empty(B, device=DEV)
    kn.ctc_fwd(d_log, tg32, il, tl, lse, lpb, alpha, nll)
    got = nll.cpu().double()
    assert ((got - nll_ref.detach()).abs() <= 1e-5 * nll_ref.detach().abs().clamp(min=1)).all(), (got, nll_ref)
    grad = torch.empty(B, T, V, device=DEV, dtype=torch.float32)
    kn.ctc_bwd(d_log, tg32, il, tl, lse, lpb, alpha, nll, beta, grad, 1.0)
    close(grad.cpu().double(), gref, max(2e-3, 1.25 * err32), f"ctc grad ({kind})")


# ----------------------------------------------------------- label-smoothed KL
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lsm_kl(dtype):
    kn = K()
    R, V, s = 77, 4233, 0.1
    logits = (torch.randn(R, V) * 3).to(dtype)
    tg = torch.randint(0, V, (R,))
    tg[::5] = -1
    x = logits.double().requires_grad_()
    td = torch.full((R, V), s / (V - 1), dtype=torch.float64)
    td.scatter_(1, tg.clamp(min=0).unsqueeze(1), 1 - s)
    kl = F.kl_div(x.log_softmax(1), td, reduction="none").masked_fill((tg == -1).unsqueeze(1), 0)
    ref_rows = kl.sum(1)
    gref = torch.autograd.grad(kl.sum() * 0.5, x)[0]
    lse = torch.empty(R, device=DEV)
    rows = torch.empty(R, device=DEV)
    dl = logits.to(DEV)
    t32 = tg.to(DEV, torch.int32)
    kn.lsm_kl_fwd(dl, t32, -1, s, lse, rows)
    close(rows, ref_rows.detach(), 1e-5, "kl rows")
    grad = torch.empty(R, V, device=DEV)
    kn.lsm_kl_bwd(dl, t32, -1, s, lse, grad, 0.5)
    close(grad, gref, 1e-5, "kl grad")
    out = torch.empty(1, device=DEV)
    kn.loss_combine(rows, 0.7, rows[:5].contiguous(), 0.3, out)
    close(out, 0.7 * ref_rows.sum() + 0.3 * ref_rows[:5].sum(), 1e-5, "combine")


def test_losses_padded_rows():
    """CTC / smoothed-KL on [.., V] views of [.., roundup8(V)] buffers (the model's logits
    layout) give bit-identical results to the contiguous layout."""
    kn = K()
    B, T, V, L = 3, 40, 4233, 6
    logits, tg, ilen, tlen = _ctc_case(B, T, V, L, 11, torch.bfloat16)
    d_log = logits.to(DEV)
    pad = kn.padded_rows(B * T, V, torch.bfloat16, DEV).view(B, T, V)
    pad.copy_(d_log)
    tg32, il, tl = tg.to(DEV, torch.int32), ilen.to(DEV, torch.int32), tlen.to(DEV, torch.int32)
    S = 2 * L + 1
    outs = []
    for x in (d_log, pad):
        lse, lpb = torch.empty(B * T, device=DEV), torch.empty(B * T * (L + 1), device=DEV)
        alpha, beta = torch.empty(B * T * S, device=DEV), torch.empty(B * T * S, device=DEV)
        nll = torch.empty(B, device=DEV)
        kn.ctc_fwd(x, tg32, il, tl, lse, lpb, alpha, nll)
        g = kn.padded_rows(B * T, V, torch.bfloat16, DEV).view(B, T, V) if x is pad else torch.empty_like(x)
        kn.ctc_bwd(x, tg32, il, tl, lse, lpb, alpha, nll, beta, g, 1.0)
        rows, lse2 = torch.empty(B * T, device=DEV), torch.empty(B * T, device=DEV)
        t2 = torch.randint(0, V, (B * T,), generator=torch.Generator().manual_seed(3)).to(DEV, torch.int32)
        x2 = x.reshape(B * T, V)
        kn.lsm_kl_fwd(x2, t2, -1, 0.1, lse2, rows)
        g2 = kn.padded_rows(B * T, V, torch.bfloat16, DEV) if x is pad else torch.empty_like(x2)
        kn.lsm_kl_bwd(x2, t2, -1, 0.1, lse2, g2, 0.5)
        outs.append((nll.cpu(), g.float().cpu(), rows.cpu(), g2.float().cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


# ------------------------------------------------------------------ attention
def _rel_shift_ref(x):
    # literal restatement of liteasr/nets/attention.py:99-118 (zero_triu=False)
    zero_pad = torch.zeros((x.size()[:3] + (1,)), dtype=x.dtype)
    xp = torch.cat([zero_pad, x], dim=-1).view(x.size()[:2] + (x.size(3) + 1, x.size(2)))
    return xp[:, :, 1:].view_as(x)


@pytest.mark.parametrize("relpos", [True, False])
def test_attn_softmax(relpos):
    kn = K()
    B, H, T, ldS = 3, 2, 37, 40
    ac = torch.randn(B, H, T, ldS)
    bd = torch.randn(B, H, T, ldS)
    xl = torch.tensor([37, 20, 5])
    mask = (torch.arange(T)[None, :] >= xl[:, None]).to(torch.uint8)  # (B, T) key padding
    s = ac[..., :T].double() + (_rel_shift_ref(bd[..., :T].double()) if relpos else 0)
    s = s.masked_fill(mask.bool()[:, None, None, :], -1e38)
    sr = s.clone().requires_grad_()
    P_ref = torch.softmax(sr, -1)
    P = torch.empty(B, H, T, ldS, device=DEV)
    kn.attn_softmax_fwd(ac.to(DEV), bd.to(DEV) if relpos else None, B, H, T, T, ldS,
                        mask.to(DEV), T, 0, P)
    close(P[..., :T], P_ref.detach(), 1e-5, "softmax fwd")
    assert (P[..., T:] == 0).all()
    dP = torch.randn(B, H, T, ldS)
    dS_ref = torch.autograd.grad(P_ref, sr, dP[..., :T].double())[0]
    dS_ref = dS_ref.masked_fill(mask.bool()[:, None, None, :], 0)
    dS = torch.empty(B, H, T, ldS, device=DEV)
    kn.attn_softmax_bwd(P, dP.to(DEV), B, H, T, T, ldS, mask.to(DEV), T, 0, dS)
    close(dS[..., :T], dS_ref, 1e-5, "softmax bwd")
    if relpos:
        # rel_shift backward == autograd of the literal rel_shift
        bdr = bd[..., :T].double().requires_grad_()
        y = _rel_shift_ref(bdr)
        gref = torch.autograd.grad(y, bdr, dS_ref)[0]
        dBD = torch.empty(B * H, T, ldS, device=DEV)
        kn.relshift_bwd(dS.view(B * H, T, ldS), B * H, T, ldS, dBD)
        close(dBD.view(B, H, T, ldS)[..., :T], gref, 1e-6, "relshift bwd")


@pytest.mark.parametrize("B,H,T,dk,chunk", [(2, 4, 249, 64, 0), (3, 4, 130, 64, 0), (2, 16, 249, 32, 16),
                                             (1, 2, 1, 64, 0), (2, 3, 77, 32, 0)])
def test_relattn_fwd_qb_bit_identical(B, H, T, dk, chunk):
    """lasr_relattn_fwd_qb (the positional biases folded into the attention forward) equals
    lasr_qbias_fwd + lasr_relattn_fwd bit for bit: qu, qv, ctx and the row statistics
    (attention.py:93-96 pos_bias_u / v, :120-154)."""
    kn = K()
    torch.manual_seed(T + dk)
    d = dk * H
    bf = torch.bfloat16
    qkv = (torch.randn(B * T, 3 * d, device=DEV) * 0.5).to(bf)
    pos = (torch.randn(T, d, device=DEV) * 0.5).to(bf)
    bu, bv = torch.randn(d, device=DEV) * 0.1, torch.randn(d, device=DEV) * 0.1
    xl = torch.full((B,), T, device=DEV)
    xl[1::2] = max(T - 17, 1)
    pad = torch.arange(T, device=DEV)[None, :] >= xl[:, None]
    if chunk:
        tri = (torch.arange(T, device=DEV)[None, :] // chunk) > (torch.arange(T, device=DEV)[:, None] // chunk)
        mask, msb, msq = kn.pad_mask16((pad[:, None, :] | tri[None]).to(torch.uint8), B, T, T)
    else:
        mask, msb, msq = pad.to(torch.uint8).contiguous(), T, 0
    outs = []
    for fused in (False, True):
        qu = torch.full((B * T, d), 7.0, dtype=bf, device=DEV)
        qv = torch.full_like(qu, 7.0)
        stats = torch.empty(B * H * T * 2, device=DEV)
        ctx = torch.empty(B * T, d, dtype=bf, device=DEV)
        if fused:
            kn.relattn_fwd_qb(qkv[:, :d], bu, bv, qu, qv, qkv[:, d:2 * d], qkv[:, 2 * d:], pos, B, H, T, mask, msb,
                              msq, dk ** -0.5, stats, ctx)
        else:
            kn.qbias_fwd(qkv, B, T, H, dk, bu, bv, qu, qv)
            kn.relattn_fwd(qu, qv, qkv[:, d:2 * d], qkv[:, 2 * d:], pos, B, H, T, mask, msb, msq, dk ** -0.5, stats,
                           ctx)
        torch.cuda.synchronize()
        outs.append((qu, qv, ctx, stats))
    for name, a, b in zip(("qu", "qv", "ctx", "stats"), outs[0], outs[1]):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("B,H,T,masking,dk", [(2, 2, 37, "pad", 64), (3, 4, 130, "pad", 64), (2, 4, 249, "pad", 64),
                                               (2, 2, 100, "chunk", 64), (2, 1, 64, "none", 64), (1, 1, 1, "none", 64),
                                               (2, 16, 249, "chunk", 32), (3, 3, 70, "pad", 32),
                                               (2, 4, 999, "pad", 64), (2, 16, 500, "chunk", 32),
                                               (3, 4, 200, "chunk", 32), (3, 2, 300, "chunk", 64)])
def test_relattn_fused(B, H, T, masking, dk):
    """attn_flash.hip fwd + bwd vs the literal reference chain (attention.py:120-154) in fp64 on
    the same bf16-rounded operands; one utterance fully masked when masking == "pad" or (B = 3)
    "chunk" (the kernels skip the chunk mask's fully masked blocks only for rows that have an
    unmasked key: a fully masked row keeps its uniform attention)."""
    kn = K()
    torch.manual_seed(T)
    d = dk * H
    scale = dk ** -0.5
    bf = torch.bfloat16
    qkv = (torch.randn(B * T, 3 * d) * 0.5).to(bf)
    qu = (torch.randn(B * T, d) * 0.5).to(bf)
    qv = (torch.randn(B * T, d) * 0.5).to(bf)
    pos = (torch.randn(T, d) * 0.5).to(bf)
    dctx = torch.randn(B * T, d).to(bf)
    if masking == "pad":
        xl = torch.tensor([T, max(T // 3, 1), 0][:B])
        mask = (torch.arange(T)[None, :] >= xl[:, None]).to(torch.uint8).contiguous()  # (B, T)
        msb, msq, m4 = T, 0, mask.bool()[:, None, None, :]
    elif masking == "chunk":
        xl = torch.tensor([T, T - 17, 0][:B])
        pad = torch.arange(T)[None, :] >= xl[:, None]
        tri = (torch.arange(T)[None, :] // 16) > (torch.arange(T)[:, None] // 16)
        mask = (pad[:, None, :] | tri[None]).to(torch.uint8).contiguous()  # (B, T, T)
        msb, msq, m4 = T * T, T, mask.bool()[:, None]
    else:
        mask, msb, msq, m4 = None, 0, 0, None

    def heads(t):
        return t.double().view(B, T, H, dk).permute(0, 2, 1, 3)

    Qu = heads(qu).requires_grad_()
    Qv = heads(qv).requires_grad_()
    Kh = heads(qkv[:, d:2 * d]).requires_grad_()
    Vh = heads(qkv[:, 2 * d:]).requires_grad_()
    Pp = pos.double().view(T, H, dk).permute(1, 0, 2).unsqueeze(0).requires_grad_()
    ac = Qu @ Kh.transpose(-1, -2)
    bd = Qv @ Pp.transpose(-1, -2)
    bd.retain_grad()
    S = (ac + _rel_shift_ref(bd)) * scale
    if m4 is not None:
        S = S.masked_fill(m4, -1e38)
    P = torch.softmax(S, -1)
    ctx_ref = (P @ Vh).permute(0, 2, 1, 3).reshape(B * T, d)
    ctx_ref.backward(dctx.double())

    g = lambda t: t.to(DEV)
    stats = torch.empty(B * H * T * 2, device=DEV)
    ctx = torch.empty(B * T, d, dtype=bf, device=DEV)
    qkv_d, mask_d = g(qkv), (g(mask) if mask is not None else None)
    kn.relattn_fwd(g(qu), g(qv), qkv_d[:, d:2 * d], qkv_d[:, 2 * d:], g(pos), B, H, T, mask_d, msb, msq,
                   scale, stats, ctx)
    close(ctx, ctx_ref.detach(), 2e-2, "relattn ctx")

    ldS = (T + 7) // 8 * 8
    Dbuf = torch.empty(B * H * T, device=DEV)
    dqu = torch.empty(B * T, d, dtype=bf, device=DEV)
    dbd = torch.full((B, H, T, ldS), float("nan"), dtype=bf, device=DEV)
    dqkv = torch.zeros(B * T, 3 * d, dtype=bf, device=DEV)
    kn.relattn_bwd(g(qu), g(qv), qkv_d[:, d:2 * d], qkv_d[:, 2 * d:], g(pos), B, H, T, mask_d, msb, msq,
                   scale, stats, ctx, g(dctx), Dbuf, dqu, dbd, ldS, dqkv[:, d:2 * d], dqkv[:, 2 * d:])
    unh = lambda t: t.permute(0, 2, 1, 3).reshape(B * T, d)
    close(dqu, unh(Qu.grad), 2e-2, "relattn dqu")
    close(dqkv[:, d:2 * d], unh(Kh.grad), 2e-2, "relattn dk")
    close(dqkv[:, 2 * d:], unh(Vh.grad), 2e-2, "relattn dv")
    assert not dbd[..., :T].isnan().any(), "dbd entries left unwritten"
    close(dbd[..., :T].float() * scale, bd.grad, 2e-2, "relattn dbd")
    # head-major dBD ([H][B][T][ldS], the positional-gradient GEMM layout): same values
    dbdh = torch.full((H, B, T, ldS), float("nan"), dtype=bf, device=DEV)
    dqkv2 = torch.zeros_like(dqkv)
    kn.relattn_bwd(g(qu), g(qv), qkv_d[:, d:2 * d], qkv_d[:, 2 * d:], g(pos), B, H, T, mask_d, msb, msq,
                   scale, stats, ctx, g(dctx), Dbuf, torch.empty_like(dqu), dbdh, ldS, dqkv2[:, d:2 * d],
                   dqkv2[:, 2 * d:], dbd_head_major=True)
    assert torch.equal(dbdh.permute(1, 0, 2, 3)[..., :T], dbd[..., :T])


def test_qbias_and_reduce():
    kn = K()
    B, T, H, dk = 2, 9, 4, 8
    D = H * dk
    qkv = torch.randn(B * T, 3 * D, device=DEV)
    bu = torch.randn(D, device=DEV)
    bv = torch.randn(D, device=DEV)
    qu = torch.empty(B * T, D, device=DEV)
    qv = torch.empty(B * T, D, device=DEV)
    kn.qbias_fwd(qkv, B, T, H, dk, bu, bv, qu, qv)
    close(qu, qkv[:, :D] + bu, 1e-6)
    close(qv, qkv[:, :D] + bv, 1e-6)
    dqkv = torch.zeros(B * T, 3 * D, device=DEV)
    du = torch.zeros(D, device=DEV)
    dv = torch.zeros(D, device=DEV)
    kn.qbias_bwd(qu, qv, B, T, H, dk, dqkv, du, dv)
    close(dqkv[:, :D], qu + qv, 1e-6)
    close(du, qu.sum(0), 1e-5)
    close(dv, qv.sum(0), 1e-5)
    src = torch.randn(B, H, T, dk, device=DEV)
    dst = torch.empty(T, D, device=DEV)
    kn.reduce_batch(src, B, H, T, dk, dst)
    close(dst, src.sum(0).permute(1, 0, 2).reshape(T, D), 1e-6)


# ----------------------------------------------------------------------- conv
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_subsampling_convs(dtype):
    kn = K()
    B, T, Fd, Cc = 2, 41, 80, 32
    x = torch.randn(B, T, Fd, device=DEV)
    w1 = torch.randn(Cc, 1, 3, 3, device=DEV) * 0.3
    b1 = torch.randn(Cc, device=DEV) * 0.1
    T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
    y1 = torch.empty(B, T1, F1, Cc, device=DEV, dtype=dtype)
    kn.conv1_fwd(x, w1.view(Cc, 9), b1, y1)
    xr = x.double().requires_grad_()
    w1r = w1.double().requires_grad_()
    b1r = b1.double().requires_grad_()
    y1r = F.relu(F.conv2d(xr.unsqueeze(1), w1r, b1r, stride=2))  # (B,C,T1,F1)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(y1, y1r.permute(0, 2, 3, 1), tol, "conv1")
    # conv2 via im2col + gemm
    w2 = torch.randn(Cc, Cc, 3, 3, device=DEV) * 0.1
    b2 = torch.randn(Cc, device=DEV) * 0.1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    col = torch.empty(B * T2 * F2, 9 * Cc, device=DEV, dtype=dtype)
    kn.im2col(y1, col)
    w2p = torch.empty(Cc, 9 * Cc, device=DEV, dtype=dtype)
    kn.permute_last2(w2.reshape(Cc, Cc, 9), Cc, Cc, 9, w2p)  # [Cout][Cin][9] -> [Cout][9][Cin]
    y2 = torch.empty(B * T2 * F2, Cc, device=DEV, dtype=dtype)
    from liteasr_amd import _native as Nn
    kn.linear(col, w2p, y2, bias=b2, act=Nn.ACT_RELU)
    y2r = F.relu(F.conv2d(y1r, w2.double(), b2.double(), stride=2))
    close(y2.view(B, T2, F2, Cc), y2r.permute(0, 2, 3, 1), 5e-5 if dtype == torch.float32 else 3e-2, "conv2")
    # backward: dcol = dy2 @ w2p ; col2im with relu mask ; conv1 weight grad
    dy2 = torch.randn(B * T2 * F2, Cc, device=DEV).to(dtype)
    dcol = torch.empty(B * T2 * F2, 9 * Cc, device=DEV, dtype=dtype)
    kn.gemm(dy2, w2p, dcol)
    dy1 = torch.empty_like(y1)
    kn.col2im(dcol, y1, dy1)
    y2pre = F.conv2d(y1r, w2.double(), b2.double(), stride=2)
    gy1 = torch.autograd.grad(y2pre, y1r, dy2.double().view(B, T2, F2, Cc).permute(0, 3, 1, 2), retain_graph=True)[0]
    close(dy1, (gy1 * (y1r > 0)).permute(0, 2, 3, 1), 5e-5 if dtype == torch.float32 else 3e-2, "col2im")
    dw1 = torch.zeros(Cc, 9, device=DEV)
    db1 = torch.zeros(Cc, device=DEV)
    kn.conv1_bwd(x, dy1, dw1, db1)
    y1pre = F.conv2d(xr.unsqueeze(1), w1r, b1r, stride=2)
    gw, gb = torch.autograd.grad(y1pre, (w1r, b1r), dy1.double().permute(0, 3, 1, 2))
    close(dw1, gw.view(Cc, 9), 1e-5, "conv1 dw")
    close(db1, gb, 1e-5, "conv1 db")
    # reverse permute with accumulate
    acc = torch.ones(Cc, Cc, 9, device=DEV)
    kn.permute_last2(w2p.float(), Cc, Cc, 9, acc, reverse=True, accumulate=True)
    close(acc, 1 + w2p.float().view(Cc, 9, Cc).permute(0, 2, 1), 1e-6, "permute rev")


@pytest.mark.parametrize("B,T,Fd,Cc,ref64", [(2, 41, 80, 128, True), (2, 42, 81, 128, True), (3, 67, 40, 256, True),
                                             (32, 1000, 80, 256, False)])
def test_conv2_implicit_gemm(B, T, Fd, Cc, ref64):
    """lasr_conv2_gemm (conv2 without im2col / col2im buffers) against the explicit im2col
    path and, at small sizes, fp64 conv2d: forward bit-identical to im2col + GEMM (same k
    order per output), weight / bias gradients within fp32 accumulation error, data gradient
    within one bf16 rounding; odd and even T1/F1 (every output parity class, both edges), and
    the full config-2 size (B 32, T 1000, 80-d)."""
    from liteasr_amd import _native as Nn

    kn = K()
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + T)
    T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    M2 = B * T2 * F2
    bf = torch.bfloat16
    y1 = torch.relu(torch.randn(B, T1, F1, Cc, generator=g)).to(bf).to(DEV)
    w2 = (torch.randn(Cc, Cc, 3, 3, generator=g) / (3 * Cc ** 0.5)).to(DEV)
    b2 = (torch.randn(Cc, generator=g) * 0.1).to(DEV)
    w2p = torch.empty(Cc, 9 * Cc, device=DEV, dtype=bf)
    kn.permute_last2(w2.reshape(Cc, Cc, 9), Cc, Cc, 9, w2p)
    # forward: implicit vs explicit
    y2 = torch.empty(M2, Cc, device=DEV, dtype=bf)
    kn.conv2_fwd(y1, w2p, b2, y2)
    col = torch.empty(M2, 9 * Cc, device=DEV, dtype=bf)
    kn.im2col(y1, col)
    y2e = torch.empty_like(y2)
    small_grid = kn.SMALL_GRID_SPLIT
    kn.SMALL_GRID_SPLIT = False  # the reference GEMM in one K pass (no small-grid split)
    try:
        kn.linear(col, w2p, y2e, bias=b2, act=Nn.ACT_RELU)
    finally:
        kn.SMALL_GRID_SPLIT = small_grid
    assert torch.equal(y2.view(torch.int16), y2e.view(torch.int16)), "conv2 fwd != im2col + GEMM"
    # backward operands: dy2 with its zero tail
    rows = kn.conv2_dy2_rows(M2)
    dy2f = torch.zeros(rows, Cc, device=DEV, dtype=bf)
    dy2f[:M2] = (torch.randn(M2, Cc, generator=g) * (y2.float().cpu() > 0)).to(bf).to(DEV)
    dy2 = dy2f[:M2]
    dw = torch.empty(Cc, 9 * Cc, device=DEV)
    db = torch.full((Cc,), 0.5, device=DEV)
    kn.conv2_dw(dy2f, y1, dw, rowsum=db)
    dy1 = torch.empty_like(y1)
    kn.conv2_dx(dy2f, w2p, y1, dy1)
    torch.cuda.synchronize()
    dwe = torch.empty_like(dw)
    kn.gemm(dy2.t(), col, dwe, split_k=0)
    close(dw, dwe, 1e-5, "conv2 dW vs explicit")
    close(db - 0.5, dy2.float().sum(0), 1e-5, "conv2 db")
    if not ref64:
        dcol = torch.empty_like(col)
        kn.gemm(dy2, w2p, dcol)
        dy1e = torch.empty_like(y1)
        kn.col2im(dcol, y1, dy1e)
        close(dy1, dy1e, 2e-2, "conv2 dX vs explicit")
        return
    y1r = y1.double().permute(0, 3, 1, 2).requires_grad_()
    w2r = w2p.double().view(Cc, 3, 3, Cc).permute(0, 3, 1, 2).contiguous().requires_grad_()
    pre = F.conv2d(y1r, w2r, b2.double(), stride=2)
    close(y2.view(B, T2, F2, Cc), F.relu(pre).permute(0, 2, 3, 1), 1e-2, "conv2 fwd vs fp64")
    gy1, gw = torch.autograd.grad(pre, (y1r, w2r), dy2.double().view(B, T2, F2, Cc).permute(0, 3, 1, 2))
    close(dw.view(Cc, 3, 3, Cc), gw.permute(0, 2, 3, 1), 1e-5, "conv2 dW vs fp64")
    ref = (gy1 * (y1r > 0)).permute(0, 2, 3, 1)
    close(dy1, ref, 8e-3, "conv2 dX vs fp64")
    # every position written (no stale values): masked positions exactly zero
    assert torch.equal(dy1[y1 <= 0].float(), torch.zeros_like(dy1[y1 <= 0].float()))


@pytest.mark.parametrize("B,T,Fd,Cc,ref64", [(2, 42, 81, 256, True), (3, 67, 40, 256, True), (2, 41, 80, 512, True),
                                             (32, 1000, 80, 256, False)])
def test_conv2_dx_w1(B, T, Fd, Cc, ref64):
    """LASR_CONV2_DX_W1: the conv2 data gradient reduced in its epilogue into conv1's weight
    and bias gradients (dy1 never stored) against conv2_dx + conv1_bwd -- the same bf16 dy1
    values, summed in another fp32 order -- and, at small sizes, fp64 autograd of
    conv1(x) . conv2 (within dy1's bf16 rounding); odd and even T1/F1 (every parity class
    and both edges, rows past each class's last tile), C 256 and 512 (two column tiles), and
    the full config-2 size.  Accumulates into dw1 / db1; deterministic."""
    kn = K()
    g = torch.Generator(device="cpu").manual_seed(B * 7 + T + Cc)
    T1, F1 = (T - 3) // 2 + 1, (Fd - 3) // 2 + 1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    M2 = B * T2 * F2
    bf = torch.bfloat16
    x = torch.randn(B, T, Fd, generator=g).to(DEV)
    y1 = torch.relu(torch.randn(B, T1, F1, Cc, generator=g)).to(bf).to(DEV)
    w2 = (torch.randn(Cc, Cc, 3, 3, generator=g) / (3 * Cc ** 0.5)).to(DEV)
    w2p = torch.empty(Cc, 9 * Cc, device=DEV, dtype=bf)
    kn.permute_last2(w2.reshape(Cc, Cc, 9), Cc, Cc, 9, w2p)
    dy2f = torch.zeros(kn.conv2_dy2_rows(M2), Cc, device=DEV, dtype=bf)
    dy2f[:M2] = torch.randn(M2, Cc, generator=g).to(bf).to(DEV)
    assert kn.conv2_dx_w1_ok(Cc)
    dw1 = torch.full((Cc, 9), 0.25, device=DEV)
    db1 = torch.full((Cc,), -0.5, device=DEV)
    kn.conv2_dx_w1(dy2f, w2p, y1, x, dw1, db1)
    dy1 = torch.empty_like(y1)
    kn.conv2_dx(dy2f, w2p, y1, dy1)
    dw1e = torch.zeros(Cc, 9, device=DEV)
    db1e = torch.zeros(Cc, device=DEV)
    kn.conv1_bwd(x, dy1, dw1e, db1e)
    torch.cuda.synchronize()
    assert torch.isfinite(dw1).all() and torch.isfinite(db1).all()
    close(dw1 - 0.25, dw1e, 1e-4, "conv1 dW1 fused vs conv2_dx + conv1_bwd")
    close(db1 + 0.5, db1e, 1e-4, "conv1 db1 fused vs conv2_dx + conv1_bwd")
    # deterministic: a second call adds exactly the same values
    dw2 = torch.zeros(Cc, 9, device=DEV)
    db2 = torch.zeros(Cc, device=DEV)
    kn.conv2_dx_w1(dy2f, w2p, y1, x, dw2, db2)
    dw3 = torch.zeros(Cc, 9, device=DEV)
    db3 = torch.zeros(Cc, device=DEV)
    kn.conv2_dx_w1(dy2f, w2p, y1, x, dw3, db3)
    torch.cuda.synchronize()
    assert torch.equal(dw2, dw3) and torch.equal(db2, db3)
    if not ref64:
        return
    y1r = y1.double().permute(0, 3, 1, 2).requires_grad_()
    w2r = w2p.double().view(Cc, 3, 3, Cc).permute(0, 3, 1, 2).contiguous()
    pre = F.conv2d(y1r, w2r, None, stride=2)
    (gy1,) = torch.autograd.grad(pre, (y1r,), dy2f[:M2].double().view(B, T2, F2, Cc).permute(0, 3, 1, 2))
    dy1r = gy1 * (y1r.detach() > 0)
    w1r = torch.zeros(Cc, 1, 3, 3, dtype=torch.float64, device=DEV, requires_grad=True)
    b1r = torch.zeros(Cc, dtype=torch.float64, device=DEV, requires_grad=True)
    y1pre = F.conv2d(x.double().unsqueeze(1), w1r, b1r, stride=2)
    gw, gb = torch.autograd.grad(y1pre, (w1r, b1r), dy1r)
    close(dw2, gw.view(Cc, 9), 1e-2, "conv1 dW1 fused vs fp64")
    close(db2, gb, 1e-2, "conv1 db1 fused vs fp64")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Cc,T", [(64, 70), (200, 133)])
def test_conformer_conv_module_pieces(dtype, Cc, T):
    kn = K()
    B, Kk = 3, 15
    z1 = torch.randn(B, T, 2 * Cc, device=DEV).to(dtype)
    w = torch.randn(Cc, Kk, device=DEV) * 0.2
    bias = torch.randn(Cc, device=DEV) * 0.1
    y = torch.empty(B, T, Cc, device=DEV, dtype=dtype)
    nparts = kn.dwconv_nparts(B, T)
    stats = torch.empty(nparts * 3 * Cc, device=DEV)
    kn.glu_dwconv_fwd(z1, B, T, Cc, Kk, w, bias, y, stats)
    zr = z1.double().requires_grad_()
    g = F.glu(zr.transpose(1, 2), dim=1)
    wr = w.double().requires_grad_()
    br = bias.double().requires_grad_()
    yr = F.conv1d(g, wr.unsqueeze(1), br, padding=(Kk - 1) // 2, groups=Cc)  # (B,C,T)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(y, yr.transpose(1, 2), tol, "dwconv fwd")
    gamma = torch.randn(Cc, device=DEV)
    beta_ = torch.randn(Cc, device=DEV)
    rm = torch.zeros(Cc, device=DEV)
    rv = torch.ones(Cc, device=DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    mean, rstd, scale, shift = [torch.empty(Cc, device=DEV) for _ in range(4)]
    kn.bn_finalize(stats, nparts, Cc, 1e-5, 0.1, gamma, beta_, rm, rv, nbt, mean, rstd, scale, shift, True)
    bn = torch.nn.BatchNorm1d(Cc).double()
    with torch.no_grad():
        bn.weight.copy_(gamma.double())
        bn.bias.copy_(beta_.double())
    yq = y.double().cpu().transpose(1, 2).requires_grad_()  # BN on the stored y
    u = bn(yq)
    close(rm, bn.running_mean, 1e-5, "running_mean")
    close(rv, bn.running_var, 1e-5, "running_var")
    assert int(nbt.item()) == 1
    h = torch.empty(B * T, Cc, device=DEV, dtype=dtype)
    kn.bn_act_fwd(y.view(B * T, Cc), scale, shift, h)
    hr = u * torch.sigmoid(u)
    close(h, hr.transpose(1, 2).reshape(B * T, Cc), tol, "bn swish fwd")
    dh = torch.randn(B * T, Cc, device=DEV).to(dtype)
    dgm = torch.zeros(Cc, device=DEV)
    dbt = torch.zeros(Cc, device=DEV)
    dyb = torch.empty(B * T, Cc, device=DEV, dtype=torch.float32)
    kn.bn_act_bwd(y.view(B * T, Cc), dh, scale, shift, mean, rstd, gamma, dgm, dbt, dyb)
    gy, gw_, gb_ = torch.autograd.grad(hr, (yq, bn.weight, bn.bias), dh.double().cpu().view(B, T, Cc).transpose(1, 2))
    close(dyb, gy.transpose(1, 2).reshape(B * T, Cc), 1e-4, "bn dy")
    close(dgm, gw_, 1e-4, "bn dgamma")
    close(dbt, gb_, 1e-4, "bn dbeta")
    # dwconv backward from an arbitrary dy
    dy = torch.randn(B, T, Cc, device=DEV)
    dz1 = torch.empty_like(z1)
    dw = torch.zeros(Cc, Kk, device=DEV)
    db = torch.zeros(Cc, device=DEV)
    kn.glu_dwconv_bwd(z1, dy, B, T, Cc, Kk, w, dz1, dw, db)
    gz, gw2, gb2 = torch.autograd.grad(yr, (zr, wr, br), dy.double().transpose(1, 2))
    close(dz1, gz, tol, "dwconv dz1")
    close(dw, gw2, 1e-5 if dtype == torch.float32 else 1e-2, "dwconv dw")
    close(db, gb2, 1e-5, "dwconv db")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Cc,T,offset", [(66, 50, 0), (64, 41, 2)])
def test_glu_dwconv_unvectorised(dtype, Cc, T, offset):
    """The GLU + depthwise kernels' 2-channel path: C not a multiple of 8, or rows not 16-B
    aligned (a view starting 2 elements into its buffer), against fp64."""
    kn = K()
    B, Kk = 2, 15
    z1 = torch.randn(B * T * 2 * Cc + offset, device=DEV).to(dtype)[offset:].view(B, T, 2 * Cc)
    w = torch.randn(Cc, Kk, device=DEV) * 0.2
    bias = torch.randn(Cc, device=DEV) * 0.1
    y = torch.empty(B, T, Cc, device=DEV, dtype=dtype)
    stats = torch.empty(kn.dwconv_nparts(B, T) * 3 * Cc, device=DEV)
    kn.glu_dwconv_fwd(z1, B, T, Cc, Kk, w, bias, y, stats)
    zr = z1.double().requires_grad_()
    wr = w.double().requires_grad_()
    br = bias.double().requires_grad_()
    yr = F.conv1d(F.glu(zr.transpose(1, 2), dim=1), wr.unsqueeze(1), br, padding=(Kk - 1) // 2, groups=Cc)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    close(y, yr.transpose(1, 2), tol, "dwconv fwd")
    dy = torch.randn(B, T, Cc, device=DEV)
    dz1 = torch.empty(B * T * 2 * Cc + offset, device=DEV, dtype=dtype)[offset:].view(B, T, 2 * Cc)
    dw = torch.zeros(Cc, Kk, device=DEV)
    db = torch.zeros(Cc, device=DEV)
    kn.glu_dwconv_bwd(z1, dy, B, T, Cc, Kk, w, dz1, dw, db)
    gz, gw2, gb2 = torch.autograd.grad(yr, (zr, wr, br), dy.double().transpose(1, 2))
    close(dz1, gz, tol, "dwconv dz1")
    close(dw, gw2, 1e-5 if dtype == torch.float32 else 1e-2, "dwconv dw")
    close(db, gb2, 1e-5, "dwconv db")


# ------------------------------------------------------------------ elementwise
def test_embed_pe_and_prep():
    kn = K()
    B, L, D, V = 3, 5, 16, 11
    ids = torch.randint(0, V, (B, L + 1), device=DEV, dtype=torch.int32)
    ids[0, 0] = ids[1, 2] = ids[2, 4] = 3
    E = torch.randn(V, D, device=DEV)
    pe = torch.randn(50, D, device=DEV)
    y = torch.empty(B * (L + 1), D, device=DEV)
    kn.embed_pe_fwd(ids, L + 1, E, pe, 4.0, y)
    ref = E[ids.long()] * 4.0 + pe[: L + 1].unsqueeze(0)
    close(y, ref.view(-1, D), 1e-6, "embed fwd")
    dy = torch.randn(B * (L + 1), D, device=DEV)
    dE = torch.zeros(V, D, device=DEV)
    kn.embed_bwd(ids, dy, 4.0, dE)
    ref = torch.zeros(V, D, device=DEV, dtype=torch.float64).index_add_(0, ids.view(-1).long(), dy.double() * 4)
    close(dE, ref, 1e-6, "embed bwd")
    # decoder-sized: 1312 rows (several ballot chunks), a frequent id (eos padding) and
    # rare ones, against an fp64 index_add
    R, D2, V2 = 1312, 256, 4233
    ids2 = torch.randint(0, V2, (R,), device=DEV, dtype=torch.int32)
    ids2[::3] = V2 - 1
    dy2 = torch.randn(R, D2, device=DEV)
    dE2 = torch.zeros(V2, D2, device=DEV)
    kn.embed_bwd(ids2, dy2, 1.0, dE2)
    ref2 = torch.zeros(V2, D2, device=DEV, dtype=torch.float64).index_add_(0, ids2.long(), dy2.double())
    close(dE2, ref2, 1e-6, "embed bwd R=1312")
    # u2 bookkeeping vs literal python restatement
    xlens = torch.tensor([100, 97, 3], device=DEV)
    ys = torch.tensor([[5, 6, 7, 8], [2, 2, -1, -1], [-1, -1, -1, -1]], device=DEV)
    ylens = torch.tensor([4, 2, 0], device=DEV)
    Tx, Tsub = 100, ((100 - 1) // 2 - 1) // 2
    out = {
        "ys_in": torch.empty(3, 5, dtype=torch.int32, device=DEV),
        "tgt": torch.empty(3, 5, dtype=torch.int32, device=DEV),
        "tgt_ctc": torch.empty(3, 4, dtype=torch.int32, device=DEV),
        "dec_mask": torch.empty(3, 5, 5, dtype=torch.uint8, device=DEV),
        "enc_mask": torch.empty(3, Tsub, dtype=torch.uint8, device=DEV),
        "pred_len": torch.empty(3, dtype=torch.int32, device=DEV),
        "ylen": torch.empty(3, dtype=torch.int32, device=DEV),
    }
    kn.u2_prep(xlens, ys, ylens, Tx, Tsub, 9, 9, 0, out)
    assert out["ys_in"].tolist() == [[9, 5, 6, 7, 8], [9, 2, 2, 9, 9], [9, 9, 9, 9, 9]]
    assert out["tgt"].tolist() == [[5, 6, 7, 8, 9], [2, 2, 9, -1, -1], [9, -1, -1, -1, -1]]
    assert out["pred_len"].tolist() == [((x - 1) // 2 - 1) // 2 for x in [100, 97, 3]]
    pm = torch.arange(Tx)[None, :] >= xlens.cpu()[:, None]
    assert torch.equal(out["enc_mask"].cpu().bool(), pm[:, :-2:2][:, :-2:2])
    tri = torch.arange(5)[None, :] > torch.arange(5)[:, None]
    ysm = torch.arange(5)[None, :] >= (ylens.cpu() + 1)[:, None]
    assert torch.equal(out["dec_mask"].cpu().bool(), ysm[:, None, :] | tri[None])
    # padded rows (lasr_u2_prep_ld, what the model's _prep uses): the same masks in the first
    # L+1 / T' columns, 1 (masked) in the padding; chunk mode's [B, T', T'] mask likewise
    pad = dict(out, dec_mask=torch.zeros(3, 5, 16, dtype=torch.uint8, device=DEV))
    kn.u2_prep(xlens, ys, ylens, Tx, Tsub, 9, 9, 0, pad)
    assert torch.equal(pad["dec_mask"][:, :, :5], out["dec_mask"]) and bool((pad["dec_mask"][:, :, 5:] == 1).all())
    ck = 4
    P = (Tsub + 15) // 16 * 16
    chk = dict(out, chunk_mask=torch.zeros(3, Tsub, P, dtype=torch.uint8, device=DEV),
               enc_mask=torch.empty_like(out["enc_mask"]))
    kn.u2_prep(xlens, ys, ylens, Tx, Tsub, 9, 9, ck, chk)
    t = torch.arange(Tsub)
    cm = pm[:, :-2:2][:, :-2:2][:, None, :] | ((t[None, :] // ck) > (t[:, None] // ck))[None]
    assert torch.equal(chk["chunk_mask"][:, :, :Tsub].cpu().bool(), cm)
    assert bool((chk["chunk_mask"][:, :, Tsub:] == 1).all())
    assert torch.equal(chk["enc_mask"], out["enc_mask"])  # the key mask in the same launch


def _prep_case(B, Tx, L, seed):
    g = torch.Generator().manual_seed(seed)
    xlens = torch.randint(1, Tx + 1, (B,), generator=g)
    xlens[0] = Tx
    ylens = torch.randint(0, L + 1, (B,), generator=g)
    ys = torch.randint(1, 50, (B, L), generator=g)
    ys[torch.arange(L)[None, :] >= ylens[:, None]] = -1
    Tsub = ((Tx - 1) // 2 - 1) // 2
    P = (Tsub + 15) // 16 * 16
    out = {
        "ys_in": torch.empty(B, L + 1, dtype=torch.int32, device=DEV),
        "tgt": torch.empty(B, L + 1, dtype=torch.int32, device=DEV),
        "tgt_ctc": torch.empty(B, L, dtype=torch.int32, device=DEV),
        "dec_mask": torch.empty(B, L + 1, (L + 16) // 16 * 16, dtype=torch.uint8, device=DEV),
        "enc_mask": torch.empty(B, Tsub, dtype=torch.uint8, device=DEV),
        "chunk_mask": torch.empty(B, Tsub, P, dtype=torch.uint8, device=DEV),
        "pred_len": torch.empty(B, dtype=torch.int32, device=DEV),
        "ylen": torch.empty(B, dtype=torch.int32, device=DEV),
    }
    return xlens, ys, ylens, Tsub, out


def _chunk_ref(xlens, Tx, Tsub, c):
    """liteasr/utils/mask.py: padding_mask(xlens)[:, :-2:2][:, :-2:2] | triangle_mask(T', stage=c)."""
    pm = (torch.arange(Tx)[None, :] >= xlens[:, None])[:, :-2:2][:, :-2:2]
    t = torch.arange(Tsub)
    return pm[:, None, :] | ((t[None, :] // c) > (t[:, None] // c))[None]


@pytest.mark.parametrize("Tx,c", [(1000, 1), (1000, 16), (1000, 25), (1000, 249), (1000, 0), (4000, 7), (61, 3)])
def test_u2_prep_device_chunk(Tx, c):
    """Device-scalar chunk mode (lasr_u2_prep_chunk mode 2, what a captured dynamic-chunk step
    replays): the mask equals padding | triangle_mask(T', stage=c) bit for bit, c <= 0 or
    c >= T' is full context, and the padding columns are masked; every other output equals
    the chunk-free call's."""
    kn = K()
    xlens, ys, ylens, Tsub, out = _prep_case(5, Tx, 12, seed=Tx + c)
    ref_out = {k: torch.empty_like(v) for k, v in out.items()}
    kn.u2_prep(xlens.to(DEV), ys.to(DEV), ylens.to(DEV), Tx, Tsub, 9, 9, 0, ref_out)
    cd = torch.tensor([c], dtype=torch.int32, device=DEV)
    kn.u2_prep(xlens.to(DEV), ys.to(DEV), ylens.to(DEV), Tx, Tsub, 9, 9, 0, out, chunk_mode=kn.CHUNK_DEVICE,
               chunk_dev=cd)
    ce = c if 0 < c < Tsub else Tsub
    assert torch.equal(out["chunk_mask"][:, :, :Tsub].cpu().bool(), _chunk_ref(xlens, Tx, Tsub, ce))
    assert bool((out["chunk_mask"][:, :, Tsub:] == 1).all())
    for k in ("ys_in", "tgt", "tgt_ctc", "dec_mask", "enc_mask", "pred_len", "ylen"):
        assert torch.equal(out[k], ref_out[k]), k


def test_u2_prep_sampled_chunk_matches_host_draw():
    """Sampled mode (lasr_u2_prep_chunk mode 3, the dynamic-chunk training step): the device
    draws c from (seed, step counter), writes it to the device scalar, and builds the mask with
    it; the host mirror (FusedEncoderModel.dynamic_chunk_size) gives the same c for every
    counter value, and the draws follow WeNet's distribution (about half full context, the
    rest spread over 1..25)."""
    from liteasr_amd.models._fused import FusedEncoderModel as F

    kn = K()
    Tx = 1000
    xlens, ys, ylens, Tsub, out = _prep_case(3, Tx, 8, seed=3)
    xd, yd, ld = xlens.to(DEV), ys.to(DEV), ylens.to(DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    cd = torch.zeros(1, dtype=torch.int32, device=DEV)
    seen = []
    for step in list(range(40)) + [2**32 + 5, 2**40 + 77]:
        ctr.fill_(step)
        kn.u2_prep(xd, yd, ld, Tx, Tsub, 9, 9, 0, out, chunk_mode=kn.CHUNK_SAMPLE, chunk_dev=cd, ctr=ctr,
                   chunk_seed=88, chunk_max=25)
        c = int(cd.item())
        assert c == F.dynamic_chunk_size(88, step, Tsub, 25), step
        assert torch.equal(out["chunk_mask"][:, :, :Tsub].cpu().bool(), _chunk_ref(xlens, Tx, Tsub, c)), step
        seen.append(c)
    host = [F.dynamic_chunk_size(88, s, Tsub, 25) for s in range(4000)]
    full = sum(c == Tsub for c in host) / len(host)
    assert 0.45 < full < 0.55 and set(c for c in host if c != Tsub) == set(range(1, 26)), full
    assert len(set(seen)) > 5


def test_adam_noam_clip():
    kn = K()
    n = 50000
    torch.manual_seed(0)
    p0 = torch.randn(n)
    g = torch.randn(n) * 3
    ref_p = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref_p], lr=1.0, betas=(0.9, 0.98), eps=1e-9)
    p = p0.to(DEV)
    plp = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    state = torch.zeros(5, device=DEV)
    nparts = kn.sumsq_nparts(n)
    ws = torch.empty(nparts, device=DEV)
    for step in range(1, 4):
        gs = g * step
        ref_p.grad = gs.clone()
        norm = torch.nn.utils.clip_grad_norm_([ref_p], 5.0)
        lr = 1.0 * 256 ** -0.5 * min(step ** -0.5, step * 25000 ** -1.5)
        for grp in opt.param_groups:
            grp["lr"] = lr
        opt.step()
        gd = gs.to(DEV)
        kn.sumsq_partial(gd, ws)
        kn.adam_step(p, plp, gd, m, v, ws, nparts, state, 5.0, 1, 0.0, 1.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)
        st = state.cpu()
        assert st[0].item() == step
        assert abs(st[2].item() - norm.item()) <= 1e-4 * norm.item()
        assert abs(st[1].item() - lr) <= 1e-6 * lr
    close(p, ref_p.detach(), 1e-5, "adam params")
    close(plp, ref_p.detach(), 1e-2, "adam bf16 copy")
    # NaN norm skips the step and leaves everything untouched
    p_before = p.clone()
    gnan = g.clone()
    gnan[7] = float("nan")
    kn.sumsq_partial(gnan.to(DEV), ws)
    kn.adam_step(p, None, gnan.to(DEV), m, v, ws, nparts, state, 5.0, 1, 0.0, 1.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)
    assert state[3].item() == 1.0 and state[0].item() == 3
    assert torch.equal(p, p_before)


@pytest.mark.parametrize("max_norm", [0.0, 1.0, float("inf")])
def test_clip_coef_matches_torch(max_norm):
    """clip coefficient = min(max_norm / (norm + 1e-6), 1) for any max_norm, exactly as
    torch.nn.utils.clip_grad_norm_ (the reference's default clip_grad_norm is 0.0,
    liteasr/config/__init__.py:78, which zeroes the gradient); +inf is 'no clipping'."""
    kn = K()
    n = 4096
    g = torch.randn(n, generator=torch.Generator().manual_seed(3))
    ref = torch.zeros(n, requires_grad=True)
    ref.grad = g.clone()
    torch.nn.utils.clip_grad_norm_([ref], max_norm)
    coef_ref = (ref.grad.double().norm() / g.double().norm()).item()
    p = torch.zeros(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    state = torch.zeros(5, device=DEV)
    nparts = kn.sumsq_nparts(n)
    ws = torch.empty(nparts, device=DEV)
    gd = g.to(DEV)
    kn.sumsq_partial(gd, ws)
    kn.adam_step(p, None, gd, m, v, ws, nparts, state, max_norm, 0, 1e-3, 1.0, 1.0, 1.0, 0.9, 0.999, 1e-8, 0.0)
    coef = state[4].item()
    assert abs(coef - coef_ref) <= 1e-6, (coef, coef_ref)
    assert state[3].item() == 0.0 and state[0].item() == 1.0
    # Adam's first moment is (1 - beta1) * coef * g
    close(m, 0.1 * coef_ref * g.to(DEV), 1e-6, "m after clipped step")


@pytest.mark.parametrize("name", ["t249", "t999"])
def test_ctc_against_reference_golden_full_size(name):
    """SURVEY §8(c) F-c: the fused log-softmax + CTC alpha/beta kernels at (T' 249, B 4,
    V 4233, L 40) and (T' 999, B 2, V 4233, L 150) against the reference's HybridCTCLoss
    (ctc_weight 1) outputs in tests/golden/ctc_large.npz (logits regenerated from their
    seed).  Per-utterance loss within 1e-5 relative.  Gradient (blank + label + 16 random
    columns, every frame), measured against the float64 restatement: ours within
    max(2e-3, 1.5 x the reference's own fp32 error on the same logits) -- the golden is
    aten's fp32 CTC, 1.4e-3 / 8.1e-3 of max off float64 here (the lattice accumulates
    hundreds of fp32 log-prob additions) -- and ours vs the golden within the sum of both."""
    import os
    import sys

    import numpy as np

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    sys.path.insert(0, root)
    from inputs import ctc_large_inputs

    from oracle import ctc_ref

    kn = K()
    d = np.load(os.path.join(root, "tests", "golden", "ctc_large.npz"))
    Tp, B, V, L, seed = d[f"{name}_dims"].tolist()
    xlens, ys, ylens, h = ctc_large_inputs(Tp, B, V, L, seed)
    assert torch.equal(h.reshape(-1)[:64], torch.from_numpy(d[f"{name}_logit_head"]))
    ilen = ((xlens - 1) // 2 - 1) // 2
    cols = torch.from_numpy(d[f"{name}_cols"])
    S = 2 * L + 1
    dl = h.to(DEV)
    tg32, il, tl = ys.to(DEV, torch.int32), ilen.to(DEV, torch.int32), ylens.to(DEV, torch.int32)
    lse = torch.empty(B * Tp, device=DEV)
    lpb = torch.empty(B * Tp * (L + 1), device=DEV)
    alpha = torch.empty(B * Tp * S, device=DEV)
    beta = torch.empty(B * Tp * S, device=DEV)
    nll = torch.empty(B, device=DEV)
    kn.ctc_fwd(dl, tg32, il, tl, lse, lpb, alpha, nll, beta=beta)
    grad = torch.empty(B, Tp, V, device=DEV)
    kn.ctc_bwd(dl, tg32, il, tl, lse, lpb, alpha, nll, beta, grad, 1.0 / B, beta_ready=True)
    got = nll.cpu().double().numpy()
    ref = d[f"{name}_loss_per_utt"]
    assert np.allclose(got, ref, rtol=1e-5, atol=0), (got, ref)
    gg = grad.cpu().double()[:, :, cols]
    g64 = torch.zeros_like(gg)
    for b in range(B):
        lp = torch.log_softmax(h[b, : ilen[b]].double(), -1).numpy()
        _, g = ctc_ref.ctc_nll_and_grad(lp, ys[b, : ylens[b]].numpy())
        g64[b, : ilen[b]] = torch.from_numpy(g)[:, cols] / B
    gold = torch.from_numpy(d[f"{name}_grad_cols"]).double()
    m = g64.abs().max().item()
    err_ref = (gold - g64).abs().max().item() / m  # the reference's own fp32 error
    err_ours = (gg - g64).abs().max().item() / m
    assert err_ours <= max(2e-3, 1.5 * err_ref), (err_ours, err_ref)
    close(gg, gold, err_ref + err_ours + 1e-6, "ctc grad vs reference golden")


def test_reduce_multi_many_segments_bit_identical():
    """lasr_reduce_multi over 150 segments (three 64-segment launches, the many-partial
    segments' blocks first in each) gives the bits of one launch per segment: both summation
    modes (P <= 64 slabs, P > 64 LayerNorm-style partial rows), split outputs, accumulate and
    overwrite, unaligned column counts; against float64 at the fp32 bar."""
    from liteasr_amd import _native as N

    kn = K()
    g = torch.Generator().manual_seed(150)
    segs = []
    for i in range(150):
        P = [2, 3, 4, 8, 64, 65, 498, 31][i % 8]
        Nc = [4096, 512, 516, 130, 2048 * 3][i % 5]
        split = Nc // 2 if i % 3 == 0 else None
        if split is not None and i % 2:
            split -= split % 4
        part = torch.randn(P, Nc, generator=g).to(DEV)
        o0 = torch.randn(split if split else Nc, generator=g).to(DEV)
        o1 = torch.randn(Nc - split, generator=g).to(DEV) if split else None
        segs.append((part, P, Nc, o0, o1, split, i % 4 != 1))
    refs = []
    for part, P, Nc, o0, o1, split, acc in segs:
        s = part.double().sum(0)
        full = (torch.cat([o0, o1]) if o1 is not None else o0).double()
        refs.append(s + full if acc else s)

    def run(batched):
        outs = [(o0.clone(), o1.clone() if o1 is not None else None) for _, _, _, o0, o1, _, _ in segs]
        rows = [N.ReduceSeg(kn.ptr(p), Nc, P, int(acc), kn.ptr(a), kn.ptr(b), sp if sp else Nc)
                for (p, P, Nc, _, _, sp, acc), (a, b) in zip(segs, outs)]
        if batched:
            arr = (N.ReduceSeg * len(rows))(*rows)
            N.call("lasr_reduce_multi", arr, len(rows), kn.stream())
        else:
            for r in rows:
                arr = (N.ReduceSeg * 1)(r)
                N.call("lasr_reduce_multi", arr, 1, kn.stream())
        torch.cuda.synchronize()
        return [torch.cat([a, b]) if b is not None else a for a, b in outs]

    one, many = run(False), run(True)
    for i, (a, b, r) in enumerate(zip(one, many, refs)):
        assert torch.equal(a, b), i
        close(b, r, 1e-5, f"segment {i}")
