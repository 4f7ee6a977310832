"""Round-6 launch fusions, each pinned bit for bit against the path it replaces: one bf16
training step (dropout 0.1, so the fused dropout-backward draws are exercised) with the fusion
on and off must give torch.equal losses, flat gradients and BN buffers.  The switches are
module attributes (not environment variables): the product path is the fused one."""

import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import u2_oracle as O  # noqa: E402

CFG = O.default_cfg(enc_layers=2, dec_layers=3)  # small-model widths (d 256, ff 2048, V 4233)


def _step(cfg, B=3, T=300, L=9, dropout=0.1, seed=4):
    from liteasr_amd.criterions.hybrid_ctc_attn import HybridCTCLoss, HybridCTCLossConfig
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    c = U2Config(input_dim=cfg["input_dim"], vocab_size=cfg["vocab_size"], enc_dim=cfg["enc_dim"],
                 enc_ff_dim=cfg["enc_ff"], enc_attn_heads=cfg["enc_heads"], enc_layers=cfg["enc_layers"],
                 dec_dim=cfg["dec_dim"], dec_ff_dim=cfg["dec_ff"], dec_attn_heads=cfg["dec_heads"],
                 dec_layers=cfg["dec_layers"], dropout_rate=dropout, compute_dtype="bf16")
    resolve_self(c)
    c.enc_attn_dropout_rate = c.dec_self_attn_dropout_rate = c.dec_src_attn_dropout_rate = 0.0
    m = U2(c)
    m.load_state_dict({**O.init_params(cfg, seed=seed), **O.init_buffers(cfg)}, strict=False)
    m = m.cuda().train()
    crit = HybridCTCLoss(HybridCTCLossConfig(vocab_size=cfg["vocab_size"], smoothing=0.1, ctc_weight=0.3))
    xs, xl, ys, yl = [t.cuda() for t in O.synthetic_batch(B, T, L, cfg["vocab_size"], seed=seed)]
    loss = crit(m, xs, xl, ys, yl)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), m.store.grad.clone(), [b.clone() for b in m.bn_flat_buffers()]


def _same(a, b):
    assert a[0] == b[0], (a[0], b[0])
    assert torch.equal(a[1], b[1]), (a[1] - b[1]).abs().max().item()
    for x, y in zip(a[2], b[2]):
        assert torch.equal(x, y)


def test_decoder_branch_grad_in_layernorm_bwd(monkeypatch):
    """The decoder FFN branch gradient (its residual dropout's backward) written by the
    LayerNorm backward that produces the layer output gradient, vs a branch_grad launch."""
    from liteasr_amd.nets import functional as FN

    on = _step(CFG)
    monkeypatch.setattr(FN, "DEC_GB_IN_LN", False)
    off = _step(CFG)
    _same(on, off)


@pytest.mark.parametrize("B,L,d", [(3, 9, 256), (8, 40, 256), (4, 20, 512)])
def test_splitk_reduce_with_layernorm(monkeypatch, B, L, d):
    """The decoder's FFN fc2 split-K reduction with the next LayerNorm (lasr_gemm_ln_fwd) and the
    fc1 input-gradient reduction with the LayerNorm backward in front of the FFN
    (lasr_gemm_ln_bwd), vs the separate reduction and norm launches; d 512 = config 4's width."""
    from liteasr_amd.nets import functional as FN

    cfg = CFG if d == 256 else O.default_cfg(enc_dim=512, enc_heads=8, enc_layers=1, dec_dim=512, dec_heads=8,
                                             dec_layers=2)
    on = _step(cfg, B=B, L=L)
    monkeypatch.setattr(FN, "SPLITK_LN", False)
    off = _step(cfg, B=B, L=L)
    _same(on, off)


@pytest.mark.parametrize("enc_heads,d", [(4, 256), (16, 512)])
def test_qbias_bwd_in_positional_gemm_reduction(monkeypatch, enc_heads, d):
    """The encoder attention's positional-bias gradient blocks in the positional-projection
    gradient GEMM's split-K reduction launch (lasr_gemm_qbias_bwd), vs two launches."""
    from liteasr_amd.nets import functional as FN

    cfg = O.default_cfg(enc_dim=d, enc_heads=enc_heads, enc_layers=2, dec_dim=d, dec_heads=enc_heads, dec_layers=1)
    on = _step(cfg, B=4, T=1000, L=12)
    monkeypatch.setattr(FN, "QBIAS_IN_REDUCE", False)
    off = _step(cfg, B=4, T=1000, L=12)
    _same(on, off)


@pytest.mark.parametrize("d,heads", [(256, 4), (512, 16)])
def test_dw_group_longest_slice_first(monkeypatch, d, heads):
    """The grouped weight-gradient blocks laid out longest K slice first
    (lasr_gemm_dw_group_order) vs call order: only the block order changes, so the step is
    bit-identical; d 512 = config 4's widths, where the encoder group mixes split-2 FFN blocks
    with split-4 / split-8 projection blocks."""
    from liteasr_amd import kernels as K

    cfg = O.default_cfg(enc_dim=d, enc_heads=heads, enc_layers=2, dec_dim=d, dec_heads=heads, dec_layers=1)
    on = _step(cfg, B=8, T=1000, L=12)
    monkeypatch.setattr(K, "DW_GROUP_LPT", False)
    off = _step(cfg, B=8, T=1000, L=12)
    monkeypatch.setattr(K, "DW_GROUP_LPT", True)
    K._flush_gemm_group()  # (restores the library's setting for the tests after this one)
    _same(on, off)


@pytest.mark.parametrize("d,heads", [(256, 4), (512, 16)])
def test_narrow_output_tiles(monkeypatch, d, heads):
    """The planner's 64 x 64 tiles for outputs at most 64 wide (the per-head d_k GEMMs:
    lasr_gemm_narrow_tiles) vs the wider tiles it used to pick: one step bit-identical."""
    from liteasr_amd import kernels as K

    cfg = O.default_cfg(enc_dim=d, enc_heads=heads, enc_layers=2, dec_dim=d, dec_heads=heads, dec_layers=1)
    on = _step(cfg, B=8, T=1000, L=12)
    monkeypatch.setattr(K, "GEMM_NARROW_TILES", False)
    off = _step(cfg, B=8, T=1000, L=12)
    _same(on, off)


@pytest.mark.parametrize("d,heads", [(256, 4), (512, 16)])
def test_bn_backward_in_dwconv_window(monkeypatch, d, heads):
    """The conv module's BatchNorm + Swish backward computed inside the depthwise-conv / GLU
    backward's window load (lasr_bn_act_glu_dwconv_bwd) vs bn_act_bwd storing an fp32 dy that
    glu_dwconv_bwd reads: one bf16 step bit-identical, BN running statistics included."""
    from liteasr_amd.nets import functional as FN

    cfg = O.default_cfg(enc_dim=d, enc_heads=heads, enc_layers=2, dec_dim=d, dec_heads=heads, dec_layers=1)
    on = _step(cfg, B=4, T=1000, L=12)
    monkeypatch.setattr(FN, "BN_GLU_FUSED", False)
    off = _step(cfg, B=4, T=1000, L=12)
    _same(on, off)


@pytest.mark.parametrize("d,heads", [(256, 4), (512, 16)])
def test_layer_boundary_norm_backwards_chained(monkeypatch, d, heads):
    """A Conformer layer's first-norm backward and the previous layer's final-norm backward in
    one launch (lasr_layernorm2_bwd: the previous layer receives dx4 and its branch gradient)
    vs two lasr_layernorm_bwd launches with the fp32 gradient between them: one bf16 step of
    three encoder layers bit-identical."""
    from liteasr_amd.nets import functional as FN

    cfg = O.default_cfg(enc_dim=d, enc_heads=heads, enc_layers=3, dec_dim=d, dec_heads=heads, dec_layers=1)
    on = _step(cfg, B=4, T=1000, L=12)
    monkeypatch.setattr(FN, "LN2_BWD_CHAIN", False)
    off = _step(cfg, B=4, T=1000, L=12)
    _same(on, off)


@pytest.mark.parametrize("d,heads", [(256, 4), (512, 16)])
def test_layer_reductions_held_across_layers(monkeypatch, d, heads):
    """The encoder layers' parameter-gradient reductions queued across the layer nodes and
    launched together at layer 0 (kernels.deferred_reductions(hold=True)) vs one reduction
    launch per layer node: one bf16 step of four encoder layers bit-identical, nothing left
    queued after the backward."""
    from liteasr_amd import kernels as kn
    from liteasr_amd.nets import functional as FN

    cfg = O.default_cfg(enc_dim=d, enc_heads=heads, enc_layers=4, dec_dim=d, dec_heads=heads, dec_layers=1)
    on = _step(cfg, B=4, T=1000, L=12)
    assert kn.held_reductions() == 0
    monkeypatch.setattr(FN, "LAYER_RED_HOLD", False)
    off = _step(cfg, B=4, T=1000, L=12)
    _same(on, off)
