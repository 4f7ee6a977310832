"""Paraformer (liteasr/models/paraformer.py) on the fused HIP encoder.

Same config schema, registry name ("Paraformer"), state_dict keys and call conventions as
the reference: ``model(xs, xlens, ys, ylens) -> (hs_attn (B, L, V), sum_alpha (B,))``,
with ``ParaformerLoss`` (criterions/paraformer_loss.py) on top.  The encoder is U2's fused
Conformer stack (models/_fused.py); everything after it is one fused autograd node
(nets/functional.py ParaformerHeadsFn): CIF predictor with the integrate-and-fire scan in
csrc/cif.hip, the parallel decoder on the decoder-layer kernels, the glancing sampler.

The glancing sampler draws with Python's ``random`` module exactly like the reference
(``random.sample`` per utterance, glancing_sampler.py:27), so seeding ``random`` reproduces
its replace maps; it needs the first pass's argmax on the host (one device->host copy per
step, as in the reference).  Extensions (default off): ``compute_dtype`` ("bf16" default,
"fp32" parity build).
"""

from __future__ import annotations

import random
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor

from ..config import II, MISSING, LiteasrDataclass
from ..nets import functional as FN
from ..nets.modules import ParallelDecoder, PositionalEncoding, Predictor, TransformerEncoder
from . import register_model
from ._fused import FusedEncoderModel


@dataclass
class ParaformerConfig(LiteasrDataclass):
    name: Optional[str] = field(default="Paraformer")
    dropout_rate: float = field(default=0.0)
    use_rel: bool = field(default=True)
    input_dim: int = field(default=MISSING)
    enc_dim: int = field(default=256)
    enc_ff_dim: int = field(default=2048)
    enc_attn_heads: int = field(default=4)
    enc_dropout_rate: float = II("model.dropout_rate")
    enc_pos_dropout_rate: float = II("model.enc_dropout_rate")
    enc_attn_dropout_rate: float = II("model.enc_dropout_rate")
    enc_ff_dropout_rate: float = II("model.enc_dropout_rate")
    enc_layers: int = field(default=12)
    activation: str = field(default="swish")
    sample_ratio: float = field(default=0.75)
    vocab_size: int = field(default=MISSING)
    dec_dim: int = field(default=256)
    dec_ff_dim: int = field(default=2048)
    dec_attn_heads: int = field(default=4)
    dec_dropout_rate: float = II("model.dropout_rate")
    dec_self_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_src_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_ff_dropout_rate: float = II("model.dec_dropout_rate")
    dec_layers: int = field(default=6)
    pos_dropout_rate: float = II("model.dec_dropout_rate")
    # liteasr_amd extension
    compute_dtype: str = field(default="bf16")


@register_model("Paraformer", dataclass=ParaformerConfig)
class Paraformer(FusedEncoderModel):
    def __init__(self, cfg: ParaformerConfig, task=None):
        super().__init__()
        g = lambda k, d=None: getattr(cfg, k, d)  # noqa: E731
        V = g("vocab_size")
        self.encoder = TransformerEncoder(
            use_rel=g("use_rel", True), i_dim=g("input_dim"), h_dim=g("enc_dim"), ff_dim=g("enc_ff_dim"),
            n_head=g("enc_attn_heads"), n_layer=g("enc_layers"), dropout_rate=float(g("enc_dropout_rate")),
            pos_dropout_rate=float(g("enc_pos_dropout_rate")), attn_dropout_rate=float(g("enc_attn_dropout_rate")),
            ff_dropout_rate=float(g("enc_ff_dropout_rate")), activation=g("activation", "swish"), arch="conformer")
        # the reference wires the source-attention dropout to dec_ff_dropout_rate (paraformer.py:88)
        self.decoder = ParallelDecoder(
            i_dim=V, h_dim=g("dec_dim"), ff_dim=g("dec_ff_dim"), n_head=g("dec_attn_heads"), n_layer=g("dec_layers"),
            dropout_rate=float(g("dec_dropout_rate")), self_attn_dropout_rate=float(g("dec_self_attn_dropout_rate")),
            src_attn_dropout_rate=float(g("dec_ff_dropout_rate")), ff_dropout_rate=float(g("dec_ff_dropout_rate")))
        self.embed = nn.Embedding(V, g("dec_dim"))
        self.pe = PositionalEncoding(g("dec_dim"), float(g("pos_dropout_rate")))
        self.predictor = Predictor(g("enc_dim"))
        self.sample_ratio = float(g("sample_ratio", 0.75))
        self.pos_dropout_rate = float(g("pos_dropout_rate"))
        self.ignore = -1
        self.blank = 0
        self.eos = V - 1
        self.sos = V - 1
        self.vocab_size = V
        cd = str(g("compute_dtype", "bf16")).lower()
        self.compute_dtype = torch.float32 if cd in ("fp32", "float32", "float") else torch.bfloat16
        self.chunk_size = 0
        self.rng = random  # the glancing sampler's generator (module-level random, as the reference)
        self.last_glance = None
        self._finalize()

    def _head_units(self):
        """ParaformerHeadsFn.backward order: decoder, target embedding, predictor."""
        return ["decoder", "embed", "predictor"]

    def embed_weight(self):
        return self.store.view("embed.weight")

    def embed_grad(self):
        return self.store.grad_view("embed.weight")

    def forward(self, xs, xlens, ys, ylens):
        """paraformer.py:97-113."""
        x, prep, env = self._run_encoder(xs, xlens, ys, ylens)
        env.pred_len, env.ylen = prep.pred_len, prep.ylen
        ylens_host = ylens.detach().cpu().long()
        ys_d = ys.to(device=xs.device, dtype=torch.int64)
        hs_attn, sum_alpha = FN.ParaformerHeadsFn.apply(x, self.predictor.conv.weight, self, env, ys_d,
                                                        ylens_host, self.rng)
        self.last_count = int(ylens_host.sum())
        return hs_attn.view(prep.B, ys.shape[1], -1), sum_alpha

    def get_pred_len(self, xlens) -> Tensor:
        """paraformer.py:122-124."""
        return super().get_pred_len(xlens)

    def get_target(self, ys, ylens) -> Tensor:
        return ys

    def get_target_len(self, ylens) -> Tensor:
        return ylens

    @classmethod
    def build_model(cls, cfg: ParaformerConfig, task=None):
        cfg.input_dim = task.feat_dim
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)
