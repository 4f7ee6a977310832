"""U2: Conformer encoder + Transformer decoder + CTC (liteasr/models/u2.py), HIP path.

Same config schema, registry name, state_dict and call conventions as the reference:
``model(xs, xlens, ys, ylens) -> (h_attn (B, L+1, V), h_ctc (B, T', V))``.  The compute
runs in the fused HIP nodes of liteasr_amd.nets.functional; bookkeeping (masks,
decoder inputs, targets, CTC lengths) is one device kernel (lasr_u2_prep).

Extensions (default off = reference behaviour):
  compute_dtype  "bf16" (default; fp32 masters/accumulation) or "fp32" (parity build)
  chunk_size     > 0 adds triangle_mask(T', stage=chunk_size) to the encoder
                 self-attention mask (the dynamic-chunk config's oracle-by-composition)
  dynamic_chunk  True: in training, a chunk size is drawn per step on the device (WeNet's
                 distribution: full context with probability ~1/2, else c in 1..max_chunk)
                 and the mask is padding | triangle_mask(T', stage=c) -- BASELINE config 4
  max_chunk      upper end of the dynamic draw (25)
"""

from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Optional, Tuple

import torch
from torch import Tensor

from ..config import II, MISSING, LiteasrDataclass
from ..nets import functional as FN
from .. import decoding as D
from ..nets.modules import CTC, TransformerDecoder, TransformerEncoder
from ..utils.cfg import enum_value
from . import register_model
from ._fused import FusedEncoderModel


class EncoderArch(Enum):
    Transformer = "transformer"
    Conformer = "conformer"


class DecoderArch(Enum):
    Transformer = "transformer"


@dataclass
class U2Config(LiteasrDataclass):
    name: Optional[str] = field(default="U2")
    dropout_rate: float = field(default=0.0)
    enc_arch: EncoderArch = field(default=EncoderArch.Conformer)
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
    dec_arch: DecoderArch = field(default=DecoderArch.Transformer)
    vocab_size: int = field(default=MISSING)
    dec_dim: int = field(default=256)
    dec_ff_dim: int = field(default=2048)
    dec_attn_heads: int = field(default=4)
    dec_dropout_rate: float = II("model.dropout_rate")
    dec_pos_dropout_rate: float = II("model.dec_dropout_rate")
    dec_self_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_src_attn_dropout_rate: float = II("model.dec_dropout_rate")
    dec_ff_dropout_rate: float = II("model.dec_dropout_rate")
    dec_layers: int = field(default=6)
    # liteasr_amd extensions
    compute_dtype: str = field(default="bf16")
    chunk_size: int = field(default=0)
    dynamic_chunk: bool = field(default=False)
    max_chunk: int = field(default=25)


def _arch(v, enum):
    v = enum_value(v)
    if isinstance(v, str):
        for e in enum:
            if v.lower() in (e.value, e.name.lower()):
                return e.value
    return v


@register_model("U2", dataclass=U2Config)
class U2(FusedEncoderModel):
    def __init__(self, cfg: U2Config, task=None):
        super().__init__()
        g = lambda k, d=None: getattr(cfg, k, d)  # noqa: E731
        self.encoder = TransformerEncoder(
            use_rel=g("use_rel", True), i_dim=g("input_dim"), h_dim=g("enc_dim"), ff_dim=g("enc_ff_dim"),
            n_head=g("enc_attn_heads"), n_layer=g("enc_layers"), dropout_rate=float(g("enc_dropout_rate")),
            pos_dropout_rate=float(g("enc_pos_dropout_rate")), attn_dropout_rate=float(g("enc_attn_dropout_rate")),
            ff_dropout_rate=float(g("enc_ff_dropout_rate")), activation=g("activation", "swish"),
            arch=_arch(g("enc_arch", "conformer"), EncoderArch))
        self.decoder = TransformerDecoder(
            i_dim=g("vocab_size"), h_dim=g("dec_dim"), ff_dim=g("dec_ff_dim"), n_head=g("dec_attn_heads"),
            n_layer=g("dec_layers"), dropout_rate=float(g("dec_dropout_rate")),
            pos_dropout_rate=float(g("dec_pos_dropout_rate")),
            self_attn_dropout_rate=float(g("dec_self_attn_dropout_rate")),
            src_attn_dropout_rate=float(g("dec_src_attn_dropout_rate")),
            ff_dropout_rate=float(g("dec_ff_dropout_rate")), arch=_arch(g("dec_arch", "transformer"), DecoderArch))
        self.ctc = CTC(i_dim=g("enc_dim"), o_dim=g("vocab_size"), dropout_rate=float(g("dropout_rate", 0.0)))
        self.ignore = -1
        self.blank = 0
        self.sos = g("vocab_size") - 1
        self.eos = g("vocab_size") - 1
        cd = str(g("compute_dtype", "bf16")).lower()
        self.compute_dtype = torch.float32 if cd in ("fp32", "float32", "float") else torch.bfloat16
        self.chunk_size = int(g("chunk_size", 0) or 0)
        self.dynamic_chunk = bool(g("dynamic_chunk", False))
        self.chunk_max = int(g("max_chunk", 25) or 25)
        self.vocab_size = g("vocab_size")
        self._finalize()

    def get_target(self, ys, ylens) -> Tuple[Tensor, Tensor]:
        """liteasr/models/u2.py:323-333."""
        ignore = torch.full((ys.size(0), 1), self.ignore, dtype=ys.dtype, device=ys.device)
        tgt_attn = torch.cat([ys, ignore], dim=1)
        tgt_attn[torch.arange(len(ylens), device=ys.device), ylens] = self.eos
        return tgt_attn, ys

    def get_target_len(self, ylens) -> Tensor:
        return ylens

    # ----------------------------------------------------------------- forward
    def forward(self, xs, xlens, ys, ylens):
        x, prep, env = self._run_encoder(xs, xlens, ys, ylens)
        B, T, L1 = prep.B, prep.T, prep.L + 1
        h_attn, h_ctc = FN.HeadsFn.apply(x, self.ctc.ctc_lo.weight, self, env)
        return h_attn.view(B, L1, -1), h_ctc.view(B, T, -1)

    # --------------------------------------------------------------- inference
    def _prep_targets(self, ys, ylens, B, Tx):
        """_prep for a decoder-only pass: every one of the Tx frames valid."""
        xs = torch.empty(B, Tx, 0, device=ys.device)  # shape / device only
        xlens = torch.full((B,), Tx, dtype=torch.int64, device=ys.device)
        return self._prep(xs, xlens, ys, ylens)

    @torch.no_grad()
    def inference(self, x):
        """liteasr/models/u2.py:160-161."""
        return self.attention_rescore(x)

    @torch.no_grad()
    def attention(self, x):
        """liteasr/models/u2.py:163-216 (beam 10); returns the best hypothesis incl. sos."""
        return D.attention_beam_search(self, x, beam=10)

    @torch.no_grad()
    def _ctc_prefix_beam_search(self, x):
        """liteasr/models/u2.py:218-263: ([(tokens tuple, score)], h (1, T', d))."""
        hyps, h, T = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return [(tuple(t), sc) for t, sc in hyps], h.view(1, T, -1).clone()

    @torch.no_grad()
    def ctc_prefix_beam_search(self, x):
        """liteasr/models/u2.py:265-267."""
        hyps, _, _ = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return tuple(hyps[0][0])

    @torch.no_grad()
    def attention_rescore(self, x):
        """liteasr/models/u2.py:269-317 (ctc weight 0.5)."""
        hyps, h, T = D.ctc_prefix_beam_search_nbest(self, x, beam=10)
        return tuple(hyps[D.rescore(self, hyps, h, T, ctc_weight=0.5)][0])

    @classmethod
    def build_model(cls, cfg: U2Config, task=None):
        cfg.input_dim = task.feat_dim
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)
