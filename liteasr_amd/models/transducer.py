"""Transducer (liteasr/models/transducer.py) on the fused HIP encoder.

Same config schema, registry name ("transducer"), state_dict keys and call conventions as
the reference: ``model(xs, xlens, ys, ylens) -> h_jnt (B, T', Lmax + 1, V)`` (raw joint
logits; the RNN-T criterion, criterions/rnnt.py, applies the log-softmax), get_pred_len /
get_target / get_target_len.  The encoder is U2's fused Conformer stack (models/_fused.py);
everything after it -- encoder after_norm, lin_enc, the LSTM prediction network
(nets/rnn_decoder.py), lin_dec, the tanh joint and lin_jnt -- is one fused autograd node
(nets/functional.py TransducerHeadsFn) on csrc/rnnt.hip and the GEMM kernels.

Initialisation follows the reference's _init_module (transducer.py:223-231: LeCun normal for
the prediction network and the three joint projections, N(0, 1) embedding, forget-gate
biases 1) after the same construction order, so torch.manual_seed(s) gives the same
weights.  Extensions (default off): compute_dtype ("bf16" default, "fp32" parity build).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import Enum
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor

from ..config import II, MISSING, LiteasrDataclass
from ..nets import functional as FN
from ..nets.modules import Joint, RNNDecoder, TransformerEncoder
from ..utils.cfg import enum_value
from . import register_model
from ._fused import FusedEncoderModel


class EncoderArch(Enum):
    Transformer = "transformer"
    Conformer = "conformer"


class DecoderArch(Enum):
    LSTM = "lstm"


@dataclass
class TransducerConfig(LiteasrDataclass):
    name: Optional[str] = field(default="transducer")
    joint_dim: int = field(default=768)
    dropout_rate: float = field(default=0.0)
    enc_arch: EncoderArch = field(default=EncoderArch.Transformer)
    use_rel: bool = field(default=True)
    input_dim: int = field(default=MISSING)
    enc_dim: int = field(default=256)
    enc_ff_dim: int = field(default=2048)
    enc_attn_heads: int = field(default=4)
    enc_dropout_rate: float = II("model.dropout_rate")
    enc_pos_dropout_rate: float = II("model.enc_dropout_rate")
    enc_attn_dropout_rate: float = II("model.enc_dropout_rate")
    enc_ff_dropout_rate: float = II("model.enc_dropout_rate")
    enc_layers: int = field(default=4)
    activation: str = field(default="relu")
    dec_arch: DecoderArch = field(default=DecoderArch.LSTM)
    vocab_size: int = field(default=MISSING)
    dec_dim: int = field(default=256)
    dec_units: int = field(default=2048)
    dec_dropout_rate: float = II("model.dropout_rate")
    dec_layers: int = field(default=2)
    # liteasr_amd extension
    compute_dtype: str = field(default="bf16")


def _lecun(module):
    """liteasr/nets/initialization.py:8-30."""
    for p in module.parameters():
        data = p.data
        if data.dim() == 1:
            data.zero_()
        elif data.dim() == 2:
            data.normal_(0, 1.0 / math.sqrt(data.size(1)))
        else:
            n = data.size(1)
            for k in data.size()[2:]:
                n *= k
            data.normal_(0, 1.0 / math.sqrt(n))


@register_model("transducer", dataclass=TransducerConfig)
class Transducer(FusedEncoderModel):
    def __init__(self, cfg: TransducerConfig, task=None):
        super().__init__()
        g = lambda k, d=None: getattr(cfg, k, d)  # noqa: E731
        arch = enum_value(g("enc_arch", "transformer"))
        arch = arch.lower() if isinstance(arch, str) else arch
        self.encoder = TransformerEncoder(
            use_rel=g("use_rel", True), i_dim=g("input_dim"), h_dim=g("enc_dim"), ff_dim=g("enc_ff_dim"),
            n_head=g("enc_attn_heads"), n_layer=g("enc_layers"), dropout_rate=float(g("enc_dropout_rate")),
            pos_dropout_rate=float(g("enc_pos_dropout_rate")), attn_dropout_rate=float(g("enc_attn_dropout_rate")),
            ff_dropout_rate=float(g("enc_ff_dropout_rate")), activation=g("activation", "relu"), arch=arch)
        V = g("vocab_size")
        self.decoder = RNNDecoder(i_dim=V, h_dim=g("dec_dim"), h_units=g("dec_units"), n_layer=g("dec_layers"),
                                  dropout_rate=float(g("dec_dropout_rate")))
        J = g("joint_dim")
        self.lin_enc = nn.Linear(g("enc_dim"), J)
        self.lin_dec = nn.Linear(g("dec_units"), J, bias=False)
        self.lin_jnt = nn.Linear(J, V)
        self.joint_activation = nn.Tanh()
        self.ignore = -1
        self.blank = 0
        self.sos = self.eos = V - 1  # only for the shared bookkeeping kernel (unused here)
        self.vocab_size = V
        cd = str(g("compute_dtype", "bf16")).lower()
        self.compute_dtype = torch.float32 if cd in ("fp32", "float32", "float") else torch.bfloat16
        self.chunk_size = 0
        # transducer.py:223-231
        _lecun(self.decoder)
        _lecun(self.lin_enc)
        _lecun(self.lin_dec)
        _lecun(self.lin_jnt)
        self.decoder.embed.weight.data.normal_(0, 1)
        for cell in self.decoder.dec_layers:
            n = cell.bias_ih.size(0)
            cell.bias_ih.data[n // 4:n // 2].fill_(1.0)
        self._finalize()
        joint = Joint(self)
        joint._store = self.store
        object.__setattr__(self, "joint_params", joint)  # a view bundle, not a submodule

    def _head_units(self):
        """TransducerHeadsFn.backward order: lin_jnt, lin_dec, the prediction network, lin_enc."""
        return ["lin_jnt", "lin_dec", "decoder", "lin_enc"]

    def forward(self, xs, xlens, ys, ylens):
        """transducer.py:106-121."""
        x, prep, env = self._run_encoder(xs, xlens, ys, ylens)
        B, T = prep.B, prep.T
        ys_d = ys.to(device=xs.device, dtype=torch.int64)
        U1 = ys_d.shape[1] + 1
        # _preprocess ys_in (transducer.py:211-214), time-major for the prediction network
        ys_in = torch.cat([torch.zeros(B, 1, dtype=torch.int64, device=xs.device),
                           ys_d.masked_fill(ys_d == self.ignore, self.blank)], 1)
        ids = ys_in.t().contiguous().view(-1).to(torch.int32)
        h = FN.TransducerHeadsFn.apply(x, self.lin_jnt.weight, self, env, ids, U1)
        return h.view(B, T, U1, self.vocab_size)

    def get_pred_len(self, xlens) -> Tensor:
        """transducer.py:186-188."""
        return super().get_pred_len(xlens)

    def get_target(self, ys, ylens) -> Tensor:
        return ys

    def get_target_len(self, ylens) -> Tensor:
        return ylens

    @classmethod
    def build_model(cls, cfg: TransducerConfig, task=None):
        cfg.input_dim = task.feat_dim
        cfg.vocab_size = task.vocab_size
        return cls(cfg, task)
