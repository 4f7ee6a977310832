"""RNN-T loss (liteasr/criterions/rnnt.py): the batch-mean transducer loss of the raw joint
logits with the log-softmax fused, blank = blank_id, on csrc/rnnt.hip.  Both of the
reference's back ends (trans_type "warp-transducer": warprnnt_pytorch.RNNTLoss(blank),
reduction mean; "warp-rnnt": warp_rnnt.rnnt_loss(log_softmax(x), ..., reduction="mean",
gather=True)) compute this same quantity; the kernel is one implementation for both."""

from dataclasses import dataclass, field
from typing import Optional

import torch

from ..config import LiteasrDataclass
from ..nets.functional import RNNTLossFn
from . import LiteasrLoss, register_criterion


@dataclass
class RNNTLossConfig(LiteasrDataclass):
    name: Optional[str] = field(default="rnnt")
    trans_type: str = field(default="warp-transducer")
    blank_id: int = field(default=0)


@register_criterion("rnnt", dataclass=RNNTLossConfig)
class RNNTLoss(LiteasrLoss):
    def __init__(self, cfg: RNNTLossConfig, task=None):
        super().__init__(cfg)
        if cfg.trans_type not in ("warp-transducer", "warp-rnnt"):
            raise NotImplementedError(cfg.trans_type)
        self.trans_type = cfg.trans_type
        self.blank_id = cfg.blank_id

    @classmethod
    def build_criterion(cls, cfg, task):
        return cls(cfg, task)

    def __call__(self, model, xs, xlens, ys, ylens):
        """rnnt.py:45-51."""
        pred_pad = model(xs, xlens, ys, ylens)
        dev = pred_pad.device
        target = model.get_target(ys, ylens).to(device=dev, dtype=torch.int32).contiguous()
        pred_len = model.get_pred_len(xlens).to(device=dev, dtype=torch.int32)
        target_len = model.get_target_len(ylens).to(device=dev, dtype=torch.int32)
        return RNNTLossFn.apply(pred_pad, target, pred_len, target_len, int(self.blank_id))
