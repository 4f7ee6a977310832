"""Fused flat Adam with in-kernel gradient clipping and NaN-skip.

One sum-of-squares pass over the flat grad buffer, one finalize kernel (norm, clip
coefficient, NaN check, step counter, Noam lr -- all on the device) and one update
pass that also refreshes the low-precision working copy of the weights.  Semantics:
torch.nn.utils.clip_grad_norm_ (liteasr/trainer.py:153-156) + skip when the norm is
NaN (:157) + torch.optim.Adam (liteasr/optims/adam.py:27-34) under Noam
(liteasr/optims/noam.py:33-46).  No host synchronisation.
"""

from __future__ import annotations

import torch

from .. import kernels as K
from ..utils.param_store import FlatParams


def find_store(params) -> FlatParams:
    params = list(params)
    for p in params:
        st = getattr(p, "_lasr_store", None)
        if st is not None:
            return st
    raise TypeError("fused Adam expects parameters of a liteasr_amd model (FlatParams-backed)")


class FlatAdamState:
    def __init__(self, store: FlatParams):
        self.store = store
        dev = store.flat.device
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        self.state = torch.zeros(5, dtype=torch.float32, device=dev)
        self.nparts = K.sumsq_nparts(store.numel)
        self.ws = torch.empty(self.nparts, dtype=torch.float32, device=dev)

    def to(self, dev):
        for k in ("m", "v", "state", "ws"):
            setattr(self, k, getattr(self, k).to(dev))

    def step(self, max_norm, lr_mode, lr, factor, model_dim, warmup, beta1, beta2, eps, wd):
        st = self.store
        if K.held_reductions():  # an encoder layer's gradient reductions were never launched
            raise RuntimeError("FusedAdam.step: parameter-gradient reductions still queued")
        if self.m.device != st.flat.device:
            self.to(st.flat.device)
        g = st.ensure_grad()
        work = st.working()
        lp = None if work is st.flat else work
        K.sumsq_partial(g, self.ws)
        K.adam_step(st.flat, lp, g, self.m, self.v, self.ws, self.nparts, self.state, max_norm,
                    lr_mode, lr, factor, model_dim, warmup, beta1, beta2, eps, wd)
        st.mark_work_synced()

    def read(self):
        s = self.state.tolist()
        return {"step": int(s[0]), "lr": s[1], "grad_norm": s[2], "skipped": bool(s[3]), "clip_coef": s[4]}
