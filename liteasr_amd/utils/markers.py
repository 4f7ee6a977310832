"""roctx ranges around the fused autograd nodes (SURVEY §5 tracing plan).

Off by default (one module-level flag test per node call).  ``enable()`` -- or
``LASR_ROCTX=1`` in the environment, or ``bench.py --profile`` -- turns every decorated
node's forward and backward into a named range (``ConformerLayerFn.fwd`` ...), so a
``rocprofv3 --kernel-trace --marker-trace`` run attributes each kernel to its node.  The
ranges go through ``torch.cuda.nvtx``, which the ROCm build of torch routes to roctx.
Ranges are host-side: they mark launch spans, so profile an eager step (a replayed
hipGraph issues no host calls per node)."""

from __future__ import annotations

import functools
import os

ENABLED = os.environ.get("LASR_ROCTX", "0") == "1"


def enable(on: bool = True) -> None:
    global ENABLED
    ENABLED = bool(on)


def _push(tag):
    import torch

    torch.cuda.nvtx.range_push(tag)


def _pop():
    import torch

    torch.cuda.nvtx.range_pop()


def ranged(cls):
    """Class decorator for a torch.autograd.Function: roctx ranges around forward / backward."""
    for name, suffix in (("forward", "fwd"), ("backward", "bwd")):
        fn = cls.__dict__[name].__func__
        tag = f"{cls.__name__}.{suffix}"

        def make(fn=fn, tag=tag):
            @functools.wraps(fn)
            def wrapper(*args, **kwargs):
                if not ENABLED:
                    return fn(*args, **kwargs)
                _push(tag)
                try:
                    return fn(*args, **kwargs)
                finally:
                    _pop()

            return staticmethod(wrapper)

        setattr(cls, name, make())
    return cls
