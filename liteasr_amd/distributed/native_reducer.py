"""ctypes binding of libliteasr_comm.so (include/liteasr_comm.h): the bucketed gradient
reducer as a C-ABI over RCCL, the comm-side boundary SURVEY §8(b) plans (``lasr_reducer_*``).

``FlatReducer(..., comm="native")`` drives it instead of ``torch.distributed.all_reduce``:
each bucket's in-place ``ncclAllReduce(ncclAvg)`` runs on the library's own HIP stream after
an event recorded on the producing stream, in bucket order, and ``finalize`` makes the
consumer stream wait.  The communicator is the library's own (``ncclCommInitRank`` from a
unique id that rank 0 creates and the process group broadcasts), so it works under any
torch.distributed backend.  Reference mechanism replaced: torch DDP at
liteasr/trainer.py:76-88.  No fallback: a missing library raises.
"""

from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libliteasr_comm.so")

_SIGS = {
    "lasr_reducer_uid_bytes": (ctypes.c_int, []),
    "lasr_reducer_get_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "lasr_reducer_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                           ctypes.c_int]),
    "lasr_reducer_create_from_comm": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                                     ctypes.POINTER(ctypes.c_int64),
                                                     ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "lasr_reducer_mark_grad_ready": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "lasr_reducer_finalize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lasr_reducer_launched": (ctypes.c_int, [ctypes.c_void_p]),
    "lasr_reducer_reset": (ctypes.c_int, [ctypes.c_void_p]),
    "lasr_reducer_rebind": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "lasr_reducer_set_single_rank_collectives": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "lasr_reducer_grad": (ctypes.c_void_p, [ctypes.c_void_p]),
    "lasr_reducer_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "lasr_comm_last_error": (ctypes.c_char_p, []),
}


def load():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_PATH):
            raise RuntimeError(f"{_PATH} missing: run `make` (no fallback for the native reducer)")
        lib = ctypes.CDLL(_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _LIB = lib
    return _LIB


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {load().lasr_comm_last_error().decode()} (rc {rc})")


def unique_id(process_group=None) -> bytes:
    """Rank 0 creates the RCCL id; every rank of the group receives the same bytes."""
    L = load()
    buf = ctypes.create_string_buffer(L.lasr_reducer_uid_bytes())
    if dist.get_rank(process_group) == 0:
        _check(L.lasr_reducer_get_unique_id(buf), "lasr_reducer_get_unique_id")
    obj = [bytes(buf.raw)]
    src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=process_group)
    return obj[0]


class NativeReducer:
    """Buckets = [(lo, hi)] element ranges of the flat fp32 gradient ``grad`` (on the GPU)."""

    def __init__(self, grad: torch.Tensor, buckets, uid: bytes, world: int, rank: int):
        assert grad.is_cuda and grad.dtype == torch.float32 and grad.is_contiguous()
        L = load()
        self.grad = grad  # keeps the buffer alive as long as the reducer
        self.device = grad.device.index
        n = len(buckets)
        lo = (ctypes.c_int64 * n)(*[int(b[0]) for b in buckets])
        hi = (ctypes.c_int64 * n)(*[int(b[1]) for b in buckets])
        self._h = ctypes.c_void_p()
        _check(L.lasr_reducer_create(ctypes.byref(self._h), uid, world, rank, grad.device.index,
                                     grad.data_ptr(), grad.numel(), lo, hi, n), "lasr_reducer_create")

    @staticmethod
    def _stream(stream):
        return (stream or torch.cuda.current_stream()).cuda_stream

    def mark(self, bucket: int, stream=None):
        _check(load().lasr_reducer_mark_grad_ready(self._h, bucket, self._stream(stream)),
               "lasr_reducer_mark_grad_ready")

    def finalize(self, stream=None):
        _check(load().lasr_reducer_finalize(self._h, self._stream(stream)), "lasr_reducer_finalize")

    def launched(self) -> int:
        return load().lasr_reducer_launched(self._h)

    def reset(self):
        """Drop the current step's marks (an abandoned backward); launches nothing."""
        _check(load().lasr_reducer_reset(self._h), "lasr_reducer_reset")

    def grad_ptr(self) -> int:
        return load().lasr_reducer_grad(self._h) or 0

    def rebind(self, grad: torch.Tensor):
        """Average ``grad`` from now on (same numel, same device; between steps only).  The
        communicator, stream and events belong to the creation device: a buffer on another
        device is refused (here and by the C side)."""
        assert grad.dtype == torch.float32 and grad.is_contiguous()
        if not grad.is_cuda or grad.device.index != self.device:
            raise RuntimeError(f"NativeReducer.rebind: the buffer is on {grad.device}, the reducer on cuda:{self.device} "
                               "(a device move of the model needs a new DistributedDataParallel wrapper)")
        _check(load().lasr_reducer_rebind(self._h, grad.data_ptr(), grad.numel()), "lasr_reducer_rebind")
        self.grad = grad

    def set_single_rank_collectives(self, on: bool):
        """World 1 issues no collective by default (the average is the identity); ``on`` issues
        the 1-rank RCCL all-reduces anyway, to measure their cost beside the backward."""
        _check(load().lasr_reducer_set_single_rank_collectives(self._h, int(bool(on))),
               "lasr_reducer_set_single_rank_collectives")

    def close(self):
        if self._h:
            load().lasr_reducer_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
