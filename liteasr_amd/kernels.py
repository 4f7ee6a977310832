"""Torch-tensor front end of the HIP kernels (thin: strides/pointers/stream only).

Every function here launches kernels from libliteasr_hip.so on the current HIP stream
(``torch.cuda.current_stream()``) and never synchronises, so a training step built
from them can be captured into a hipGraph.  Tensors must live on the GPU; there is
no CPU path (the CPU restatement lives in ``oracle/`` and is test-only).
"""

from __future__ import annotations

import contextlib
import os
import ctypes as C
import math
from typing import Optional

import torch

from . import _native as N

_DT = {torch.float32: N.F32, torch.bfloat16: N.BF16}


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------------ workspace ---
class _Workspace:
    """One growing fp32 scratch buffer per device (stream-ordered reuse)."""

    def __init__(self):
        self.buf = {}
        self.frozen = False

    def get(self, nfloats: int, device) -> torch.Tensor:
        nfloats = max(int(nfloats), 1)
        key = torch.device(device).index
        b = self.buf.get(key)
        if b is None or b.numel() < nfloats:
            if self.frozen or torch.cuda.is_current_stream_capturing():
                raise RuntimeError(
                    "workspace growth during graph capture; run a warm-up step first"
                )
            b = torch.empty(int(nfloats * 1.25) + 1024, dtype=torch.float32, device=device)
            self.buf[key] = b
        return b


WS = _Workspace()


# --------------------------------------------------------- deferred reductions ---
class _Deferred:
    """Parameter-gradient reductions parked until the end of a backward node: the
    partial-sum buffers of LayerNorm gamma/beta, the positional biases and the split-K
    weight gradients (+ their bias rowsums) are collected and finished by ONE
    lasr_reduce_multi launch, with each reduction's usual summation order."""

    def __init__(self):
        self.depth = 0
        self.segs = []
        self.gemms = []  # queued partials-only dW GEMMs: (tile key, args, operand refs)
        self.held = []  # reductions of finished `hold` blocks, not yet launched
        self.done = []  # their on_done callbacks, in block order


_DEFER = _Deferred()


@contextlib.contextmanager
def deferred_reductions(hold=False, on_done=None):
    """Within the block, gradient outputs of layernorm_bwd / qbias_bwd / split-K weight
    GEMMs (split_k=0, beta 0 or 1, fp32 contiguous C) are only complete after the block
    exits; nothing inside may read them.  on_done() runs once they are complete.

    hold=True (the encoder layers' backward nodes): the grouped weight-gradient launches still
    run at the end of the block, but its reductions wait in a queue (their partial buffers
    alive) for the next block that does not hold, or flush_reductions(): the reductions of
    several layers then share lasr_reduce_multi launches, each with its usual summation order,
    and the held blocks' on_done callbacks run after them, in order."""
    _DEFER.depth += 1
    ok = False
    try:
        yield
        ok = True
    finally:
        _DEFER.depth -= 1
        if _DEFER.depth == 0:
            if hold and ok:
                if _DEFER.gemms:
                    _flush_gemm_group()
                _DEFER.held.extend(_DEFER.segs)
                _DEFER.segs = []
                if on_done is not None:
                    _DEFER.done.append(on_done)
            else:
                if on_done is not None:
                    _DEFER.done.append(on_done)
                flush_reductions()


def held_reductions():
    """Number of reductions queued by hold blocks and not yet launched."""
    return len(_DEFER.held)


def _defer(part, P, Ncols, out0, out1=None, split=None, accumulate=True):
    _DEFER.segs.append((part, int(P), int(Ncols), out0, out1, int(split if split is not None else Ncols),
                        int(accumulate)))


# Grouped weight gradients: dW GEMMs marked group=True inside a deferred_reductions block are
# queued and launched at its end, one lasr_gemm_dw_group launch per planned tile (<= 8
# problems each), before the reductions (tests set DW_GROUP = False to compare with lone launches).
DW_GROUP = True
# plan tile -> group (lasr_gemm_dw_group runs the 64 x 128 / 128 x 64 plans, the FFN-sized
# weights, on 128 x 128 tiles)
_GROUP_TILES = {(64, 64): (64, 64), (64, 128): (128, 128), (128, 64): (128, 128)}
# grouped problems fill the chip together: each takes 1/div of the K slices the planner gives
# a lone launch (fewer fp32 partial slabs to write and reduce); 128 x 128 groups keep half
# (the other divisors measured slower)
DW_GROUP_SPLIT_DIV = {(64, 64): 4, (128, 128): 2}
# Direct grouped weight gradients: FFN-sized problems with >= this many full-K 128 x 128 tiles
# (the d 512 FFN weights: 64 each, a group of four = 256 tiles) skip the K split and write the
# gradient itself (beta = 1), no fp32 partial slab to write and reduce.  Measured at config 4
# (VERDICT r05 item 3): 20.13 -> 20.74 ms per step, the full-K 128 x 128 tiles are L2-feed bound
# where the 256 x 128 split-2 tiles are not (profiles/r06/step_ab_dw_direct_large_rejected.jsonl,
# DESIGN §4); 0 = off.  tests/test_kernels_gpu.py::test_gemm_dw_group_direct pins the path.
DW_DIRECT_MIN_TILES = 0


# GEMMs whose 64 x 64 grid cannot fill half the chip and whose K is long are split over K
# (lasr_gemm autosplit; the split-K reduction applies the epilogue).
SMALL_GRID_SPLIT = True
SMALL_GRID_TILES = 128  # (64 x 64 tiles below which a K >= 1024 GEMM is split)


def _group_div(key):
    d = DW_GROUP_SPLIT_DIV
    return d.get(key, 1) if isinstance(d, dict) else d
_GROUP_MAX = 8


# grouped dW blocks laid out longest K slice first (lasr_gemm_dw_group_order; same bits)
DW_GROUP_LPT = True
_dw_order_set = [None]


def _flush_gemm_group():
    q, _DEFER.gemms = _DEFER.gemms, []
    if _dw_order_set[0] != DW_GROUP_LPT:
        N.call("lasr_gemm_dw_group_order", int(DW_GROUP_LPT))
        _dw_order_set[0] = DW_GROUP_LPT
    byt = {}
    for key, args, refs in q:
        byt.setdefault(key, []).append(args)
    for key, lst in byt.items():
        for i in range(0, len(lst), _GROUP_MAX):
            chunk = lst[i:i + _GROUP_MAX]
            arr = (N.GemmArgs * len(chunk))(*chunk)
            N.call("lasr_gemm_dw_group", arr, len(chunk), stream())
    # the operand references in q die here, after the launches were enqueued


def _flush_node_end(segs):
    if _DEFER.gemms:
        _flush_gemm_group()
    if segs:
        arr = (N.ReduceSeg * len(segs))()
        for i, (part, P, Ncols, o0, o1, split, acc) in enumerate(segs):
            arr[i] = N.ReduceSeg(ptr(part), Ncols, P, acc, ptr(o0), ptr(o1), split)
        N.call("lasr_reduce_multi", arr, len(segs), stream())


def flush_reductions():
    segs = _DEFER.held + _DEFER.segs
    _DEFER.held, _DEFER.segs = [], []
    done, _DEFER.done = _DEFER.done, []
    if segs or _DEFER.gemms:
        _flush_node_end(segs)
    for fn in done:
        fn()
    # the partial buffers are released here; the caching allocator hands their memory only
    # to work stream-ordered after the reduction



# ----------------------------------------------------------------------- GEMM ---
# the planner's 64 x 64 tiles for outputs at most 64 wide (lasr_gemm_narrow_tiles; same bits)
GEMM_NARROW_TILES = True
_narrow_set = [None]


def _split(t: torch.Tensor):
    """(batch strides (s1, s2), batch shape (z1, z2), row stride, col stride)."""
    nb = t.dim() - 2
    assert 0 <= nb <= 2, "gemm operands take at most 2 batch dims"
    st = t.stride()
    sh = t.shape
    if nb == 0:
        return (0, 0), (1, 1), st[0], st[1]
    if nb == 1:
        return (st[0], 0), (sh[0], 1), st[1], st[2]
    return (st[0], st[1]), (sh[0], sh[1]), st[2], st[3]


def gemm(
    a: torch.Tensor,
    b: torch.Tensor,
    c: torch.Tensor,
    *,
    alpha: float = 1.0,
    alpha_dev: Optional[torch.Tensor] = None,
    beta: float = 0.0,
    bias: Optional[torch.Tensor] = None,
    act: int = N.ACT_NONE,
    zout: Optional[torch.Tensor] = None,
    aux: Optional[torch.Tensor] = None,
    aux_act: int = N.ACT_NONE,
    drop_p: float = 0.0,
    drop_seed: int = 0,
    res: Optional[torch.Tensor] = None,
    res_scale: float = 1.0,
    split_k: int = 1,
    rowsum: Optional[torch.Tensor] = None,
    plan_only: bool = False,
    zout_mode: int = 0,
    group: bool = False,
    tile: Optional[tuple] = None,
    ksub: int = 0,
    ln_fwd: Optional[tuple] = None,
    ln_bwd: Optional[object] = None,
    qbias: Optional[tuple] = None,
):
    """c = epilogue(alpha * a @ b) for logical views a (..,M,K), b (..,K,N), c (..,M,N).

    Views may be arbitrarily strided as long as each operand has one unit stride
    (the kernel handles K-contiguous and M/N-contiguous operands).

    tile=(tile_m, tile_n) / ksub: per-call plan overrides of the LDS-DMA tile and ring-stage depth
    (A/B tools, bit-identity tests); None / 0 = the planner.

    group=True (a split-K weight gradient inside deferred_reductions): the launch itself may
    be deferred to the end of the block and grouped with the block's other dW GEMMs, so
    the caller must not modify a or b before the block exits.

    ln_fwd=(gamma, beta, eps, y, mean, rstd): the LayerNorm of c's rows follows
    (lasr_gemm_ln_fwd: in the split-K reduction launch when K is split).  ln_bwd=lnb (an
    object with x, g, mean, rstd, dx, dgamma, dbeta, dres, gb, bscale, bp, bseed): the
    LayerNorm backward of c = dln follows (lasr_gemm_ln_bwd), its dgamma / dbeta partials
    deferred or reduced like layernorm_bwd's.  qbias=(dqu, dqv, B, T, H, dk, dqkv, du, dv):
    qbias_bwd's work runs beside this GEMM's split-K reduction (lasr_gemm_qbias_bwd)."""
    if _narrow_set[0] != GEMM_NARROW_TILES:
        N.call("lasr_gemm_narrow_tiles", int(GEMM_NARROW_TILES))
        _narrow_set[0] = GEMM_NARROW_TILES
    M, K = a.shape[-2], a.shape[-1]
    K2, Nn = b.shape[-2], b.shape[-1]
    assert K == K2 and c.shape[-2] == M and c.shape[-1] == Nn, (a.shape, b.shape, c.shape)
    assert a.dtype == b.dtype
    (sa1, sa2), (za1, za2), a_m, a_k = _split(a)
    (sb1, sb2), (zb1, zb2), b_k, b_n = _split(b)
    (sc1, sc2), (zc1, zc2), c_m, c_n = _split(c)
    assert c_n == 1, "C must be row-contiguous"
    z1, z2 = zc1, zc2
    assert (za1, za2) == (z1, z2) and (zb1, zb2) == (z1, z2), "batch shapes differ"
    if a_k != 1 and a_m != 1:
        raise ValueError("A needs a unit stride")
    if b_k != 1 and b_n != 1:
        raise ValueError("B needs a unit stride")
    args = N.GemmArgs()
    args.M, args.N, args.K = M, Nn, K
    args.batch, args.batch_div = z1 * z2, z2
    args.A, args.lda_m, args.lda_k, args.sa1, args.sa2 = ptr(a), a_m, a_k, sa1, sa2
    # B logical [K,N]: kernel wants ldb_n (stride along n) and ldb_k (stride along k)
    args.B, args.ldb_n, args.ldb_k, args.sb1, args.sb2 = ptr(b), b_n, b_k, sb1, sb2
    args.C, args.ldc, args.sc1, args.sc2 = ptr(c), c_m, sc1, sc2
    if a_k == 1 and a_m == 1:
        args.lda_k = 1
    if b_k == 1 and b_n == 1:
        args.ldb_k = 1
    args.in_dtype, args.c_dtype = dt(a), dt(c)
    args.alpha, args.alpha_dev, args.beta = alpha, ptr(alpha_dev), beta
    args.bias = ptr(bias)
    args.act = act
    args.zout = ptr(zout)
    args.zout_mode = zout_mode
    if aux is not None:
        args.aux, args.aux_dtype, args.ldaux, args.aux_act = ptr(aux), dt(aux), aux.stride(0), aux_act
    args.drop_p, args.drop_seed = drop_p, drop_seed
    if tile is not None:
        args.tile_m, args.tile_n = int(tile[0]), int(tile[1])
    args.ksub = int(ksub)
    if res is not None:
        args.res, args.res_dtype, args.ldres, args.res_scale = ptr(res), dt(res), res.stride(0), res_scale
    auto_split = (split_k == 1 and SMALL_GRID_SPLIT and rowsum is None and zout is None and not group
                  and a.dtype == torch.bfloat16 and z1 * z2 == 1 and K >= 1024
                  and ((M + 63) // 64) * ((Nn + 63) // 64) < SMALL_GRID_TILES)
    if auto_split:  # small grid, long K (the decoder's B*(L+1)-row GEMMs): split K, reduce with the epilogue
        split_k = 0
    args.split_k = split_k
    if rowsum is not None:
        # fused bias gradient rowsum[m] += sum_k a[m, k] (fp32, a M-contiguous)
        assert rowsum.dtype == torch.float32 and rowsum.is_contiguous() and rowsum.numel() == M
        assert z1 * z2 == 1 and a_m == 1, "rowsum needs batch 1 and an M-contiguous A"
        args.rowsum = ptr(rowsum)
    if split_k != 1 or rowsum is not None:
        ns = 64 if split_k <= 0 else split_k
        need = ns * z1 * z2 * M * Nn + (ns + 128) * M if rowsum is not None else ns * z1 * z2 * M * Nn
        ws = WS.get(need, c.device)
        args.workspace, args.workspace_bytes = ptr(ws), ws.numel() * 4
    if plan_only:
        tm, tn, sp, fl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        N.call("lasr_gemm_plan", C.byref(args), C.byref(tm), C.byref(tn), C.byref(sp), C.byref(fl))
        if plan_only == "flags":
            return tm.value, tn.value, sp.value, fl.value
        return tm.value, tn.value, sp.value
    if (_DEFER.depth and split_k == 0 and not auto_split and beta in (0.0, 1.0) and alpha == 1.0 and alpha_dev is None
            and bias is None and act == N.ACT_NONE and zout is None and aux is None and res is None
            and drop_p <= 0.0 and z1 * z2 == 1 and c.dtype == torch.float32 and c.is_contiguous()):
        tm, tn, sp, fl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        N.call("lasr_gemm_plan", C.byref(args), C.byref(tm), C.byref(tn), C.byref(sp), C.byref(fl))
        sp = sp.value
        grouped = (group and DW_GROUP and (tm.value, tn.value) in _GROUP_TILES
                   and (fl.value & 1) and a_m == 1 and b_n == 1 and a.dtype == torch.bfloat16)
        if (grouped and DW_DIRECT_MIN_TILES > 0 and _GROUP_TILES[(tm.value, tn.value)] == (128, 128)
                and ((M + 127) // 128) * ((Nn + 127) // 128) >= DW_DIRECT_MIN_TILES):
            # full-K direct problem of the group: C itself (beta 0 / 1), its bias rowsum direct
            args.split_k = 1
            args.workspace, args.workspace_bytes = None, 0
            _DEFER.gemms.append(((128, 128, "direct"), N.GemmArgs.from_buffer_copy(args), (a, b, c, rowsum)))
            return c
        div = _group_div(_GROUP_TILES[(tm.value, tn.value)]) if grouped else 1
        if grouped and (div > 1 or sp < 2):
            # short K too (the positional-projection weight, K = T'): two slices join the group
            sp = max(2, sp // max(1, div))
            args.split_k = -sp
            N.call("lasr_gemm_plan", C.byref(args), C.byref(tm), C.byref(tn), C.byref(C.c_int()), C.byref(fl))
            grouped = (tm.value, tn.value) in _GROUP_TILES and bool(fl.value & 1)
        if sp > 1:
            # partials-only launch (split_k = -1) into a buffer that lives until the flush
            # rowsum partials (fused) or the column-sum scratch (unfused, fp32 operands)
            nrs = (sp + 128) * M if rowsum is not None else 0
            part = torch.empty(sp * M * Nn + nrs, dtype=torch.float32, device=c.device)
            # the explicit slice count on both paths: `part` is sized for sp slices, and a
            # re-derived auto split (-1) could differ from sp after the group adjustment
            args.split_k = -sp
            args.workspace, args.workspace_bytes = ptr(part), part.numel() * 4
            if grouped:
                key = _GROUP_TILES[(tm.value, tn.value)]
                _DEFER.gemms.append((key, N.GemmArgs.from_buffer_copy(args), (a, b)))
            else:
                N.call("lasr_gemm", C.byref(args), stream())
            _defer(part, sp, M * Nn, c, accumulate=beta == 1.0)
            if rowsum is not None and fl.value & 2:  # LASR_PLAN_ROWSUM_FUSED: partials follow C's
                _defer(part[sp * M * Nn:], sp, M, rowsum)
            return c
    if ln_fwd is not None:
        g_, b_, eps, y, mean, rstd = ln_fwd
        assert c.dtype == torch.float32 and c.is_contiguous() and z1 * z2 == 1 and rowsum is None
        N.call("lasr_gemm_ln_fwd", C.byref(args), ptr(g_), ptr(b_), float(eps), ptr(y), dt(y), ptr(mean), ptr(rstd),
               stream())
        return c
    if qbias is not None:
        dqu, dqv, B_, T_, H_, dk_, dqkv, du, dv = qbias
        assert c.dtype == dqu.dtype == dqv.dtype == dqkv.dtype
        D_ = H_ * dk_
        nchunk = (B_ * T_ + 63) // 64  # QB_ROWS (qbias.h)
        part = torch.empty(nchunk * 2 * D_, dtype=torch.float32, device=c.device)
        N.call("lasr_gemm_qbias_bwd", C.byref(args), ptr(dqu), ptr(dqv), dt(dqu), B_, T_, H_, dk_, ptr(dqkv),
               dqkv.stride(0), ptr(part), part.numel(), stream())
        if _DEFER.depth:
            _defer(part, nchunk, 2 * D_, du, dv, split=D_)
        else:
            arr = (N.ReduceSeg * 1)()
            arr[0] = N.ReduceSeg(ptr(part), 2 * D_, nchunk, 1, ptr(du), ptr(dv), D_)
            N.call("lasr_reduce_multi", arr, 1, stream())
        return c
    if ln_bwd is not None:
        q = ln_bwd
        assert c.is_contiguous() and z1 * z2 == 1 and rowsum is None
        nblk = (M + 15) // 16  # lasr_layernorm_bwd's 16-row blocks
        defer = _DEFER.depth and q.dgamma is not None and q.dbeta is not None
        # (its own buffer: the GEMM's split-K partials live in WS)
        part = torch.empty(nblk * 2 * Nn, dtype=torch.float32, device=c.device)
        N.call("lasr_gemm_ln_bwd", C.byref(args), ptr(q.x), dt(q.x), ptr(q.g), ptr(q.mean), ptr(q.rstd),
               ptr(q.dres), dt(q.dres) if q.dres is not None else 0, ptr(q.dx), dt(q.dx), ptr(part), part.numel(),
               ptr(q.gb), dt(q.gb) if q.gb is not None else 0, float(q.bscale), float(q.bp), int(q.bseed), stream())
        if defer:
            _defer(part, nblk, 2 * Nn, q.dgamma, q.dbeta, split=Nn)
        elif q.dgamma is not None or q.dbeta is not None:
            assert q.dgamma is not None and q.dbeta is not None
            arr = (N.ReduceSeg * 1)()
            arr[0] = N.ReduceSeg(ptr(part), 2 * Nn, nblk, 1, ptr(q.dgamma), ptr(q.dbeta), Nn)
            N.call("lasr_reduce_multi", arr, 1, stream())
        return c
    N.call("lasr_gemm", C.byref(args), stream())
    return c


def gemm_plan(a, b, c, flags=False, **kw):
    """(tile_m, tile_n, split_k) lasr_gemm would use for this call (nothing is launched);
    flags=True appends the LASR_PLAN_* bits (LDS-DMA path, fused rowsum, 64-deep stages)."""
    return gemm(a, b, c, plan_only="flags" if flags else True, **kw)


def linear(x, w, out, bias=None, **kw):
    """out[M,N] = x[M,K] @ w[N,K]^T (+bias, epilogue kw)."""
    return gemm(x, w.t(), out, bias=bias, **kw)


def dropout_scale(p: float) -> float:
    """Multiplier of kept elements at drop probability p (1 when p <= 0)."""
    return float(N.load().lasr_dropout_scale(float(p))) if p > 0 else 1.0


def colsum(x2d: torch.Tensor, out: torch.Tensor, accumulate=True):
    M, Nn = x2d.shape
    nchunk = max(1, min((M + 63) // 64, 128))  # colsum_chunks in norm.hip
    ws = WS.get(nchunk * Nn, x2d.device)
    N.call("lasr_colsum", ptr(x2d), dt(x2d), M, Nn, x2d.stride(0), ptr(out), int(accumulate),
           ptr(ws), ws.numel(), stream())


# ------------------------------------------------------------------ LayerNorm ---
def layernorm_fwd(x, gamma, beta, eps, y, mean, rstd, y2=None, p2=0.0, seed2=0):
    rows, D = x.shape
    N.call("lasr_layernorm_fwd", ptr(x), dt(x), rows, D, ptr(gamma), ptr(beta), eps, ptr(y),
           dt(y), ptr(mean), ptr(rstd), ptr(y2), dt(y2) if y2 is not None else 0, p2, seed2,
           stream())


def layernorm2_fwd(x, g1, b1, g2, b2, eps, y, mean1, rstd1, z, mean2, rstd2):
    """y = LN1(x) (fp32), z = LN2(y) (bf16), one launch (lasr_layernorm2_fwd)."""
    rows, D = x.shape
    N.call("lasr_layernorm2_fwd", ptr(x), rows, D, ptr(g1), ptr(b1), ptr(g2), ptr(b2), eps, ptr(y), ptr(mean1),
           ptr(rstd1), ptr(z), ptr(mean2), ptr(rstd2), stream())


def layernorm_bwd(x, dy, gamma, mean, rstd, dx, dgamma, dbeta, dres=None, gb=None,
                  bscale=1.0, bp=0.0, bseed=0):
    rows, D = x.shape
    nblk = (rows + 15) // 16  # LN_ROWS_PER_BLOCK (norm.hip)
    defer = _DEFER.depth and dgamma is not None and dbeta is not None
    if defer:
        ws = torch.empty(nblk * 2 * D, dtype=torch.float32, device=x.device)
        og, ob = None, None
    else:
        ws = WS.get(nblk * 2 * D, x.device)
        og, ob = dgamma, dbeta
    N.call("lasr_layernorm_bwd", ptr(x), dt(x), ptr(dy), dt(dy), rows, D, ptr(gamma), ptr(mean),
           ptr(rstd), ptr(dres), dt(dres) if dres is not None else 0, ptr(dx), dt(dx),
           ptr(og), ptr(ob), ptr(ws), ws.numel(), ptr(gb),
           dt(gb) if gb is not None else 0, bscale, bp, bseed, stream())
    if defer:
        _defer(ws, nblk, 2 * D, dgamma, dbeta, split=D)


def layernorm2_bwd(x1, dy1, dres1, g1, mean1, rstd1, dgamma1, dbeta1, x2, g2, mean2, rstd2, dx2, dgamma2, dbeta2,
                   gb2=None, bscale=1.0, bp=0.0, bseed=0):
    """Two LayerNorm backwards per row (lasr_layernorm2_bwd): dx1 = dres1 + LN1'(dy1) (not
    stored), dx2 = LN2'(dx1), gb2 = bscale * drop(dx2); both norms' gamma / beta gradients
    accumulate (deferred inside deferred_reductions)."""
    rows, D = x1.shape
    assert x1.dtype == x2.dtype == dres1.dtype == dx2.dtype == torch.float32
    assert dy1.shape == x1.shape == x2.shape == dres1.shape == dx2.shape
    nblk = (rows + 15) // 16  # LN_ROWS_PER_BLOCK (norm.hip)
    part1 = torch.empty(nblk * 2 * D, dtype=torch.float32, device=x1.device)
    part2 = torch.empty(nblk * 2 * D, dtype=torch.float32, device=x1.device)
    N.call("lasr_layernorm2_bwd", ptr(x1), ptr(dy1), dt(dy1), ptr(dres1), rows, D, ptr(g1), ptr(mean1), ptr(rstd1),
           ptr(part1), ptr(x2), ptr(g2), ptr(mean2), ptr(rstd2), ptr(dx2), ptr(part2), ptr(gb2),
           dt(gb2) if gb2 is not None else 0, bscale, bp, bseed, stream())
    if _DEFER.depth:
        _defer(part1, nblk, 2 * D, dgamma1, dbeta1, split=D)
        _defer(part2, nblk, 2 * D, dgamma2, dbeta2, split=D)
        return
    arr = (N.ReduceSeg * 2)()
    arr[0] = N.ReduceSeg(ptr(part1), 2 * D, nblk, 1, ptr(dgamma1), ptr(dbeta1), D)
    arr[1] = N.ReduceSeg(ptr(part2), 2 * D, nblk, 1, ptr(dgamma2), ptr(dbeta2), D)
    N.call("lasr_reduce_multi", arr, 2, stream())


# ------------------------------------------------- full-row GEMM + LayerNorm ---
def _al16(t):
    return t is None or t.data_ptr() % 16 == 0


# The row kernel's main loop ingests the whole weight per 32-row workgroup, one workgroup per CU:
# measured faster than GEMM + norm up to K = 768 (tools/row_ln_bench.py, profiles/r03), slower at
# K = 2048, where the 64 x 64 GEMM's 2-3 workgroups per CU keep more of the LDS-DMA in flight
# (whole step with the FFN fc2 + norm on the row kernel: 9.83 -> 9.98 ms,
# profiles/r05/step_ab_row_ln_k2048.jsonl).
ROW_LN_MAX_K = 1024
# widest output the product runs on the row kernel: at d 512 (config 4) a 32-row tile streams the
# whole 512 x K weight per tile and the GEMM + LayerNorm launches are faster (whole large step
# 19.25 -> 18.95 ms with the row kernels off, profiles/r06/step_ab_row_ln_large.jsonl); the
# kernels still take D 512 (tests/test_row_ln_gpu.py)
ROW_LN_MAX_D = 256


def row_ln_ok(a, w, D, max_k=None, max_d=None):
    """Whether lasr_linear_res_ln / lasr_linear_dx_ln_bwd take a GEMM with A = a [M, K] and the
    D-wide output: bf16, D in (256, 512), K % 64 == 0, unit column strides, 16-B rows; and
    (the product policy) K <= max_k (default ROW_LN_MAX_K), D <= max_d (ROW_LN_MAX_D)."""
    Kd = a.shape[-1]
    return (a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and D in (256, 512)
            and D <= (ROW_LN_MAX_D if max_d is None else max_d) and a.dim() == 2
            and Kd % 64 == 0 and Kd <= (ROW_LN_MAX_K if max_k is None else max_k) and a.stride(1) == 1
            and a.stride(0) % 8 == 0 and w.is_contiguous() and _al16(a) and _al16(w))


def linear_res_ln(x, w, out, y1, mean1, rstd1, g1, b1, eps, *, bias=None, res, res_scale=1.0, drop_p=0.0,
                  drop_seed=0, g2=None, b2=None, y2=None, mean2=None, rstd2=None):
    """out = res + res_scale * dropout(x @ w^T + bias) (fp32), y1 = LN1(out), optionally
    y2 = LN2(y1): one launch (lasr_linear_res_ln), bit-identical to linear(..., res=...) +
    layernorm_fwd / layernorm2_fwd.  x [M, K] bf16, w [D, K]; [M, D] buffers contiguous."""
    M, Kd = x.shape
    D = w.shape[0]
    a = N.RowLnArgs()
    a.M, a.D, a.K = M, D, Kd
    a.A, a.lda, a.W, a.ldw = ptr(x), x.stride(0), ptr(w), w.stride(0)
    a.gamma1, a.beta1, a.eps, a.mean1, a.rstd1 = ptr(g1), ptr(b1), eps, ptr(mean1), ptr(rstd1)
    a.bias, a.res, a.res_scale, a.drop_p, a.drop_seed = ptr(bias), ptr(res), res_scale, drop_p, drop_seed
    a.out, a.y1, a.y1_dtype = ptr(out), ptr(y1), dt(y1)
    if g2 is not None:
        a.gamma2, a.beta2, a.y2, a.mean2, a.rstd2 = ptr(g2), ptr(b2), ptr(y2), ptr(mean2), ptr(rstd2)
    N.call("lasr_linear_res_ln", C.byref(a), stream())


def linear_dx_ln_bwd(dy, w, x, gamma, mean, rstd, dx, dgamma, dbeta, dres=None, gb=None, bscale=1.0, bp=0.0,
                     bseed=0):
    """dln = bf16(dy @ w) (dy [M, K] bf16, w [K, D]) and the LayerNorm backward of it in one
    launch (lasr_linear_dx_ln_bwd): bit-identical to gemm(dy, w, dln) + layernorm_bwd(x, dln,
    ...).  The dgamma / dbeta partials are reduced like layernorm_bwd's (deferred inside a
    deferred_reductions block)."""
    M, Kd = dy.shape
    D = w.shape[1]
    nblk = (M + 15) // 16
    defer = _DEFER.depth and dgamma is not None and dbeta is not None
    part = torch.empty(nblk * 2 * D, dtype=torch.float32, device=dy.device) if defer else \
        WS.get(nblk * 2 * D, dy.device)
    a = N.RowLnArgs()
    a.M, a.D, a.K = M, D, Kd
    a.A, a.lda, a.W, a.ldw = ptr(dy), dy.stride(0), ptr(w), w.stride(0)
    a.gamma1, a.mean1, a.rstd1 = ptr(gamma), ptr(mean), ptr(rstd)
    a.x, a.dres, a.dx, a.gb, a.bscale, a.bp, a.bseed = ptr(x), ptr(dres), ptr(dx), ptr(gb), bscale, bp, bseed
    a.part = ptr(part)
    if not defer:  # reduced in the same call, as layernorm_bwd's immediate path
        a.dgamma, a.dbeta = ptr(dgamma), ptr(dbeta)
    N.call("lasr_linear_dx_ln_bwd", C.byref(a), stream())
    if defer:
        _defer(part, nblk, 2 * D, dgamma, dbeta, split=D)


def branch_grad(dx, gb, scale, p=0.0, seed=0):
    N.call("lasr_branch_grad", ptr(dx), dt(dx), dx.numel(), ptr(gb), dt(gb), scale, p, seed,
           stream())


# ------------------------------------------------------------------------ CTC ---
def _rows_ld(x, lead):
    """Row stride of a logits view whose rows are (possibly padded) vocab vectors."""
    ld = x.stride(-2)
    assert x.stride(-1) == 1 and ld >= x.shape[-1], "logits rows must be unit-stride"
    for d in range(lead):
        assert x.stride(d) == ld * math.prod(x.shape[d + 1:-1]), "logits rows must be evenly spaced"
    return ld


def ctc_fwd(logits, targets, ilen, tlen, lse, lp, alpha, nll, beta=None):
    """beta given: the beta recursion runs in the forward launch too (then ctc_bwd with
    beta_ready=True)."""
    B, T, V = logits.shape
    Lmax = targets.shape[1]
    N.call("lasr_ctc_fwd", ptr(logits), dt(logits), B, T, V, _rows_ld(logits, 1), ptr(targets), Lmax,
           ptr(ilen), ptr(tlen), ptr(lse), ptr(lp), ptr(alpha), ptr(beta), ptr(nll), stream())


def ctc_bwd(logits, targets, ilen, tlen, lse, lp, alpha, nll, beta, grad, gscale, gdev=None,
            beta_ready=False):
    B, T, V = logits.shape
    Lmax = targets.shape[1]
    ld = _rows_ld(logits, 1)
    assert grad.shape == logits.shape and _rows_ld(grad, 1) == ld
    N.call("lasr_ctc_bwd", ptr(logits), dt(logits), B, T, V, ld, ptr(targets), Lmax, ptr(ilen),
           ptr(tlen), ptr(lse), ptr(lp), ptr(alpha), ptr(nll), ptr(beta), int(beta_ready), ptr(grad),
           dt(grad), gscale, ptr(gdev), stream())


def lsm_kl_fwd(logits, target, ignore, smoothing, lse, loss_rows):
    R, V = logits.shape
    N.call("lasr_lsm_kl_fwd", ptr(logits), dt(logits), R, V, _rows_ld(logits, 0), ptr(target), ignore,
           smoothing, ptr(lse), ptr(loss_rows), stream())


def lsm_kl_bwd(logits, target, ignore, smoothing, lse, grad, gscale, gdev=None):
    R, V = logits.shape
    ld = _rows_ld(logits, 0)
    assert grad.shape == logits.shape and _rows_ld(grad, 0) == ld
    N.call("lasr_lsm_kl_bwd", ptr(logits), dt(logits), R, V, ld, ptr(target), ignore, smoothing,
           ptr(lse), ptr(grad), dt(grad), gscale, ptr(gdev), stream())


def padded_rows(rows, V, dtype, device, align=8):
    """[rows, V] view of a [rows, roundup(V, align)] buffer (16-B aligned vocab rows)."""
    Vp = (V + align - 1) // align * align
    return torch.empty(rows, Vp, dtype=dtype, device=device)[:, :V]


def loss_combine(a, wa, b, wb, out):
    N.call("lasr_loss_combine", ptr(a), a.numel(), wa, ptr(b), b.numel() if b is not None else 0,
           wb, ptr(out), stream())


# ------------------------------------------------------------------ attention ---
def qbias_fwd(qkv, B, T, H, dk, bu, bv, qu, qv):
    N.call("lasr_qbias_fwd", ptr(qkv), dt(qkv), B, T, H, dk, qkv.stride(0), ptr(bu), ptr(bv),
           ptr(qu), ptr(qv), stream())


def qbias_bwd(dqu, dqv, B, T, H, dk, dqkv, du, dv):
    rows = B * T
    D = H * dk
    nchunk = (rows + 63) // 64  # QB_ROWS (attn.hip)
    if _DEFER.depth:
        ws = torch.empty(nchunk * 2 * D, dtype=torch.float32, device=dqu.device)
        N.call("lasr_qbias_bwd", ptr(dqu), ptr(dqv), dt(dqu), B, T, H, dk, ptr(dqkv), dqkv.stride(0),
               None, None, ptr(ws), ws.numel(), stream())
        _defer(ws, nchunk, 2 * D, du, dv, split=D)
        return
    ws = WS.get(nchunk * 2 * D, dqu.device)
    N.call("lasr_qbias_bwd", ptr(dqu), ptr(dqv), dt(dqu), B, T, H, dk, ptr(dqkv), dqkv.stride(0),
           ptr(du), ptr(dv), ptr(ws), ws.numel(), stream())


def attn_softmax_fwd(s_ac, s_bd, B, H, Tq, Tk, ldS, mask, msb, msq, P, drop_p=0.0, seed=0,
                     Praw=None):
    N.call("lasr_attn_softmax_fwd", ptr(s_ac), ptr(s_bd), int(s_bd is not None), B, H, Tq, Tk,
           ldS, ptr(mask), msb, msq, ptr(P), dt(P), drop_p, seed, ptr(Praw), stream())


def attn_softmax_bwd(P, dPd, B, H, Tq, Tk, ldS, mask, msb, msq, dS, drop_p=0.0, seed=0):
    N.call("lasr_attn_softmax_bwd", ptr(P), dt(P), ptr(dPd), B, H, Tq, Tk, ldS, ptr(mask), msb,
           msq, drop_p, seed, ptr(dS), dt(dS), stream())


def relshift_bwd(dS, Z, T, ldS, dBD):
    N.call("lasr_relshift_bwd", ptr(dS), dt(dS), Z, T, ldS, ptr(dBD), stream())


def pad_mask16(mask, B, Tq, Tk):
    """A query-dependent mask [B, Tq, Tk] (u8, any layout) as a view of a buffer whose rows are
    16-B aligned (the forward kernels stage its tiles by LDS-DMA): (view, msb, msq).  Padding
    columns are 1 (masked); the view is the same tensor when already aligned."""
    if mask.stride(-1) == 1 and mask.stride(-2) % 16 == 0 and mask.stride(0) % 16 == 0 and mask.data_ptr() % 16 == 0:
        return mask, mask.stride(0), mask.stride(-2)
    P = (Tk + 15) // 16 * 16
    buf = torch.ones(B, Tq, P, dtype=torch.uint8, device=mask.device)
    buf[:, :, :Tk] = mask
    v = buf[:, :, :Tk]
    return v, v.stride(0), v.stride(1)


def _fwd_mask(mask, msb, msq, B, Tq, Tk):
    """(mask, msb, msq) for the forward kernels: query-dependent masks re-laid out with 16-B
    aligned rows when they are not (callers that build masks per step pre-align them)."""
    if mask is None or msq == 0:
        return mask, msb, msq
    if msq % 16 == 0 and msb % 16 == 0 and mask.data_ptr() % 16 == 0:
        return mask, msb, msq
    # element (b, i, j) sits at data_ptr + b*msb + i*msq + j of the caller's storage (the kernels'
    # addressing): view that storage directly -- a reshape of a non-contiguous mask would copy it
    # and leave msb / msq describing the original
    m = torch.as_strided(mask, (B, Tq, Tk), (msb, msq, 1), mask.storage_offset())
    return pad_mask16(m, B, Tq, Tk)


def relattn_fwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx):
    """Fused rel-pos self-attention (bf16, d_k 32 or 64); 2-D row-major operands (row
    strides read from the tensors), stats [B*H*T*2] fp32 out, ctx [B*T, H*d_k] out."""
    mask, msb, msq = _fwd_mask(mask, msb, msq, B, T, T)
    N.call("lasr_relattn_fwd", ptr(qu), ptr(qv), qu.stride(0), ptr(k), ptr(v), k.stride(0), ptr(pos),
           pos.stride(0), B, H, T, qu.shape[1] // H, ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx),
           ctx.stride(0), stream())


def relattn_fwd_qb(q, bu, bv, qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx):
    """relattn_fwd with qbias_fwd folded in: q (the qkv projection's q slot) and the fp32
    pos_bias_u / v in; qu = q + u and qv = q + v are formed by the attention kernel and written
    to qu / qv (same strides) for the backward (lasr_relattn_fwd_qb)."""
    assert qv.stride(0) == qu.stride(0) and bu.dtype == torch.float32 and bv.dtype == torch.float32
    mask, msb, msq = _fwd_mask(mask, msb, msq, B, T, T)
    N.call("lasr_relattn_fwd_qb", ptr(q), q.stride(0), ptr(bu), ptr(bv), ptr(qu), ptr(qv), qu.stride(0), ptr(k),
           ptr(v), k.stride(0), ptr(pos), pos.stride(0), B, H, T, qu.shape[1] // H, ptr(mask), msb, msq, scale,
           ptr(stats), ptr(ctx), ctx.stride(0), stream())


def relattn_bwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dqu,
                dbd, ldS, dk, dv, dbd_head_major=False):
    assert qv.stride(0) == qu.stride(0) and dqu.stride(0) == qu.stride(0)
    assert v.stride(0) == k.stride(0) and dv.stride(0) == dk.stride(0) and dctx.stride(0) == ctx.stride(0)
    mask, msb, msq = _fwd_mask(mask, msb, msq, B, T, T)
    N.call("lasr_relattn_bwd", ptr(qu), ptr(qv), qu.stride(0), ptr(k), ptr(v), k.stride(0), ptr(pos),
           pos.stride(0), B, H, T, qu.shape[1] // H, ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx), ptr(dctx),
           ctx.stride(0), ptr(Dbuf), ptr(dqu), ptr(dbd), ldS, int(dbd_head_major), ptr(dk), ptr(dv), dk.stride(0),
           stream())


def attn_split(B, H, Tq, Tk, nsplit=None):
    """Key-split count of lasr_attn_fwd_split / _bwd_split for a shape (the library's
    heuristic unless given; 1 = the one-pass entries)."""
    ns = N.load().lasr_attn_split_count(B, H, Tq, Tk) if nsplit is None else int(nsplit)
    return ns


def attn_fwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, nsplit=None):
    """Plain attention on the fused kernels (lasr_attn_fwd): q [B*Tq, H*d_k], k / v
    [B*Tk, H*d_k] row-major views (k and v share a row stride), stats [B*H*Tq*2] fp32.
    Long key runs over few query blocks (the decoder's source attention at T' 999) split
    the keys over workgroups (lasr_attn_fwd_split; nsplit overrides the heuristic)."""
    assert v.stride(0) == k.stride(0)
    mask, msb, msq = _fwd_mask(mask, msb, msq, B, Tq, Tk)
    dk_ = q.shape[1] // H
    ns = attn_split(B, H, Tq, Tk, nsplit)
    if ns > 1:
        nw = N.load().lasr_attn_split_work(B, H, Tq, dk_, ns)
        ws = WS.get(nw, q.device)
        N.call("lasr_attn_fwd_split", ptr(q), q.stride(0), ptr(k), ptr(v), k.stride(0), B, H, Tq, Tk, dk_,
               ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx), ctx.stride(0), ns, ptr(ws), ws.numel(), stream())
        return
    N.call("lasr_attn_fwd", ptr(q), q.stride(0), ptr(k), ptr(v), k.stride(0), B, H, Tq, Tk, dk_,
           ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx), ctx.stride(0), stream())


def attn_bwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dq, dk, dv, nsplit=None):
    assert dq.stride(0) == q.stride(0) and v.stride(0) == k.stride(0) and dv.stride(0) == dk.stride(0)
    assert dctx.stride(0) == ctx.stride(0)
    mask, msb, msq = _fwd_mask(mask, msb, msq, B, Tq, Tk)
    dk_ = q.shape[1] // H
    ns = attn_split(B, H, Tq, Tk, nsplit)
    if ns > 1:
        nw = N.load().lasr_attn_split_work(B, H, Tq, dk_, ns)
        ws = WS.get(nw, q.device)
        N.call("lasr_attn_bwd_split", ptr(q), q.stride(0), ptr(k), ptr(v), k.stride(0), B, H, Tq, Tk, dk_,
               ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx), ptr(dctx), ctx.stride(0), ptr(Dbuf), ptr(dq),
               ptr(dk), ptr(dv), dk.stride(0), ns, ptr(ws), ws.numel(), stream())
        return
    N.call("lasr_attn_bwd", ptr(q), q.stride(0), ptr(k), ptr(v), k.stride(0), B, H, Tq, Tk, dk_,
           ptr(mask), msb, msq, scale, ptr(stats), ptr(ctx), ptr(dctx), ctx.stride(0), ptr(Dbuf), ptr(dq),
           ptr(dk), ptr(dv), dk.stride(0), stream())


def reduce_batch(src, B, H, T, dk, dst):
    N.call("lasr_reduce_batch", ptr(src), B, H, T, dk, ptr(dst), dt(dst), stream())


# ----------------------------------------------------------------------- conv ---
def conv1_fwd(x, w, bias, y1):
    B, T, F = x.shape
    Cc = w.shape[0]
    N.call("lasr_conv1_fwd", ptr(x), B, T, F, Cc, ptr(w), ptr(bias), ptr(y1), dt(y1), stream())


def conv1_bwd(x, dy1, dw, db):
    B, T, F = x.shape
    Cc = dw.shape[0]
    T1 = (T - 3) // 2 + 1
    nparts = (B * T1 + 7) // 8  # the partial rows of the smallest block lasr_conv1_bwd may use
    ws = WS.get((nparts + 1) * 10 * Cc, x.device)
    N.call("lasr_conv1_bwd", ptr(x), B, T, F, Cc, ptr(dy1), dt(dy1), ptr(dw), ptr(db), ptr(ws),
           ws.numel(), stream())


def im2col(y1, col):
    B, T1, F1, Cc = y1.shape
    N.call("lasr_im2col3x3s2", ptr(y1), dt(y1), B, T1, F1, Cc, ptr(col), stream())


def col2im(dcol, y1, dy1):
    B, T1, F1, Cc = y1.shape
    N.call("lasr_col2im3x3s2", ptr(dcol), dt(dcol), B, T1, F1, Cc, ptr(y1), ptr(dy1), stream())


def conv2_dy2_rows(M2):
    """Rows of the dy2 buffer lasr_conv2_gemm's backward modes need (rows M2.. zero)."""
    return ((M2 + 1 + 31) // 32) * 32


def _conv2(mode, y1, out, w2p=None, bias=None, dy2=None, rowsum=None, x=None, dw1=None, db1=None):
    B, T1, F1, Cc = y1.shape
    assert y1.dtype == torch.bfloat16 and y1.is_contiguous() and (out is None or out.is_contiguous())
    a = N.Conv2Args()
    a.mode, a.B, a.T1, a.F1, a.C = mode, B, T1, F1, Cc
    a.y1, a.out = ptr(y1), ptr(out)
    if w2p is not None:
        assert w2p.dtype == torch.bfloat16 and w2p.is_contiguous() and tuple(w2p.shape) == (Cc, 9 * Cc)
        a.w2p = ptr(w2p)
    if bias is not None:
        a.bias = ptr(bias)
    if dy2 is not None:
        assert dy2.dtype == torch.bfloat16 and dy2.is_contiguous() and dy2.shape[1] == Cc
        a.dy2, a.dy2_rows = ptr(dy2), dy2.shape[0]
    if rowsum is not None:
        assert rowsum.dtype == torch.float32 and rowsum.is_contiguous() and rowsum.numel() == Cc
        a.rowsum = ptr(rowsum)
    if mode == N.CONV2_DW:
        ws = WS.get(32 * (9 * Cc * Cc + Cc), y1.device)  # K slices: <= 32 (gemm_conv.hip caps to fit)
        a.workspace, a.workspace_bytes = ptr(ws), ws.numel() * 4
    if mode == N.CONV2_DX_W1:
        assert x.dtype == torch.float32 and x.is_contiguous() and x.shape[0] == B
        assert dw1.dtype == torch.float32 and dw1.is_contiguous() and tuple(dw1.shape) == (Cc, 9)
        assert db1.dtype == torch.float32 and db1.is_contiguous() and db1.numel() == Cc
        nbytes = N.load().lasr_conv2_dx_w1_workspace(B, T1, F1, Cc)
        ws = WS.get((nbytes + 3) // 4, y1.device)
        a.workspace, a.workspace_bytes = ptr(ws), ws.numel() * 4
        a.x, a.T, a.F = ptr(x), x.shape[1], x.shape[2]
        a.dw1, a.db1 = ptr(dw1), ptr(db1)
    N.call("lasr_conv2_gemm", C.byref(a), stream())


def conv2_fwd(y1, w2p, bias, y2):
    """y2 [B*T2*F2, C] = relu(conv3x3s2(y1) + bias), y1 channels-last [B, T1, F1, C] bf16."""
    _conv2(N.CONV2_FWD, y1, y2, w2p=w2p, bias=bias)


def conv2_dw(dy2, y1, dw, rowsum=None):
    """dw [C, 9C] fp32 = dy2^T im2col(y1) (dy2: conv2_dy2_rows(M2) rows, tail zero)."""
    _conv2(N.CONV2_DW, y1, dw, dy2=dy2, rowsum=rowsum)


def conv2_dx(dy2, w2p, y1, dy1):
    """dy1 [B, T1, F1, C] bf16 = col2im(dy2 w2p) * relu'(y1)."""
    _conv2(N.CONV2_DX, y1, dy1, w2p=w2p, dy2=dy2)


def conv2_dx_w1_ok(Cc):
    """lasr_conv2_gemm's LASR_CONV2_DX_W1 mode serves this channel count."""
    return Cc % 256 == 0


def conv2_dx_w1(dy2, w2p, y1, x, dw1, db1):
    """conv2_dx's dy1 consumed in place by conv1's weight gradient (dy1 never stored):
    dw1 [C, 9] += sum dy1 (x) patch3x3s2(x), db1 [C] += sum dy1; x [B, T, F] fp32."""
    _conv2(N.CONV2_DX_W1, y1, None, w2p=w2p, dy2=dy2, x=x, dw1=dw1, db1=db1)


def permute_last2(src, Nn, A, Bd, dst, reverse=False, accumulate=False):
    N.call("lasr_permute_last2", ptr(src), dt(src), Nn, A, Bd, ptr(dst), dt(dst), int(reverse),
           int(accumulate), stream())


def dwconv_nparts(B, T):
    return N.load().lasr_dwconv_nparts(B, T)


def glu_dwconv_fwd(z1, B, T, Cc, K, w, bias, y, stats):
    N.call("lasr_glu_dwconv_fwd", ptr(z1), dt(z1), B, T, Cc, K, ptr(w), ptr(bias), ptr(y), dt(y),
           ptr(stats), stream())


def bn_finalize(stats, nparts, Cc, eps, momentum, gamma, beta, rmean, rvar, nbt, mean, rstd,
                scale, shift, update):
    """update: 0 batch stats, 1 batch stats + running update (train), 2 eval (running stats)."""
    N.call("lasr_bn_finalize", ptr(stats), nparts, Cc, eps, momentum, ptr(gamma), ptr(beta),
           ptr(rmean), ptr(rvar), ptr(nbt), ptr(mean), ptr(rstd), ptr(scale), ptr(shift),
           int(update), stream())


def bn_act_fwd(y, scale, shift, h, act=N.ACT_SWISH):
    """h = act(y * scale + shift) (the conv module's BatchNorm + Swish / ReLU)."""
    rows, Cc = y.shape
    N.call("lasr_bn_act_fwd", ptr(y), dt(y), rows, Cc, ptr(scale), ptr(shift), ptr(h), dt(h), act, stream())


def bn_act_bwd(y, dh, scale, shift, mean, rstd, gamma, dgamma, dbeta, dy, batch_stats=True, act=N.ACT_SWISH):
    """batch_stats False: eval-mode BN (mean/rstd are the running statistics)."""
    rows, Cc = y.shape
    ws = WS.get(((rows + 63) // 64 + 1) * 2 * Cc, y.device)
    N.call("lasr_bn_act_bwd", ptr(y), dt(y), ptr(dh), dt(dh), rows, Cc, ptr(scale), ptr(shift),
           ptr(mean), ptr(rstd), ptr(gamma), ptr(dgamma), ptr(dbeta), ptr(dy), dt(dy), ptr(ws),
           ws.numel(), int(bool(batch_stats)), act, stream())


def glu_dwconv_bwd(z1, dy, B, T, Cc, K, w, dz1, dw, db):
    """dw [C, K] and db [C] accumulate; partials are [nparts][C*K + C] in their layout."""
    nparts = dwconv_nparts(B, T)
    if _DEFER.depth:
        ws = torch.empty(nparts * (K + 1) * Cc, dtype=torch.float32, device=z1.device)
        N.call("lasr_glu_dwconv_bwd", ptr(z1), dt(z1), ptr(dy), dt(dy), B, T, Cc, K, ptr(w), ptr(dz1),
               None, None, ptr(ws), ws.numel(), stream())
        _defer(ws, nparts, (K + 1) * Cc, dw, db, split=K * Cc)
        return
    ws = WS.get((nparts + 1) * (K + 1) * Cc, z1.device)
    N.call("lasr_glu_dwconv_bwd", ptr(z1), dt(z1), ptr(dy), dt(dy), B, T, Cc, K, ptr(w), ptr(dz1),
           ptr(dw), ptr(db), ptr(ws), ws.numel(), stream())


def bn_act_glu_dwconv_bwd(y, dh, scale, shift, mean, rstd, gamma, dgamma, dbeta, z1, B, T, Cc, K, w, dz1, dw, db,
                          batch_stats=True, act=N.ACT_SWISH):
    """bn_act_bwd + glu_dwconv_bwd in one call (lasr_bn_act_glu_dwconv_bwd): the BN backward's dy
    is computed inside the depthwise backward's window load, never stored.  Same outputs."""
    rows = y.shape[0]
    assert rows == B * T and y.shape[1] == Cc and dh.shape == y.shape and z1.shape == (rows, 2 * Cc)
    # (its own buffer: the depthwise partials below may take WS)
    bn_ws = torch.empty(((rows + 63) // 64 + 1) * 2 * Cc, dtype=torch.float32, device=y.device)
    nparts = dwconv_nparts(B, T)
    head = (ptr(y), dt(y), ptr(dh), dt(dh), B, T, Cc, ptr(scale), ptr(shift), ptr(mean), ptr(rstd), ptr(gamma),
            ptr(dgamma), ptr(dbeta), ptr(bn_ws), bn_ws.numel(), int(bool(batch_stats)), act, ptr(z1), dt(z1), K,
            ptr(w), ptr(dz1))
    if _DEFER.depth:
        ws = torch.empty(nparts * (K + 1) * Cc, dtype=torch.float32, device=z1.device)
        N.call("lasr_bn_act_glu_dwconv_bwd", *head, None, None, ptr(ws), ws.numel(), stream())
        _defer(ws, nparts, (K + 1) * Cc, dw, db, split=K * Cc)
        return
    ws = WS.get((nparts + 1) * (K + 1) * Cc, z1.device)
    N.call("lasr_bn_act_glu_dwconv_bwd", *head, ptr(dw), ptr(db), ptr(ws), ws.numel(), stream())


# ---------------------------------------------------------------- elementwise ---
def cast(src, dst):
    N.call("lasr_cast", ptr(src), dt(src), ptr(dst), dt(dst), src.numel(), stream())


def scale_add(a, b, sa, sb, out):
    N.call("lasr_scale_add", ptr(a), dt(a), ptr(b), dt(b) if b is not None else 0, sa, sb,
           ptr(out), dt(out), out.numel(), stream())


def pe_fwd(x, rows, T, D, pe, xscale, y, p=0.0, seed=0):
    N.call("lasr_pe_fwd", ptr(x), dt(x) if x is not None else 0, rows, T, D, ptr(pe), xscale, p,
           seed, ptr(y), dt(y), stream())


def embed_pe_fwd(ids, L, E, pe, xscale, y, p=0.0, seed=0):
    R = ids.numel()
    D = E.shape[1]
    N.call("lasr_embed_pe_fwd", ptr(ids), R, L, D, ptr(E), ptr(pe), xscale, p, seed, ptr(y),
           dt(y), stream())


def embed_bwd(ids, dy, xscale, dE, p=0.0, seed=0):
    R = ids.numel()
    D = dE.shape[1]
    N.call("lasr_embed_bwd", ptr(ids), R, D, ptr(dy), dt(dy), xscale, p, seed, ptr(dE), stream())


def fill(t, value):
    N.call("lasr_fill", ptr(t), dt(t), t.numel(), float(value), stream())


CHUNK_NONE, CHUNK_FIXED, CHUNK_DEVICE, CHUNK_SAMPLE = 0, 1, 2, 3


def u2_prep(xlens, ys, ylens, Tx, Tsub, sos, eos, chunk, out, chunk_mode=None, chunk_dev=None, ctr=None,
            chunk_seed=0, chunk_max=25):
    """One lasr_u2_prep_chunk launch: out["dec_mask"] [B, L+1, ld >= L+1] (the last dimension
    is the row stride; columns past L+1 come out 1 = masked), out["enc_mask"] [B, T'] (key
    padding), the targets and lengths, and -- unless chunk_mode is CHUNK_NONE -- the
    streaming chunk mask out["chunk_mask"] [B, T', ld >= T'] (padding columns masked).
    chunk_mode defaults to CHUNK_FIXED for chunk > 0, else CHUNK_NONE; CHUNK_DEVICE reads c
    from the int32 device scalar ``chunk_dev``, CHUNK_SAMPLE draws it from (chunk_seed, the
    uint64 step counter ``ctr``) and writes it to ``chunk_dev``; c <= 0 or c >= T' is full
    context."""
    B, L = ys.shape
    if chunk_mode is None:
        chunk_mode = CHUNK_FIXED if chunk > 0 else CHUNK_NONE
    dm, em = out["dec_mask"], out["enc_mask"]
    assert dm.is_contiguous() and dm.dim() == 3 and tuple(dm.shape[:2]) == (B, L + 1) and dm.shape[-1] >= L + 1
    assert em.is_contiguous() and em.dtype == torch.uint8 and em.numel() == B * Tsub
    cm, cld = None, 0
    if chunk_mode != CHUNK_NONE:
        cm = out["chunk_mask"]
        assert cm.is_contiguous() and cm.dim() == 3 and tuple(cm.shape[:2]) == (B, Tsub) and cm.shape[-1] >= Tsub
        cld = cm.shape[-1]
    if chunk_mode in (CHUNK_DEVICE, CHUNK_SAMPLE):
        assert chunk_dev is not None and chunk_dev.dtype == torch.int32 and chunk_dev.is_cuda
    if chunk_mode == CHUNK_SAMPLE:
        assert ctr is not None and ctr.dtype == torch.int64 and ctr.is_cuda
    for k, n in (("ys_in", B * (L + 1)), ("tgt", B * (L + 1)), ("tgt_ctc", B * L), ("pred_len", B), ("ylen", B)):
        assert out[k].dtype == torch.int32 and out[k].numel() == n and out[k].is_contiguous(), k
    N.call("lasr_u2_prep_chunk", ptr(xlens), ptr(ys), ptr(ylens), B, L, Tsub, sos, eos, chunk_mode,
           int(chunk) if chunk_mode == CHUNK_FIXED else 0, ptr(chunk_dev), ptr(ctr), int(chunk_seed), int(chunk_max),
           ptr(out["ys_in"]), ptr(out["tgt"]), ptr(out["tgt_ctc"]), ptr(dm), dm.shape[-1],
           ptr(em), ptr(cm), cld, ptr(out["pred_len"]), ptr(out["ylen"]), stream())


def spec_augment(x, xlens, plan, replace_with_zero=False, out=None):
    """Batched SpecAugment (csrc/specaug.hip) on a padded fp32 [B, T, F] device batch."""
    B, T, F = x.shape
    assert x.dtype == torch.float32 and x.is_contiguous()
    assert xlens.dtype == torch.int64 and xlens.numel() == B and xlens.device == x.device
    assert plan.dtype == torch.int32 and plan.dim() == 2 and plan.shape[0] == B and plan.is_contiguous()
    assert plan.device == x.device
    if out is None:
        out = torch.empty_like(x)
    assert out.shape == x.shape and out.dtype == torch.float32 and out.is_contiguous()
    nbytes = N.load().lasr_spec_augment_ws_bytes(B, T)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=x.device)
    N.call("lasr_spec_augment", ptr(x), ptr(out), ptr(xlens), ptr(plan), plan.shape[1], B, T, F,
           int(bool(replace_with_zero)), ptr(ws), nbytes, stream())
    return out


def sumsq_nparts(n):
    return N.load().lasr_sumsq_nparts(n)


def sumsq_partial(g, ws):
    N.call("lasr_sumsq_partial", ptr(g), g.numel(), ptr(ws), ws.numel(), stream())


def adam_step(param, param_lp, grad, m, v, ws, nparts, state, max_norm, lr_mode, lr, factor,
              model_dim, warmup, beta1, beta2, eps, weight_decay):
    N.call("lasr_adam_step", ptr(param), ptr(param_lp),
           dt(param_lp) if param_lp is not None else 0, ptr(grad), ptr(m), ptr(v), param.numel(),
           ptr(ws), nparts, ptr(state), max_norm, lr_mode, lr, factor, model_dim, warmup, beta1,
           beta2, eps, weight_decay, stream())


def set_dropout_counter(ctr):
    N.call("lasr_set_dropout_counter", ptr(ctr))


def counter_add(ctr, v=1):
    N.call("lasr_counter_add", ptr(ctr), int(v), stream())


def logsoftmax_topk(logits, k, rows=None, ld=None, gather_idx=None):
    """Per row of ``logits`` (2-D, unit column stride; ``rows``/``ld`` override the row
    count/stride to walk a strided subset): log_softmax, then the k largest log-probs
    (descending, ties to the smaller index) and/or log_softmax gathered at
    ``gather_idx[r]`` (int32, -inf outside [0,V)).  Returns (vals f32 [rows,k],
    idx i32 [rows,k], gathered f32 [rows] or None)."""
    if logits.dim() != 2 or logits.stride(1) != 1:
        raise ValueError("logsoftmax_topk: logits must be 2-D with unit column stride")
    rows = logits.shape[0] if rows is None else int(rows)
    ld = logits.stride(0) if ld is None else int(ld)
    V = logits.shape[1]
    dev = logits.device
    if (rows - 1) * ld + V > logits.untyped_storage().nbytes() // logits.element_size() - logits.storage_offset():
        raise ValueError("logsoftmax_topk: rows/ld walk past the logits storage")
    vals = torch.empty(rows, k, dtype=torch.float32, device=dev)
    idx = torch.empty(rows, k, dtype=torch.int32, device=dev)
    gat = None
    if gather_idx is not None:
        if gather_idx.dtype != torch.int32 or gather_idx.numel() != rows or not gather_idx.is_contiguous():
            raise ValueError("logsoftmax_topk: gather_idx must be contiguous int32 [rows]")
        gat = torch.empty(rows, dtype=torch.float32, device=dev)
    N.call("lasr_logsoftmax_topk", ptr(logits), dt(logits), rows, V, ld, k, ptr(gather_idx),
           ptr(vals) if k > 0 else None, ptr(idx) if k > 0 else None, ptr(gat), stream())
    return vals, idx, gat


# ------------------------------------------------------------ Paraformer CIF ---
def cif_fwd(z, plen, ylen, h, B, T, U, st):
    """Integrate-and-fire forward (lasr_cif_fwd); st: SimpleNamespace receiving alpha, acc,
    fired, row, sum_alpha, mae and out ([B, U, D] fp32)."""
    D = h.shape[-1]
    a = N.CifArgs()
    a.B, a.T, a.D, a.U = B, T, D, U
    a.z, a.plen, a.ylen, a.h = ptr(z), ptr(plen), ptr(ylen), ptr(h)
    a.alpha, a.acc, a.fired, a.row = ptr(st.alpha), ptr(st.acc), ptr(st.fired), ptr(st.row)
    a.sum_alpha, a.mae, a.out = ptr(st.sum_alpha), ptr(st.mae), ptr(st.out)
    N.call("lasr_cif_fwd", C.byref(a), stream())


def cif_bwd(plen, ylen, h, B, T, U, st, gout, gsum, dz, dh):
    D = h.shape[-1]
    a = N.CifArgs()
    a.B, a.T, a.D, a.U = B, T, D, U
    a.plen, a.ylen, a.h = ptr(plen), ptr(ylen), ptr(h)
    a.alpha, a.acc, a.fired, a.row, a.sum_alpha = ptr(st.alpha), ptr(st.acc), ptr(st.fired), ptr(st.row), \
        ptr(st.sum_alpha)
    a.gout, a.gsum, a.dz, a.dh = ptr(gout), ptr(gsum), ptr(dz), ptr(dh)
    N.call("lasr_cif_bwd", C.byref(a), stream())


def glancing_mix(replace, a, b, out, out2=None, backward=False):
    """fwd: out = replace ? a : b; bwd (a = incoming gradient): out / out2 = the
    embedding / CIF branch gradients.  fp32 [rows, D], replace u8 [rows]."""
    rows, D = out.shape
    N.call("lasr_glancing_mix", rows, D, ptr(replace), ptr(a), ptr(b), ptr(out), ptr(out2), int(backward),
           stream())


# ------------------------------------------------------------------ transducer ---
def rnnt_fwd(logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll):
    """RNN-T lattice forward (lasr_rnnt_fwd): logits [B, T, U1, V] (rows unit-stride, evenly
    spaced), targets int32 [B, Lmax >= U1-1], ilen / tlen int32 [B]."""
    B, T, U1, V = logits.shape
    N.call("lasr_rnnt_fwd", ptr(logits), dt(logits), B, T, U1, V, _rows_ld(logits, 3), ptr(targets), targets.shape[1],
           ptr(ilen), ptr(tlen), blank, ptr(lse), ptr(lp), ptr(alpha), ptr(beta), ptr(nll), stream())


def rnnt_bwd(logits, targets, ilen, tlen, blank, lse, lp, alpha, beta, nll, grad, gscale, gdev=None):
    B, T, U1, V = logits.shape
    ld = _rows_ld(logits, 3)
    assert grad.shape == logits.shape and _rows_ld(grad, 3) == ld
    N.call("lasr_rnnt_bwd", ptr(logits), dt(logits), B, T, U1, V, ld, ptr(targets), targets.shape[1], ptr(ilen),
           ptr(tlen), blank, ptr(lse), ptr(lp), ptr(alpha), ptr(beta), ptr(nll), ptr(grad), dt(grad), gscale,
           ptr(gdev), stream())


def joint_fwd(e, d, B, T, U1, z):
    """z[(b T + t) U1 + u] = tanh(e[b T + t] + d[u B + b]) (lasr_joint_fwd); e, d fp32."""
    J = e.shape[1]
    assert e.is_contiguous() and d.is_contiguous() and z.is_contiguous() and e.dtype == d.dtype == torch.float32
    N.call("lasr_joint_fwd", ptr(e), ptr(d), B, T, U1, J, ptr(z), dt(z), stream())


def joint_reduce(dz, B, T, U1, de, dd):
    J = dz.shape[1]
    assert dz.is_contiguous() and de.is_contiguous() and dd.is_contiguous() and de.dtype == dd.dtype
    N.call("lasr_joint_reduce", ptr(dz), dt(dz), B, T, U1, J, ptr(de), ptr(dd), dt(de), stream())


def lstm_cell_fwd(gates, bias, c_prev, c_out, h_out):
    """gates [B, >=4H] fp32 (row stride any), h_out [B, H] (row stride any)."""
    B, H = c_out.shape
    N.call("lasr_lstm_cell_fwd", ptr(gates), gates.stride(0), ptr(bias), ptr(c_prev), B, H, ptr(c_out), ptr(h_out),
           dt(h_out), h_out.stride(0), stream())


def lstm_cell_bwd(gates, bias, c, c_prev, dh_out, dh_rec, dc_next, dgates, dc_prev):
    B, H = c.shape
    N.call("lasr_lstm_cell_bwd", ptr(gates), gates.stride(0), ptr(bias), ptr(c), ptr(c_prev), ptr(dh_out),
           dt(dh_out) if dh_out is not None else 0, dh_out.stride(0) if dh_out is not None else 0, ptr(dh_rec),
           ptr(dc_next), B, H, ptr(dgates), dt(dgates), dgates.stride(0), ptr(dc_prev), stream())
