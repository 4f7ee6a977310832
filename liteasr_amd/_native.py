"""ctypes binding of libliteasr_hip.so (C ABI declared in include/liteasr_hip.h).

The library is the product path: there is no fallback.  If it cannot be loaded the
import of any op raises, loudly.  Build it with ``make`` (or ``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libliteasr_hip.so")  # the one product path (A/B tools:
# tools/with_lib.py points this module at another build before anything loads it)

F32, BF16, I32, I64, U8 = 0, 1, 2, 3, 4
ACT_NONE, ACT_RELU, ACT_SWISH, ACT_GATE, ACT_TANH = 0, 1, 2, 3, 4

_p = C.c_void_p
_i = C.c_int
_l = C.c_int64
_f = C.c_float
_u = C.c_uint64


class GemmArgs(C.Structure):
    """Mirror of ``lasr_gemm_args``."""

    _fields_ = [
        ("M", _i), ("N", _i), ("K", _i),
        ("batch", _i), ("batch_div", _i),
        ("A", _p), ("lda_m", _l), ("lda_k", _l), ("sa1", _l), ("sa2", _l),
        ("B", _p), ("ldb_n", _l), ("ldb_k", _l), ("sb1", _l), ("sb2", _l),
        ("C", _p), ("ldc", _l), ("sc1", _l), ("sc2", _l),
        ("in_dtype", _i), ("c_dtype", _i),
        ("alpha", _f), ("alpha_dev", _p),
        ("beta", _f),
        ("bias", _p),
        ("act", _i),
        ("zout", _p),
        ("aux", _p), ("aux_dtype", _i), ("ldaux", _l), ("aux_act", _i),
        ("drop_p", _f), ("drop_seed", _u),
        ("res", _p), ("res_dtype", _i), ("ldres", _l), ("res_scale", _f),
        ("split_k", _i), ("workspace", _p), ("workspace_bytes", _l),
        ("rowsum", _p),
        ("zout_mode", _i),
        ("tile_m", _i), ("tile_n", _i), ("ksub", _i),
    ]


class Conv2Args(C.Structure):
    """Mirror of ``lasr_conv2_args``."""

    _fields_ = [
        ("mode", _i),
        ("B", _i), ("T1", _i), ("F1", _i), ("C", _i),
        ("y1", _p), ("w2p", _p), ("bias", _p),
        ("dy2", _p), ("dy2_rows", _l),
        ("out", _p), ("rowsum", _p),
        ("workspace", _p), ("workspace_bytes", _l),
        ("x", _p), ("T", _i), ("F", _i),
        ("dw1", _p), ("db1", _p),
    ]


CONV2_FWD, CONV2_DW, CONV2_DX, CONV2_DX_W1 = 0, 1, 2, 3


class CifArgs(C.Structure):
    """Mirror of ``lasr_cif_args``."""

    _fields_ = [
        ("B", _i), ("T", _i), ("D", _i), ("U", _i),
        ("z", _p), ("plen", _p), ("ylen", _p), ("h", _p),
        ("alpha", _p), ("acc", _p), ("fired", _p), ("row", _p), ("sum_alpha", _p), ("mae", _p), ("out", _p),
        ("gout", _p), ("gsum", _p), ("dz", _p), ("dh", _p),
    ]


class RowLnArgs(C.Structure):
    """Mirror of ``lasr_row_ln_args``."""

    _fields_ = [
        ("M", _i), ("D", _i), ("K", _i),
        ("A", _p), ("lda", _l), ("W", _p), ("ldw", _l),
        ("gamma1", _p), ("beta1", _p), ("eps", _f), ("mean1", _p), ("rstd1", _p),
        ("bias", _p), ("res", _p), ("res_scale", _f), ("drop_p", _f), ("drop_seed", _u),
        ("out", _p), ("y1", _p), ("y1_dtype", _i),
        ("gamma2", _p), ("beta2", _p), ("y2", _p), ("mean2", _p), ("rstd2", _p),
        ("x", _p), ("dres", _p), ("dx", _p), ("gb", _p), ("bscale", _f), ("bp", _f), ("bseed", _u),
        ("part", _p), ("dgamma", _p), ("dbeta", _p),
    ]


class ReduceSeg(C.Structure):
    """Mirror of ``lasr_reduce_seg``."""

    _fields_ = [("part", _p), ("N", _l), ("P", _i), ("accumulate", _i), ("out0", _p), ("out1", _p),
                ("split", _l)]


# name -> argtypes (all return int unless listed in _RESTYPES)
SIGNATURES = {
    "lasr_version": [],
    "lasr_last_error": [],
    "lasr_set_dropout_counter": [_p],
    "lasr_counter_add": [_p, _u, _p],
    "lasr_gemm": [C.POINTER(GemmArgs), _p],
    "lasr_gemm_plan": [C.POINTER(GemmArgs), _p, _p, _p, _p],
    "lasr_gemm_dw_group": [C.POINTER(GemmArgs), _i, _p],
    "lasr_gemm_dw_group_order": [_i],
    "lasr_gemm_narrow_tiles": [_i],
    "lasr_relattn_fwd": [_p, _p, _l, _p, _p, _l, _p, _l, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _l, _p],
    "lasr_relattn_fwd_qb": [_p, _l, _p, _p, _p, _p, _l, _p, _p, _l, _p, _l, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p,
                            _l, _p],
    "lasr_attn_fwd": [_p, _l, _p, _p, _l, _i, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _l, _p],
    "lasr_attn_bwd": [_p, _l, _p, _p, _l, _i, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _p, _l, _p, _p, _p, _p,
                      _l, _p],
    "lasr_attn_fwd_split": [_p, _l, _p, _p, _l, _i, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _l, _i, _p, _l, _p],
    "lasr_attn_bwd_split": [_p, _l, _p, _p, _l, _i, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _p, _l, _p, _p, _p,
                            _p, _l, _i, _p, _l, _p],
    "lasr_attn_split_work": [_i, _i, _i, _i, _i],
    "lasr_attn_split_count": [_i, _i, _i, _i],
    "lasr_relattn_bwd": [_p, _p, _l, _p, _p, _l, _p, _l, _i, _i, _i, _i, _p, _l, _l, _f, _p, _p, _p, _l,
                         _p, _p, _p, _i, _i, _p, _p, _l, _p],
    "lasr_reduce_multi": [C.POINTER(ReduceSeg), _i, _p],
    "lasr_linear_res_ln": [C.POINTER(RowLnArgs), _p],
    "lasr_linear_dx_ln_bwd": [C.POINTER(RowLnArgs), _p],
    "lasr_dropout_scale": [_f],
    "lasr_colsum": [_p, _i, _l, _l, _l, _p, _i, _p, _l, _p],
    "lasr_layernorm2_fwd": [_p, _l, _i, _p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _p, _p],
    "lasr_layernorm_fwd": [_p, _i, _l, _i, _p, _p, _f, _p, _i, _p, _p, _p, _i, _f, _u, _p],
    "lasr_layernorm_bwd": [_p, _i, _p, _i, _l, _i, _p, _p, _p, _p, _i, _p, _i, _p, _p, _p, _l,
                           _p, _i, _f, _f, _u, _p],
    "lasr_layernorm2_bwd": [_p, _p, _i, _p, _l, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _f, _f, _u,
                            _p],
    "lasr_branch_grad": [_p, _i, _l, _p, _i, _f, _f, _u, _p],
    "lasr_ctc_fwd": [_p, _i, _i, _i, _i, _l, _p, _i, _p, _p, _p, _p, _p, _p, _p, _p],
    "lasr_ctc_lattice": [_i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p],
    "lasr_rnnt_fwd": [_p, _i, _i, _i, _i, _i, _l, _p, _i, _p, _p, _i, _p, _p, _p, _p, _p, _p],
    "lasr_rnnt_bwd": [_p, _i, _i, _i, _i, _i, _l, _p, _i, _p, _p, _i, _p, _p, _p, _p, _p, _p, _i, _f, _p, _p],
    "lasr_joint_fwd": [_p, _p, _i, _i, _i, _i, _p, _i, _p],
    "lasr_joint_reduce": [_p, _i, _i, _i, _i, _i, _p, _p, _i, _p],
    "lasr_lstm_cell_fwd": [_p, _l, _p, _p, _i, _i, _p, _p, _i, _l, _p],
    "lasr_lstm_cell_bwd": [_p, _l, _p, _p, _p, _p, _i, _l, _p, _p, _i, _i, _p, _i, _l, _p, _p],
    "lasr_ctc_bwd": [_p, _i, _i, _i, _i, _l, _p, _i, _p, _p, _p, _p, _p, _p, _p, _i, _p, _i, _f, _p, _p],
    "lasr_lsm_kl_fwd": [_p, _i, _i, _i, _l, _p, _i, _f, _p, _p, _p],
    "lasr_lsm_kl_bwd": [_p, _i, _i, _i, _l, _p, _i, _f, _p, _p, _i, _f, _p, _p],
    "lasr_loss_combine": [_p, _i, _f, _p, _i, _f, _p, _p],
    "lasr_qbias_fwd": [_p, _i, _i, _i, _i, _i, _l, _p, _p, _p, _p, _p],
    "lasr_qbias_bwd": [_p, _p, _i, _i, _i, _i, _i, _p, _l, _p, _p, _p, _l, _p],
    "lasr_attn_softmax_fwd": [_p, _p, _i, _i, _i, _i, _i, _i, _p, _l, _l, _p, _i, _f, _u, _p, _p],
    "lasr_attn_softmax_bwd": [_p, _i, _p, _i, _i, _i, _i, _i, _p, _l, _l, _f, _u, _p, _i, _p],
    "lasr_relshift_bwd": [_p, _i, _i, _i, _i, _p, _p],
    "lasr_reduce_batch": [_p, _i, _i, _i, _i, _p, _i, _p],
    "lasr_conv1_fwd": [_p, _i, _i, _i, _i, _p, _p, _p, _i, _p],
    "lasr_conv1_bwd": [_p, _i, _i, _i, _i, _p, _i, _p, _p, _p, _l, _p],
    "lasr_conv2_gemm": [C.POINTER(Conv2Args), _p],
    "lasr_conv2_dx_w1_workspace": [_i, _i, _i, _i],
    "lasr_cif_fwd": [C.POINTER(CifArgs), _p],
    "lasr_cif_bwd": [C.POINTER(CifArgs), _p],
    "lasr_glancing_mix": [_l, _i, _p, _p, _p, _p, _p, _i, _p],
    "lasr_im2col3x3s2": [_p, _i, _i, _i, _i, _i, _p, _p],
    "lasr_col2im3x3s2": [_p, _i, _i, _i, _i, _i, _p, _p, _p],
    "lasr_permute_last2": [_p, _i, _l, _l, _l, _p, _i, _i, _i, _p],
    "lasr_glu_dwconv_fwd": [_p, _i, _i, _i, _i, _i, _p, _p, _p, _i, _p, _p],
    "lasr_dwconv_nparts": [_i, _i],
    "lasr_bn_finalize": [_p, _i, _i, _f, _f, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p],
    "lasr_bn_act_fwd": [_p, _i, _l, _i, _p, _p, _p, _i, _i, _p],
    "lasr_bn_act_bwd": [_p, _i, _p, _i, _l, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _l, _i, _i, _p],
    "lasr_glu_dwconv_bwd": [_p, _i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _l, _p],
    "lasr_bn_act_glu_dwconv_bwd": [_p, _i, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _l, _i, _i,
                                   _p, _i, _i, _p, _p, _p, _p, _p, _l, _p],
    "lasr_cast": [_p, _i, _p, _i, _l, _p],
    "lasr_scale_add": [_p, _i, _p, _i, _f, _f, _p, _i, _l, _p],
    "lasr_embed_pe_fwd": [_p, _i, _i, _i, _p, _p, _f, _f, _u, _p, _i, _p],
    "lasr_embed_bwd": [_p, _i, _i, _p, _i, _f, _f, _u, _p, _p],
    "lasr_pe_fwd": [_p, _i, _l, _i, _i, _p, _f, _f, _u, _p, _i, _p],
    "lasr_u2_prep": [_p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p],
    "lasr_u2_prep_ld": [_p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _i, _p, _p, _p],
    "lasr_gemm_qbias_bwd": [C.POINTER(GemmArgs), _p, _p, _i, _i, _i, _i, _i, _p, _l, _p, _l, _p],
    "lasr_gemm_ln_fwd": [C.POINTER(GemmArgs), _p, _p, _f, _p, _i, _p, _p, _p],
    "lasr_gemm_ln_bwd": [C.POINTER(GemmArgs), _p, _i, _p, _p, _p, _p, _i, _p, _i, _p, _l, _p, _i, _f, _f, _u, _p],
    "lasr_u2_prep_chunk": [_p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _u, _i,
                           _p, _p, _p, _p, _i, _p, _p, _i, _p, _p, _p],
    "lasr_sumsq_nparts": [_l],
    "lasr_sumsq_partial": [_p, _l, _p, _l, _p],
    "lasr_adam_step": [_p, _p, _i, _p, _p, _p, _l, _p, _i, _p, _f, _i, _f, _f, _f, _f, _f, _f,
                       _f, _f, _p],
    "lasr_fill": [_p, _i, _l, _f, _p],
    "lasr_spec_augment": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _l, _p],
    "lasr_spec_augment_ws_bytes": [_i, _i],
    "lasr_logsoftmax_topk": [_p, _i, _l, _i, _l, _i, _p, _p, _p, _p, _p],
}
_RESTYPES = {"lasr_last_error": C.c_char_p, "lasr_spec_augment_ws_bytes": C.c_int64,
             "lasr_conv2_dx_w1_workspace": C.c_int64, "lasr_attn_split_work": C.c_int64,
             "lasr_dropout_scale": C.c_float}


class NativeError(RuntimeError):
    pass


_lib = None


def load():
    """Load (once) and return the native library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"libliteasr_hip.so not found at {LIB_PATH}; build it with `make` "
            "(the HIP path has no fallback)"
        )
    lib = C.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, C.c_int)
    _lib = lib
    return lib


def call(name, *args):
    """Call ``name`` and raise NativeError on a non-zero status."""
    lib = _lib if _lib is not None else load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.lasr_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed ({rc}): {msg}")
    return rc


def exported_symbols():
    """Names of all lasr_* functions bound here."""
    return sorted(SIGNATURES)
