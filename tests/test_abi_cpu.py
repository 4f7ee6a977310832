"""C-ABI boundary checks that need no GPU: the HIP library loads, exports every function
``include/liteasr_hip.h`` declares, the ctypes signature table binds exactly that set, and
the pure host entries (version, error string, size helpers) answer.  No compute call is
made here; the compute entries are exercised in the ``-m gpu`` parity tests."""

import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HEADER = os.path.join(ROOT, "include", "liteasr_hip.h")
LIB = os.path.join(ROOT, "liteasr_amd", "lib", "libliteasr_hip.so")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(lasr_[a-z0-9_]+)\s*\(", src)))


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", ROOT, "-j8"], check=True, capture_output=True)
    return LIB


def test_header_symbols_exported(lib):
    decl = _declared()
    assert len(decl) >= 40
    missing = [s for s in decl if s not in _exported()]
    assert not missing, f"declared in liteasr_hip.h but not exported: {missing}"


def test_ctypes_table_matches_header(lib):
    from liteasr_amd import _native

    assert sorted(_native.SIGNATURES) == _declared()


def test_host_entries_without_gpu(lib):
    from liteasr_amd import _native

    L = _native.load()
    assert L.lasr_version() > 0
    assert isinstance(L.lasr_last_error(), (bytes, type(None)))
    assert L.lasr_sumsq_nparts(1 << 20) >= 1
    assert L.lasr_dwconv_nparts(4, 200) >= 1
    # dropout: 16-bit threshold round(p * 65536), kept values scaled to keep E = 1 exactly
    for p in (0.1, 0.25, 0.5):
        thr = int(p * 65536 + 0.5)
        assert abs(L.lasr_dropout_scale(p) - 65536 / (65536 - thr)) <= 1e-6
    assert L.lasr_dropout_scale(0.0) == 1.0 and L.lasr_dropout_scale(1.0) == 0.0
    # conv2 DX_W1 workspace: one [10][C] fp32 partial row per 128-row tile of the four output
    # parity classes, their 64-row group sums and the total
    for B, T1, F1, C in ((32, 499, 39, 256), (2, 20, 39, 512), (3, 32, 18, 256)):
        P = sum(-(-(B * ((T1 - pt + 1) >> 1) * ((F1 - pf + 1) >> 1)) // 128) for pt in (0, 1) for pf in (0, 1))
        assert L.lasr_conv2_dx_w1_workspace(B, T1, F1, C) == (P + -(-P // 64) + 1) * 10 * C * 4
    assert L.lasr_conv2_dx_w1_workspace(0, 20, 39, 256) == 0


def test_extern_c_no_mangling(lib):
    """Every lasr_* export is an unmangled C symbol (cgo/JNI/ctypes bindable)."""
    ex = _exported()
    assert not [s for s in ex if s.startswith("_Z") and "lasr_" in s and s.startswith("_Zlasr")]
    assert all(s in ex for s in _declared())


def test_product_path_refuses_cpu():
    """No CPU fallback: the model raises on a CPU batch instead of computing."""
    import torch
    from liteasr_amd.models.u2 import U2, U2Config
    from liteasr_amd.utils.cfg import resolve_self

    c = U2Config(input_dim=40, vocab_size=20, enc_dim=32, enc_ff_dim=64, enc_attn_heads=4, enc_layers=1,
                 dec_dim=32, dec_ff_dim=64, dec_attn_heads=4, dec_layers=1)
    resolve_self(c)
    m = U2(c)
    xs = torch.zeros(1, 40, 40)
    with pytest.raises(RuntimeError, match="HIP device only"):
        m(xs, torch.tensor([40]), torch.ones(1, 3, dtype=torch.long), torch.tensor([3]))


def test_decode_header_symbols_exported():
    """include/liteasr_decode.h <-> libliteasr_decode.so (host-only decoding library)."""
    hdr = os.path.join(ROOT, "include", "liteasr_decode.h")
    so = os.path.join(ROOT, "liteasr_amd", "lib", "libliteasr_decode.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", ROOT, so], check=True, capture_output=True)
    src = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    declared = set(re.findall(r"\b(lasr_[a-z0-9_]+)\s*\(", src))
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared == {"lasr_ctc_prefix_beam_search", "lasr_decode_last_error"}
    assert declared <= exported


def test_comm_header_symbols_exported():
    """include/liteasr_comm.h <-> libliteasr_comm.so (native bucketed reducer over RCCL) <->
    the ctypes signature table; only the pure host size query is called (no GPU here)."""
    hdr = os.path.join(ROOT, "include", "liteasr_comm.h")
    so = os.path.join(ROOT, "liteasr_amd", "lib", "libliteasr_comm.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", ROOT, so], check=True, capture_output=True)
    src = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    declared = set(re.findall(r"\b(lasr_[a-z0-9_]+)\s*\(", src))
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared <= exported, declared - exported
    from liteasr_amd.distributed import native_reducer as NR

    assert set(NR._SIGS) == declared
    L = NR.load()
    assert L.lasr_reducer_uid_bytes() == 128  # NCCL_UNIQUE_ID_BYTES


def test_switch_names_are_every_product_switch():
    """The getenv switches in csrc/ and the LASR_* environment reads in liteasr_amd/ are exactly
    the ones tested here (plus LASR_ROCTX, the tracing flag, and the decoder attention switch
    held to the materialised path in test_kernels_gpu.py)."""
    import re

    from test_switches_gpu import SWITCHES

    found = set()
    for base, _, files in os.walk(os.path.join(ROOT, "liteasr_amd")):
        for f in files:
            if f.endswith((".hip", ".h", ".cpp", ".py")):
                src = open(os.path.join(base, f)).read()
                found |= set(re.findall(r'getenv\("(LASR_[A-Z0-9_]+)"', src))
                found |= set(re.findall(r'environ\.get\("(LASR_[A-Z0-9_]+)"', src))
    assert found == set(SWITCHES) | {"LASR_ROCTX", "LASR_FUSED_DEC_ATTN"}, found
