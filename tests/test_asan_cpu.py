"""Host AddressSanitizer + UBSan run over the host-only native code (no GPU): the Kaldi ark
reader (csrc/io/ark_io.cpp) and the CTC prefix beam search (csrc/decode/prefix_beam.cpp),
compiled from their sources with -fsanitize=address,undefined next to the driver
tools/asan/host_check.cpp (every object kind read back, row limits and padded strides, the
threaded padded collator, every truncation and random byte mutations of each object, beam
search over ragged shapes and too-small token caps). Any sanitizer report or failed check
fails the test. The HIP library's host code is covered by the ABI tests and the GPU suite;
GPU-side sanitizers are not available on the GPU pool."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_libraries_under_asan_ubsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "asan"), "run"], env=env,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host sanitizer checks: clean" in out, out[-2000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
