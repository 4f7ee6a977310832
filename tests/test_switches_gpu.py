"""Every A/B switch that survives in the product is a fusion or restructuring claimed to give
the SAME bits as the path it replaced; here each is pinned at model level: one bf16 training
step of config 2's full model (12 / 6 layers, B 2 x T 1000, dropout 0.1) with the switch off
must equal the default step -- loss, the whole flat gradient and the BN running statistics,
``torch.equal``.  The node tests (tests/test_nodes_gpu.py) switch these fusions off to feed
nodes standalone, so this is what ties the shipped wiring to them.

Each step runs in its own process (the switches are read once, at import or library load);
the parent never touches the GPU.

  LASR_ROW_LN          residual projections / first-projection input gradients with the
                       LayerNorm in the GEMM epilogue (csrc/gemm_row.hip) vs GEMM + norm
  LASR_DEC_ROW_LN      the same for the decoder's attention projections
  LASR_FUSED_LN2       a layer's final norm and the next layer's first norm in one launch
  LASR_BATCH_POS_PROJ  the 12 positional projections as one strided batched GEMM
  LASR_EPI_SPEC        compile-time epilogue instances vs the runtime-branch epilogue
  LASR_DW_SLICE_XCD    grouped dW K slices tied to XCDs vs the plain block order
  LASR_CTC_REGS        the CTC lattice in registers (DPP neighbour reads, one barrier per 8
                       steps) vs one state per thread with a barrier per step"""

import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SWITCHES = ["LASR_ROW_LN", "LASR_DEC_ROW_LN", "LASR_FUSED_LN2", "LASR_BATCH_POS_PROJ", "LASR_EPI_SPEC",
            "LASR_DW_SLICE_XCD", "LASR_CTC_REGS"]


def _step(tmp_path, name, env_extra):
    out = str(tmp_path / f"{name}.pt")
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_switch_step.py"), out], env=env,
                       capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, (name, r.stdout[-2000:], r.stderr[-4000:])
    return torch.load(out, weights_only=True)


@pytest.fixture(scope="module")
def baseline(tmp_path_factory):
    return _step(tmp_path_factory.mktemp("sw"), "default", {k: "1" for k in SWITCHES})


@pytest.mark.parametrize("switch", SWITCHES)
def test_switch_off_is_bit_identical(switch, baseline, tmp_path):
    other = _step(tmp_path, switch, {**{k: "1" for k in SWITCHES}, switch: "0"})
    assert torch.equal(other["loss"], baseline["loss"]), (switch, other["loss"], baseline["loss"])
    g0, g1 = baseline["grad"], other["grad"]
    if not torch.equal(g0, g1):
        diff = (g0 - g1).abs()
        raise AssertionError(f"{switch}=0 changes the gradient: {int((diff > 0).sum())} elements, "
                             f"max {diff.max().item():.3e} (grad max {g0.abs().max().item():.3e})")
    for a, b in zip(baseline["bn"], other["bn"]):
        assert torch.equal(a, b), switch
