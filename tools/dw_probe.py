"""Kernel-trace probe of the dW GEMMs (run under rocprofv3): each shape at the planner's
choice and at a given forced tile/split, 50 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from liteasr_amd import _native as N  # noqa: E402
from liteasr_amd import kernels as K  # noqa: E402
from tools.gemm_graph_bench import make  # noqa: E402
from tools.dw_sweep import SHAPES  # noqa: E402

N.load()
for name, M, N_, Kd in SHAPES:
    a, b, c, extra = make(M, N_, Kd, "tn", torch.float32, 1, split=1)
    for tm, tn, sp in [(0, 0, 0), (64, 64, 16), (64, 64, 8), (64, 128, 8), (64, 64, 4)]:
        N.call("lasr_gemm_force_tile", tm, tn)
        N.call("lasr_gemm_force_split", sp, 0)
        for _ in range(50):
            K.gemm(a, b, c, **extra)
        torch.cuda.synchronize()
N.call("lasr_gemm_force_tile", 0, 0)
N.call("lasr_gemm_force_split", 0, 0)
