"""Times the three CTC kernels (row lse + gather, alpha/beta lattice, gradient) at the small
and long configs through bench.ctc_roofline; one JSON line per config.  LITEASR_HIP_LIB
selects the library (ablation builds from tools/gemm_exp.sh with EXP_FILES=ctc)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for name in (sys.argv[1:] or ["small", "long"]):
    r = bench.ctc_roofline(bench.CONFIGS[name], dev, iters=50)
    print(json.dumps({"cfg": name, "gather_us": r["gather_us"], "lattice_us": r["lattice_us"],
                      "grad_us": r["grad_us"]}), flush=True)
