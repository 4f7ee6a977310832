"""Times lasr_adam_step (the finalize launch + the Adam launch) over flat buffers of the small
config's parameter count and prints a hash of the updated parameters, momenta and bf16 copy
after a fixed number of steps, so that library builds (LITEASR_HIP_LIB) compare bit for bit."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 46_200_001  # ragged: exercises the scalar tail
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev).manual_seed(5)
p = torch.randn(n, device=dev, generator=gen)
g = torch.randn(n, device=dev, generator=gen) * 1e-2
m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
plp = torch.empty(n, dtype=torch.bfloat16, device=dev)
nparts = K.sumsq_nparts(n)
ws = torch.empty(nparts, device=dev)
state = torch.zeros(8, device=dev)


def step():
    K.sumsq_partial(g, ws)
    K.adam_step(p, plp, g, m, v, ws, nparts, state, 5.0, 1, 0.0, 5.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)


for _ in range(3):
    step()
torch.cuda.synchronize()
h = hashlib.sha256()
for t in (p, m, v, plp.view(torch.int16)):
    h.update(t.cpu().numpy().tobytes())
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = []
for rep in range(3):
    e0.record(s)
    for _ in range(20):
        K.adam_step(p, plp, g, m, v, ws, nparts, state, 5.0, 1, 0.0, 5.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)
    e1.record(s)
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) * 1e3 / 20)
res2 = []
for rep in range(3):
    e0.record(s)
    for _ in range(20):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    res2.append(e0.elapsed_time(e1) * 1e3 / 20)
print(json.dumps({"n": n, "adam_step_us": [round(x, 1) for x in res], "min_us": round(min(res), 1),
                  "sumsq_adam_us": round(min(res2), 1),
                  "GB_s": round(30.0 * n / min(res) / 1e3, 1), "hash": h.hexdigest()[:16]}), flush=True)
