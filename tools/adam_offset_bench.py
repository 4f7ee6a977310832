"""Adam (lasr_adam_step) over flat buffers whose bases are 2 MB-aligned (as the caching allocator
hands out large blocks) vs the same buffers at staggered offsets: whether the five concurrent
streams of the update (grad, param, m, v read; param, m, v, bf16 copy written) camp on the same
HBM channels.  One JSON line per (n, layout)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from liteasr_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")


def run(n, offs):
    gen = torch.Generator(device=dev).manual_seed(5)
    pad = 8192

    def buf(off, dtype=torch.float32):
        t = torch.empty(n + pad, dtype=dtype, device=dev)
        return t[off:off + n]
    p, g, m, v = buf(offs[0]), buf(offs[1]), buf(offs[2]), buf(offs[3])
    plp = buf(offs[4], torch.bfloat16)
    p.copy_(torch.randn(n, device=dev, generator=gen))
    g.copy_(torch.randn(n, device=dev, generator=gen) * 1e-2)
    m.zero_()
    v.zero_()
    nparts = K.sumsq_nparts(n)
    ws = torch.empty(nparts, device=dev)
    state = torch.zeros(8, device=dev)
    K.sumsq_partial(g, ws)
    for _ in range(3):
        K.adam_step(p, plp, g, m, v, ws, nparts, state, 5.0, 1, 0.0, 5.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record(s)
        for _ in range(20):
            K.adam_step(p, plp, g, m, v, ws, nparts, state, 5.0, 1, 0.0, 5.0, 256.0, 25000.0, 0.9, 0.98, 1e-9, 0.0)
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
    print(json.dumps({"n": n, "offsets": offs, "adam_us": round(best, 1), "GB_s": round(30.0 * n / best / 1e3, 1)}),
          flush=True)


for n in (46_200_000, 108_000_000):
    for offs in ((0, 0, 0, 0, 0), (0, 384, 1152, 1920, 2816), (0, 1024, 2048, 3072, 4096)):
        run(n, offs)
