"""Fused attention kernels at the BASELINE shapes, each timed as a replayed hipGraph of `iters`
launches (HIP events on the capture stream).  One JSON line per (case, direction):
  small  : encoder rel-pos MHSA of config 2 (B 32, H 4, T' 249, d_k 64, key padding)
  large  : config 4 (B 32, H 16, T' 249, d_k 32, chunk-16 streaming mask)
  long   : config 5 (B 8, H 4, T' 999, d_k 64, key padding)
  smallchunk / largepad (only when named): config 2 with the chunk-16 mask, config 4 with key padding
  dec    : the decoder's self attention of config 2 (B 32, H 4, L+1 41, causal + padding)
Algorithmic flops: forward 3 x 2*B*H*Tq*Tk*d_k (QK^T, the positional product, PV; plain
attention 2 x), backward 6 x (S recomputed twice: the query- and key-side kernels, dP, dQ, dK,
dV; plain 5 x ... see `units`)."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from liteasr_amd import kernels as K  # noqa: E402

PEAK = 2500e12


def graph_time(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def rel_case(name, B, H, T, dk, chunk):
    dev = "cuda"
    d = H * dk
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(1)
    rn = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(bf)  # noqa: E731
    qkv, qu, qv, pos, dctx = rn(B * T, 3 * d), rn(B * T, d), rn(B * T, d), rn(T, d), rn(B * T, d)
    xl = torch.full((B,), T, device=dev)
    xl[1::2] = T - 17
    pad = torch.arange(T, device=dev)[None, :] >= xl[:, None]
    if chunk:
        tri = (torch.arange(T, device=dev)[None, :] // chunk) > (torch.arange(T, device=dev)[:, None] // chunk)
        mask, msb, msq = K.pad_mask16((pad[:, None, :] | tri[None]).to(torch.uint8), B, T, T)
    else:
        mask, msb, msq = pad.to(torch.uint8).contiguous(), T, 0
    scale = dk ** -0.5
    stats = torch.empty(B * H * T * 2, device=dev)
    ctx = torch.empty(B * T, d, dtype=bf, device=dev)
    k, v = qkv[:, d:2 * d], qkv[:, 2 * d:]
    fwd = lambda: K.relattn_fwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx)  # noqa: E731
    ldS = (T + 7) // 8 * 8
    Dbuf = torch.empty(B * H * T, device=dev)
    dqu = torch.empty(B * T, d, dtype=bf, device=dev)
    dbd = torch.empty(H, B, T, ldS, dtype=bf, device=dev)
    dqkv = torch.zeros(B * T, 3 * d, dtype=bf, device=dev)
    bwd = lambda: K.relattn_bwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx, dctx, Dbuf,  # noqa: E731
                                dqu, dbd, ldS, dqkv[:, d:2 * d], dqkv[:, 2 * d:], dbd_head_major=True)
    unit = 2.0 * B * H * T * T * dk
    for dirn, fn, units in (("fwd", fwd, 3), ("bwd", bwd, 6)):
        sec = graph_time(fn)
        print(json.dumps({"case": name, "dir": dirn, "B": B, "H": H, "T": T, "dk": dk, "chunk": chunk,
                          "us": round(sec * 1e6, 2), "tflops": round(units * unit / sec / 1e12, 1),
                          "mfma_frac": round(units * unit / sec / PEAK, 4)}), flush=True)


def dec_case(name, B, H, L1, dk):
    dev = "cuda"
    d = H * dk
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(2)
    rn = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(bf)  # noqa: E731
    qkv, dctx = rn(B * L1, 3 * d), rn(B * L1, d)
    yl = torch.randint(L1 // 2, L1 + 1, (B,), device=dev)
    m = (torch.arange(L1, device=dev)[None, :] >= yl[:, None])[:, None, :] | \
        (torch.arange(L1, device=dev)[None, :] > torch.arange(L1, device=dev)[:, None])[None]
    mask, msb, msq = K.pad_mask16(m.to(torch.uint8), B, L1, L1)
    scale = dk ** -0.5
    stats = torch.empty(B * H * L1 * 2, device=dev)
    ctx = torch.empty(B * L1, d, dtype=bf, device=dev)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    fwd = lambda: K.attn_fwd(q, k, v, B, H, L1, L1, mask, msb, msq, scale, stats, ctx)  # noqa: E731
    Dbuf = torch.empty(B * H * L1, device=dev)
    dqkv = torch.zeros(B * L1, 3 * d, dtype=bf, device=dev)
    bwd = lambda: K.attn_bwd(q, k, v, B, H, L1, L1, mask, msb, msq, scale, stats, ctx, dctx, Dbuf,  # noqa: E731
                             dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:])
    unit = 2.0 * B * H * L1 * L1 * dk
    for dirn, fn, units in (("fwd", fwd, 2), ("bwd", bwd, 5)):
        sec = graph_time(fn)
        print(json.dumps({"case": name, "dir": dirn, "B": B, "H": H, "T": L1, "dk": dk, "us": round(sec * 1e6, 2),
                          "tflops": round(units * unit / sec / 1e12, 1)}), flush=True)


def src_case(name, B, H, Tq, Tk, dk, nsplit=None):
    """The decoder's source attention: Tq = L + 1 queries over the encoder output's Tk keys
    (key padding), plain scaled dot-product (no positional term); nsplit: the key split
    (None: the library's choice)."""
    dev = "cuda"
    d = H * dk
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(3)
    rn = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(bf)  # noqa: E731
    q, kv, dctx = rn(B * Tq, d), rn(B * Tk, 2 * d), rn(B * Tq, d)
    xl = torch.full((B,), Tk, device=dev)
    xl[1::2] = Tk - 17
    mask = (torch.arange(Tk, device=dev)[None, :] >= xl[:, None]).to(torch.uint8).contiguous()
    scale = dk ** -0.5
    stats = torch.empty(B * H * Tq * 2, device=dev)
    ctx = torch.empty(B * Tq, d, dtype=bf, device=dev)
    k, v = kv[:, :d], kv[:, d:]
    fwd = lambda: K.attn_fwd(q, k, v, B, H, Tq, Tk, mask, Tk, 0, scale, stats, ctx, nsplit=nsplit)  # noqa: E731
    Dbuf = torch.empty(B * H * Tq, device=dev)
    dq = torch.empty(B * Tq, d, dtype=bf, device=dev)
    dkv = torch.zeros(B * Tk, 2 * d, dtype=bf, device=dev)
    bwd = lambda: K.attn_bwd(q, k, v, B, H, Tq, Tk, mask, Tk, 0, scale, stats, ctx, dctx, Dbuf,  # noqa: E731
                             dq, dkv[:, :d], dkv[:, d:], nsplit=nsplit)
    unit = 2.0 * B * H * Tq * Tk * dk
    for dirn, fn, units in (("fwd", fwd, 2), ("bwd", bwd, 5)):
        sec = graph_time(fn)
        print(json.dumps({"case": name, "dir": dirn, "B": B, "H": H, "Tq": Tq, "Tk": Tk, "dk": dk,
                          "nsplit": K.attn_split(B, H, Tq, Tk, nsplit),
                          "us": round(sec * 1e6, 2), "tflops": round(units * unit / sec / 1e12, 1)}), flush=True)


def main():
    torch.cuda.set_device(0)
    sel = sys.argv[1:]
    cases = [("small", 32, 4, 249, 64, 0), ("large", 32, 16, 249, 32, 16), ("long", 8, 4, 999, 64, 0)]
    for c in cases:
        if not sel or c[0] in sel:
            rel_case(*c)
    # attribution cases, only when named: d_k 64 with the chunk-mask tile, d_k 32 without it
    for c in [("smallchunk", 32, 4, 249, 64, 16), ("largepad", 32, 16, 249, 32, 0)]:
        if c[0] in sel:
            rel_case(*c)
    if not sel or "dec" in sel:
        dec_case("dec", 32, 4, 41, 64)
    if not sel or "src" in sel:
        src_case("src", 32, 4, 41, 249, 64)
    if "srcsplit" in sel:  # the key split of the source attention, swept
        for ns in (1, 2, 4, 8, 16):
            src_case("srclong", 8, 4, 151, 999, 64, nsplit=ns)
        for ns in (1, 2, 4):
            src_case("src", 32, 4, 41, 249, 64, nsplit=ns)
    if not sel or "srclong" in sel:
        src_case("srclong", 8, 4, 151, 999, 64)


if __name__ == "__main__":
    main()
