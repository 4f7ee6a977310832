"""Bitwise A/B of the fused attention kernels between two builds of libliteasr_hip.so.

    LITEASR_HIP_LIB=<lib> python tools/attn_check.py dump OUT.pt   # every output of every case
    python tools/attn_check.py cmp A.pt B.pt                         # JSON line per tensor

Cases are attn_bench.py's shapes (relative-position self attention of configs 2 / 4 / 5, the
decoder's self and source attention, the long config's split source attention) on fixed
seeded inputs; outputs: ctx, stats (forward), dqu / dq, dbd, dk, dv, D (backward).  A kernel
change that keeps every product, sum and rounding (a new schedule, LDS layout or pipeline)
must compare equal bit for bit; one that changes arithmetic reports its max abs / rel error."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel_case(K, B, H, T, dk, chunk, seed):
    dev, bf = "cuda", torch.bfloat16
    d = H * dk
    g = torch.Generator(device=dev).manual_seed(seed)
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
    stats = torch.zeros(B * H * T * 2, device=dev)
    ctx = torch.zeros(B * T, d, dtype=bf, device=dev)
    k, v = qkv[:, d:2 * d], qkv[:, 2 * d:]
    K.relattn_fwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx)
    ldS = (T + 7) // 8 * 8
    Dbuf = torch.zeros(B * H * T, device=dev)
    dqu = torch.zeros(B * T, d, dtype=bf, device=dev)
    dbd = torch.zeros(H, B, T, ldS, dtype=bf, device=dev)
    dqkv = torch.zeros(B * T, 3 * d, dtype=bf, device=dev)
    K.relattn_bwd(qu, qv, k, v, pos, B, H, T, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dqu, dbd, ldS,
                  dqkv[:, d:2 * d], dqkv[:, 2 * d:], dbd_head_major=True)
    return {"ctx": ctx, "stats": stats, "dqu": dqu, "dbd": dbd[..., :T], "dk": dqkv[:, d:2 * d],
            "dv": dqkv[:, 2 * d:], "D": Dbuf}


def plain_case(K, B, H, Tq, Tk, dk, causal, nsplit, seed):
    dev, bf = "cuda", torch.bfloat16
    d = H * dk
    g = torch.Generator(device=dev).manual_seed(seed)
    rn = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.5).to(bf)  # noqa: E731
    q, kv, dctx = rn(B * Tq, d), rn(B * Tk, 2 * d), rn(B * Tq, d)
    if causal:
        yl = torch.randint(Tq // 2, Tq + 1, (B,), device=dev, generator=g)
        m = (torch.arange(Tq, device=dev)[None, :] >= yl[:, None])[:, None, :] | \
            (torch.arange(Tq, device=dev)[None, :] > torch.arange(Tq, device=dev)[:, None])[None]
        mask, msb, msq = K.pad_mask16(m.to(torch.uint8), B, Tq, Tk)
    else:
        xl = torch.full((B,), Tk, device=dev)
        xl[1::2] = Tk - 17
        mask, msb, msq = (torch.arange(Tk, device=dev)[None, :] >= xl[:, None]).to(torch.uint8).contiguous(), Tk, 0
    scale = dk ** -0.5
    stats = torch.zeros(B * H * Tq * 2, device=dev)
    ctx = torch.zeros(B * Tq, d, dtype=bf, device=dev)
    k, v = kv[:, :d], kv[:, d:]
    K.attn_fwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, nsplit=nsplit)
    Dbuf = torch.zeros(B * H * Tq, device=dev)
    dq = torch.zeros(B * Tq, d, dtype=bf, device=dev)
    dkv = torch.zeros(B * Tk, 2 * d, dtype=bf, device=dev)
    K.attn_bwd(q, k, v, B, H, Tq, Tk, mask, msb, msq, scale, stats, ctx, dctx, Dbuf, dq, dkv[:, :d], dkv[:, d:],
               nsplit=nsplit)
    return {"ctx": ctx, "stats": stats, "dq": dq, "dk": dkv[:, :d], "dv": dkv[:, d:], "D": Dbuf}


def dump(out):
    from liteasr_amd import kernels as K

    torch.cuda.set_device(0)
    res = {}
    for name, args in (("small", (32, 4, 249, 64, 0)), ("large", (32, 16, 249, 32, 16)), ("long", (8, 4, 999, 64, 0)),
                       ("odd", (3, 4, 77, 64, 0)), ("odd32", (3, 8, 130, 32, 8))):
        res[name] = rel_case(K, *args, seed=7)
    for name, args in (("dec", (32, 4, 41, 41, 64, True, None)), ("src", (32, 4, 41, 249, 64, False, None)),
                       ("srclong", (8, 4, 151, 999, 64, False, None)), ("dec32", (8, 8, 41, 41, 32, True, None))):
        res[name] = plain_case(K, *args, seed=9)
    torch.cuda.synchronize()
    torch.save({c: {k: v.cpu() for k, v in d.items()} for c, d in res.items()}, out)
    print(json.dumps({"dumped": out, "lib": os.environ.get("LITEASR_HIP_LIB", "tree")}))


def cmp(a_path, b_path):
    a, b = torch.load(a_path, weights_only=True), torch.load(b_path, weights_only=True)
    bad = 0
    for case in a:
        for k in a[case]:
            x, y = a[case][k].float(), b[case][k].float()
            fin = torch.isfinite(x) & torch.isfinite(y)
            same = torch.equal(a[case][k], b[case][k])
            d = (x[fin] - y[fin]).abs().max().item() if fin.any() else 0.0
            den = y[fin].abs().max().item() if fin.any() else 1.0
            bad += not same
            print(json.dumps({"case": case, "out": k, "bitwise_equal": same, "max_abs": d,
                              "max_rel": d / (den + 1e-30), "nonfinite_mismatch": int((torch.isfinite(x) != torch.isfinite(y)).sum())}))
    print(json.dumps({"tensors_differing": bad}))


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
