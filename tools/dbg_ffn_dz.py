import sys, torch
sys.path.insert(0, "/root/repo")
from liteasr_amd import kernels as kn, _native as Nn
M, D, F, p = 7968, 256, 2048, 0.1
g = torch.Generator().manual_seed(M + D)
bf = torch.bfloat16; DEV = "cuda"
ln = torch.randn(M, D, generator=g).to(bf).to(DEV)
w1 = (torch.randn(F, D, generator=g) / D ** 0.5).to(bf).to(DEV)
b1 = (torch.randn(F, generator=g) * 0.1).to(DEV)
w2 = (torch.randn(D, F, generator=g) / F ** 0.5).to(bf).to(DEV)
gb = torch.randn(M, D, generator=g).to(bf).to(DEV)
for pp in (0.0, 0.1):
    h = torch.empty(M, F, device=DEV, dtype=bf); gate = torch.empty_like(h)
    kn.linear(ln, w1, h, bias=b1, act=Nn.ACT_SWISH, zout=gate, zout_mode=1, drop_p=pp, drop_seed=1234)
    old = torch.empty(M, F, device=DEV, dtype=bf)
    kn.gemm(gb, w2, old, alpha=kn.dropout_scale(pp), aux=gate, aux_act=Nn.ACT_GATE)
    new = torch.empty_like(old)
    kn.ffn_dz(ln, w1, b1, gb, w2, Nn.ACT_SWISH, pp, 1234, new)
    torch.cuda.synchronize()
    u = ln.double() @ w1.double().t() + b1.double()
    s = torch.sigmoid(u); d = s * (1 + u * (1 - s))
    keep = (gate.double() != 0).double() if pp > 0 else torch.ones_like(u)
    ref = (gb.double() @ w2.double()) * d * keep * (kn.dropout_scale(pp) if pp > 0 else 1)
    sc = ref.abs().max().item()
    eo = (old.double() - ref).abs(); en = (new.double() - ref).abs()
    print("p", pp, "old err", eo.max().item() / sc, "new err", en.max().item() / sc)
    bad = en > 0.02 * sc
    idx = bad.nonzero()
    print(" bad count", int(bad.sum()), "first", idx[:8].tolist())
    if len(idx):
        r = idx[:, 0]; c = idx[:, 1]
        print(" rows mod 128 hist", torch.bincount(r % 128, minlength=128).nonzero().flatten()[:20].tolist())
        print(" cols mod 128 hist", torch.bincount(c % 128, minlength=128).nonzero().flatten()[:40].tolist())
        print(" row tiles", torch.unique(r // 128)[:10].tolist(), "col tiles", torch.unique(c // 128).tolist())
        m0, n0 = idx[0].tolist()
        print(" sample new/old/ref", new[m0, n0].item(), old[m0, n0].item(), ref[m0, n0].item(), "d", d[m0,n0].item(), "keep", keep[m0,n0].item())
