"""Per-launch time of the full-row GEMM + LayerNorm kernels (gemm_row.hip) against the
two-launch path they replace, at the small config's shapes (rows B*T' = 7968, d 256).

    python tools/row_ln_bench.py [--iters 50] [--rows 7968] [--d 256]

Prints one JSON line per case: fused us, unfused us (GEMM + norm), and the GEMM alone."""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    import torch

    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rows", type=int, default=7968)
    ap.add_argument("--d", type=int, default=256)
    args = ap.parse_args()
    import torch

    from liteasr_amd import kernels as K

    dev = "cuda"
    M, D = args.rows, args.d
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    K.set_dropout_counter(ctr)
    bf = torch.bfloat16
    g1, b1, bias = (torch.randn(D, device=dev) for _ in range(3))
    res = torch.randn(M, D, device=dev)
    for Kd in (256, 512, 768, 2048):
        x = torch.randn(M, Kd, device=dev).to(bf)
        w = (torch.randn(D, Kd, device=dev) * Kd ** -0.5).to(bf)
        out, y1 = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev, dtype=bf)
        m1, r1 = torch.empty(M, device=dev), torch.empty(M, device=dev)

        def fused():
            K.linear_res_ln(x, w, out, y1, m1, r1, g1, b1, 1e-12, bias=bias, res=res, res_scale=0.5, drop_p=0.1,
                            drop_seed=3)

        def gemm_only():
            K.linear(x, w, out, bias=bias, res=res, res_scale=0.5, drop_p=0.1, drop_seed=3)

        def unfused():
            gemm_only()
            K.layernorm_fwd(out, g1, b1, 1e-12, y1, m1, r1)

        print(json.dumps({"case": f"fwd K={Kd}", "fused_us": round(timed(fused, args.iters), 2),
                          "unfused_us": round(timed(unfused, args.iters), 2),
                          "gemm_only_us": round(timed(gemm_only, args.iters), 2)}), flush=True)
        dy = torch.randn(M, Kd, device=dev).to(bf)
        wt = (torch.randn(Kd, D, device=dev) * Kd ** -0.5).to(bf)
        xr = torch.randn(M, D, device=dev)
        dx, gb, dln = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev, dtype=bf), \
            torch.empty(M, D, device=dev, dtype=bf)
        dres = torch.randn(M, D, device=dev)
        dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)

        def bfused():
            with K.deferred_reductions():
                K.linear_dx_ln_bwd(dy, wt, xr, g1, m1, r1, dx, dg, db, dres=dres, gb=gb, bscale=1.0, bp=0.1,
                                   bseed=5)

        def bgemm():
            K.gemm(dy, wt, dln)

        def bunfused():
            with K.deferred_reductions():
                bgemm()
                K.layernorm_bwd(xr, dln, g1, m1, r1, dx, dg, db, dres=dres, gb=gb, bscale=1.0, bp=0.1, bseed=5)

        print(json.dumps({"case": f"bwd K={Kd}", "fused_us": round(timed(bfused, args.iters), 2),
                          "unfused_us": round(timed(bunfused, args.iters), 2),
                          "gemm_only_us": round(timed(bgemm, args.iters), 2),
                          "note": "fused / unfused include the deferred dgamma/dbeta reduce launch"}), flush=True)


if __name__ == "__main__":
    main()
