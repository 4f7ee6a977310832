// LayerNorm row arithmetic shared by the norm kernels (norm.hip) and the full-row GEMM
// epilogues (gemm_row.hip): one row, NPL contiguous values per lane of a 64-lane wave.
// Every operation is written out (explicit fmaf, contraction off), so both kernels produce
// the same bits whatever the compiler would fuse in their different contexts.
#pragma once
#include "common.h"

// Sum over the 64 lanes, every lane receiving the same value: pairs (l, l^1) and (l, l^2) by
// DPP quad permutes, (l, 7-l) and (l, 15-l) by the DPP half-row / row mirrors (after the
// previous steps these pair 4-lane and 8-lane groups that hold one value each), l ^ 16 by a
// ds_swizzle, and the two 32-lane halves through readlane: no ds_bpermute round trips (the
// __shfl_xor butterfly of wave_sum costs six dependent LDS-crossbar trips per reduction).
LASR_DEV float wave_sum_dpp(float v) {
  // quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401F));
  const float lo = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float hi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  return lo + hi;
}

// y = (x - mean) * rstd * g + b over the row; mean / rstd out (liteasr/nets/layer_norm.py:20,
// biased variance, eps inside the square root).
template <int D, int NPL>
LASR_DEV void ln_fwd_row(const float* v, const float* g, const float* b, float eps, float* o, float& mu,
                         float& rs) {
#pragma clang fp contract(off)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) s += v[i];
  mu = wave_sum_dpp(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const float dv = v[i] - mu;
    q = fmaf(dv, dv, q);
  }
  const float var = wave_sum_dpp(q) * (1.f / D);
  rs = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) o[i] = fmaf((v[i] - mu) * rs, g[i], b[i]);
}

// Backward of one row: x (in: the row, out: x-hat), d = dL/dy (in), gm = gamma;
// dx = rstd * (d*g - mean(d*g) - xhat * mean(d*g*xhat)) (+ r when HAS_R);
// pg += d * xhat, pb += d (the dgamma / dbeta partials, in the caller's row order).
template <int D, int NPL, bool HAS_R>
LASR_DEV void ln_bwd_row(float* x, const float* d, const float* gm, float mu, float rs, const float* r, float* pg,
                         float* pb, float* o) {
#pragma clang fp contract(off)
  float g[NPL];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    x[i] = (x[i] - mu) * rs;
    pg[i] = fmaf(d[i], x[i], pg[i]);
    pb[i] += d[i];
    g[i] = d[i] * gm[i];
    s1 += g[i];
    s2 = fmaf(g[i], x[i], s2);
  }
  s1 = wave_sum_dpp(s1) * (1.f / D);
  s2 = wave_sum_dpp(s2) * (1.f / D);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const float t = fmaf(-x[i], s2, g[i] - s1);
    o[i] = HAS_R ? fmaf(rs, t, r[i]) : rs * t;
  }
}
