// LayerNorm (eps 1e-12 in LiteASR: liteasr/nets/layer_norm.py:8-21) forward/backward,
// residual-branch gradient fusion, and deterministic column sums (bias grads).
// One wave per row, D/64 contiguous elements per lane in registers (D % 64 == 0, D <= 1024).
#include <algorithm>

#include "common.h"
#include "ln_math.h"

constexpr int LN_WAVES = 4;           // forward: one row per wave
constexpr int LN_ROWS_PER_BLOCK = 16;  // backward: rows per block (one partial row each; 16: one row per wave, 2 blocks per CU)

// Lane l owns the NPL contiguous columns [l*NPL, (l+1)*NPL) of a row (vector loads).
template <int NPL, typename TX, typename TY, typename TY2>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const TX* __restrict__ x, int64_t rows,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     TY* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd, TY2* __restrict__ y2,
                                                     DropCfg d2) {
  constexpr int D = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c0 = lane * NPL;
  float v[NPL], g[NPL], b[NPL];
  ldv<NPL>(x + row * D + c0, v);
  ldv<NPL>(gamma + c0, g);
  ldv<NPL>(beta + c0, b);
  float o[NPL], mu, rs;
  ln_fwd_row<D, NPL>(v, g, b, eps, o, mu, rs);
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
  stv<NPL>(y + row * D + c0, o);
  if (y2) {
    if (d2.p > 0.f) {
      float dm[NPL];
      drop_mul_n<NPL>(d2, drop_key(d2), (uint64_t)row * D + c0, dm);
#pragma unroll
      for (int i = 0; i < NPL; ++i) o[i] *= dm[i];
    }
    stv<NPL>(y2 + row * D + c0, o);
  }
}

// Two chained LayerNorms of one row (a Conformer layer's final norm and the next layer's
// first norm, conformer_layer.py:147 -> :130): y = LN1(x) stored fp32 (the layer output),
// z = LN2(y) stored bf16, each with its row statistics.  LN2 reads the fp32 y it just wrote,
// so z and its statistics are bit-identical to a separate lasr_layernorm_fwd on y.
template <int NPL>
__global__ __launch_bounds__(256) void ln2_fwd_kernel(const float* __restrict__ x, int64_t rows,
                                                      const float* __restrict__ g1, const float* __restrict__ b1,
                                                      const float* __restrict__ g2, const float* __restrict__ b2,
                                                      float eps, float* __restrict__ y, float* __restrict__ mean1,
                                                      float* __restrict__ rstd1, bf16_t* __restrict__ z,
                                                      float* __restrict__ mean2, float* __restrict__ rstd2) {
  constexpr int D = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c0 = lane * NPL;
  float v[NPL], g[NPL], b[NPL];
  ldv<NPL>(x + row * D + c0, v);
  ldv<NPL>(g1 + c0, g);
  ldv<NPL>(b1 + c0, b);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float o[NPL], mu, rs;
    ln_fwd_row<D, NPL>(v, g, b, eps, o, mu, rs);
    if (pass == 0) {
      if (lane == 0) { mean1[row] = mu; rstd1[row] = rs; }
      stv<NPL>(y + row * D + c0, o);
#pragma unroll
      for (int i = 0; i < NPL; ++i) v[i] = o[i];
      ldv<NPL>(g2 + c0, g);
      ldv<NPL>(b2 + c0, b);
    } else {
      if (lane == 0) { mean2[row] = mu; rstd2[row] = rs; }
      stv<NPL>(z + row * D + c0, o);
    }
  }
}

// Backward: LnbCfg::WAVES waves per block, each LN_ROWS_PER_BLOCK / WAVES rows; the
// block's dgamma/dbeta partials are combined in fixed order through LDS (deterministic).
template <int NPL>
struct LnbCfg {
  static constexpr int WAVES = NPL <= 8 ? 16 : 8;
  static constexpr int RPW = LN_ROWS_PER_BLOCK / WAVES;
};

template <int NPL, typename TX, typename TD, typename TR, typename TDX, typename TGB>
// (every pointer __restrict__: lets the compiler issue a wave's second-row loads ahead of
// its first-row stores)
__global__ __launch_bounds__(1024) void ln_bwd_kernel(const TX* __restrict__ x,
                                                      const TD* __restrict__ dy, int64_t rows,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ rstd,
                                                      const TR* __restrict__ dres, TDX* __restrict__ dx,
                                                      float* __restrict__ part, TGB* __restrict__ gb,
                                                      float bscale, DropCfg bd) {
  constexpr int D = NPL * 64, WAVES = LnbCfg<NPL>::WAVES, RPW = LnbCfg<NPL>::RPW;
  __shared__ float sp[WAVES][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * NPL;
  float pg[NPL], pb[NPL], gm[NPL];
  ldv<NPL>(gamma + c0, gm);
#pragma unroll
  for (int i = 0; i < NPL; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const uint32_t key = (gb && bd.p > 0.f) ? drop_key(bd) : 0u;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = (int64_t)blockIdx.x * LN_ROWS_PER_BLOCK + w * RPW + rr;
    if (row < rows) {
      const float mu = mean[row], rs = rstd[row];
      float xv[NPL], d[NPL];
      ldv<NPL>(x + row * D + c0, xv);
      ldv<NPL>(dy + row * D + c0, d);
      float o[NPL], r[NPL];
      if (dres) {
        ldv<NPL>(dres + row * D + c0, r);
        ln_bwd_row<D, NPL, true>(xv, d, gm, mu, rs, r, pg, pb, o);
      } else {
        ln_bwd_row<D, NPL, false>(xv, d, gm, mu, rs, r, pg, pb, o);
      }
      stv<NPL>(dx + row * D + c0, o);
      if (gb) {
        float dm[NPL];
        if (bd.p > 0.f) drop_mul_n<NPL>(bd, key, (uint64_t)(row * D + c0), dm);
#pragma unroll
        for (int i = 0; i < NPL; ++i) o[i] *= bscale * (bd.p > 0.f ? dm[i] : 1.f);
        stv<NPL>(gb + row * D + c0, o);
      }
    }
  }
  // fixed-order combine of the WAVES partials: dgamma then dbeta through one LDS array
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < NPL; ++i) sp[w][c0 + i] = pass == 0 ? pg[i] : pb[i];
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < WAVES; ++k) a += sp[k][c];
      part[(int64_t)blockIdx.x * 2 * D + pass * D + c] = a;
    }
    __syncthreads();
  }
}

// Two chained LayerNorm backwards per row, across a Conformer layer boundary (the reverse of
// ln2_fwd_kernel): the next layer's first norm (x1 fp32, dy1 = its GEMM's input gradient, dres1
// fp32: dx1 = dres1 + LN1'(dy1), kept in registers), then this layer's final norm on dx1 (x2
// fp32: dx2 = LN2'(dx1) stored, gb2 = bscale2 * drop(dx2)).  Rows, waves, the per-row
// arithmetic (ln_bwd_row) and the two partial-row layouts are ln_bwd_kernel's: bit-identical
// to lasr_layernorm_bwd run twice with dx1 stored in fp32 between them.
template <int NPL, typename TD, typename TGB>
__global__ __launch_bounds__(1024) void ln2_bwd_kernel(const float* __restrict__ x1, const TD* __restrict__ dy1,
                                                       const float* __restrict__ dres1, const float* __restrict__ g1,
                                                       const float* __restrict__ mean1, const float* __restrict__ rstd1,
                                                       float* __restrict__ part1, const float* __restrict__ x2,
                                                       const float* __restrict__ g2, const float* __restrict__ mean2,
                                                       const float* __restrict__ rstd2, float* __restrict__ dx2,
                                                       float* __restrict__ part2, TGB* __restrict__ gb2,
                                                       int64_t rows, float bscale, DropCfg bd) {
  constexpr int D = NPL * 64, WAVES = LnbCfg<NPL>::WAVES, RPW = LnbCfg<NPL>::RPW;
  __shared__ float sp[WAVES][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * NPL;
  float pg1[NPL], pb1[NPL], pg2[NPL], pb2[NPL], gm1[NPL], gm2[NPL];
  ldv<NPL>(g1 + c0, gm1);
  ldv<NPL>(g2 + c0, gm2);
#pragma unroll
  for (int i = 0; i < NPL; ++i) { pg1[i] = 0.f; pb1[i] = 0.f; pg2[i] = 0.f; pb2[i] = 0.f; }
  const uint32_t key = (gb2 && bd.p > 0.f) ? drop_key(bd) : 0u;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = (int64_t)blockIdx.x * LN_ROWS_PER_BLOCK + w * RPW + rr;
    if (row < rows) {
      float xv[NPL], d[NPL], r[NPL], o1[NPL], o2[NPL], xw[NPL];
      ldv<NPL>(x1 + row * D + c0, xv);
      ldv<NPL>(dy1 + row * D + c0, d);
      ldv<NPL>(dres1 + row * D + c0, r);
      ldv<NPL>(x2 + row * D + c0, xw);
      ln_bwd_row<D, NPL, true>(xv, d, gm1, mean1[row], rstd1[row], r, pg1, pb1, o1);
      ln_bwd_row<D, NPL, false>(xw, o1, gm2, mean2[row], rstd2[row], r, pg2, pb2, o2);
      stv<NPL>(dx2 + row * D + c0, o2);
      if (gb2) {
        float dm[NPL];
        if (bd.p > 0.f) drop_mul_n<NPL>(bd, key, (uint64_t)(row * D + c0), dm);
#pragma unroll
        for (int i = 0; i < NPL; ++i) o2[i] *= bscale * (bd.p > 0.f ? dm[i] : 1.f);
        stv<NPL>(gb2 + row * D + c0, o2);
      }
    }
  }
  // the two norms' partial rows, each combined as ln_bwd_kernel combines its own
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const float* src = pass == 0 ? pg1 : pass == 1 ? pb1 : pass == 2 ? pg2 : pb2;
    float* part = pass < 2 ? part1 : part2;
#pragma unroll
    for (int i = 0; i < NPL; ++i) sp[w][c0 + i] = src[i];
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < WAVES; ++k) a += sp[k][c];
      part[(int64_t)blockIdx.x * 2 * D + (pass & 1) * D + c] = a;
    }
    __syncthreads();
  }
}

__global__ void ln_param_reduce_kernel(const float* part, int nblk, int D, float* dgamma,
                                       float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nblk; ++k) {
    a += part[(int64_t)k * 2 * D + c];
    b += part[(int64_t)k * 2 * D + D + c];
  }
  if (dgamma) dgamma[c] += a;
  if (dbeta) dbeta[c] += b;
}

// --------------------------- dispatch helpers ------------------------------------
template <int NPL, typename TX, typename TY>
static void ln_fwd_y2(const void* x, int64_t rows, const float* g, const float* b, float eps,
                      void* y, float* mean, float* rstd, void* y2, int y2dt, DropCfg d2,
                      hipStream_t st) {
  const unsigned nb = (unsigned)cdiv(rows, LN_WAVES);
  if (y2 && y2dt == LASR_F32)
    ln_fwd_kernel<NPL, TX, TY, float><<<nb, 256, 0, st>>>((const TX*)x, rows, g, b, eps, (TY*)y, mean, rstd, (float*)y2, d2);
  else
    ln_fwd_kernel<NPL, TX, TY, bf16_t><<<nb, 256, 0, st>>>((const TX*)x, rows, g, b, eps, (TY*)y, mean, rstd, (bf16_t*)y2, d2);
}
template <int NPL>
static void ln_fwd_npl(const void* x, int xdt, int64_t rows, const float* g, const float* b,
                       float eps, void* y, int ydt, float* mean, float* rstd, void* y2, int y2dt,
                       DropCfg d2, hipStream_t st) {
  if (xdt == LASR_F32 && ydt == LASR_F32) ln_fwd_y2<NPL, float, float>(x, rows, g, b, eps, y, mean, rstd, y2, y2dt, d2, st);
  else if (xdt == LASR_F32) ln_fwd_y2<NPL, float, bf16_t>(x, rows, g, b, eps, y, mean, rstd, y2, y2dt, d2, st);
  else if (ydt == LASR_F32) ln_fwd_y2<NPL, bf16_t, float>(x, rows, g, b, eps, y, mean, rstd, y2, y2dt, d2, st);
  else ln_fwd_y2<NPL, bf16_t, bf16_t>(x, rows, g, b, eps, y, mean, rstd, y2, y2dt, d2, st);
}

// Rows are read/written D/64 contiguous elements per lane: pointers must be aligned to that
// (capped at 16 B).
static bool ln_aligned(const void* p, int D, int dt) {
  const int esz = dt == LASR_F32 ? 4 : 2;
  const int a = std::min(16, (D / 64) * esz);
  return p == nullptr || ((uintptr_t)p % a) == 0;
}

extern "C" int lasr_layernorm_fwd(const void* x, int x_dtype, int64_t rows, int D,
                                  const float* gamma, const float* beta, float eps, void* y,
                                  int y_dtype, float* mean, float* rstd, void* y2, int y2_dtype,
                                  float p2, uint64_t seed2, void* stream) {
  LASR_CHECK_ARG(D % 64 == 0 && D >= 64 && D <= 1024, "lasr_layernorm_fwd: D=%d unsupported", D);
  LASR_CHECK_ARG(ln_aligned(x, D, x_dtype) && ln_aligned(y, D, y_dtype) && ln_aligned(y2, D, y2_dtype) &&
                     ln_aligned(gamma, D, LASR_F32) && ln_aligned(beta, D, LASR_F32),
                 "lasr_layernorm_fwd: misaligned row pointer");
  if (rows <= 0) return LASR_OK;
  DropCfg d2 = mkdrop(p2, seed2);
  hipStream_t st = (hipStream_t)stream;
  switch (D / 64) {
    case 1: ln_fwd_npl<1>(x, x_dtype, rows, gamma, beta, eps, y, y_dtype, mean, rstd, y2, y2_dtype, d2, st); break;
    case 2: ln_fwd_npl<2>(x, x_dtype, rows, gamma, beta, eps, y, y_dtype, mean, rstd, y2, y2_dtype, d2, st); break;
    case 4: ln_fwd_npl<4>(x, x_dtype, rows, gamma, beta, eps, y, y_dtype, mean, rstd, y2, y2_dtype, d2, st); break;
    case 8: ln_fwd_npl<8>(x, x_dtype, rows, gamma, beta, eps, y, y_dtype, mean, rstd, y2, y2_dtype, d2, st); break;
    case 16: ln_fwd_npl<16>(x, x_dtype, rows, gamma, beta, eps, y, y_dtype, mean, rstd, y2, y2_dtype, d2, st); break;
    default: lasr_set_error("lasr_layernorm_fwd: D=%d unsupported", D); return LASR_ERR_INVALID;
  }
  return lasr_check_launch("layernorm_fwd");
}

extern "C" int lasr_layernorm2_fwd(const float* x, int64_t rows, int D, const float* g1, const float* b1,
                                   const float* g2, const float* b2, float eps, float* y, float* mean1,
                                   float* rstd1, void* z, float* mean2, float* rstd2, void* stream) {
  LASR_CHECK_ARG(D == 256 || D == 512 || D == 128 || D == 64, "lasr_layernorm2_fwd: D=%d unsupported", D);
  LASR_CHECK_ARG(ln_aligned(x, D, LASR_F32) && ln_aligned(y, D, LASR_F32) && ln_aligned(z, D, LASR_BF16) &&
                     ln_aligned(g1, D, LASR_F32) && ln_aligned(b1, D, LASR_F32) && ln_aligned(g2, D, LASR_F32) &&
                     ln_aligned(b2, D, LASR_F32),
                 "lasr_layernorm2_fwd: misaligned row pointer");
  if (rows <= 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  const unsigned nb = (unsigned)cdiv(rows, LN_WAVES);
#define LN2(NPL) ln2_fwd_kernel<NPL><<<nb, LN_WAVES * 64, 0, st>>>(x, rows, g1, b1, g2, b2, eps, y, mean1, rstd1, \
                                                                  (bf16_t*)z, mean2, rstd2)
  if (D == 64) LN2(1);
  else if (D == 128) LN2(2);
  else if (D == 256) LN2(4);
  else LN2(8);
#undef LN2
  return lasr_check_launch("layernorm2_fwd");
}

// Backward dispatch: x/dy dtypes in {f32,bf16}; dres (f32/bf16/none), dx f32/bf16, gb bf16/f32.
template <int NPL, typename TX, typename TD>
static void ln_bwd_3(const void* x, const void* dy, int64_t rows, const float* gamma,
                     const float* mean, const float* rstd, const void* dres, int dresdt, void* dx,
                     int dxdt, float* part, void* gb, int gbdt, float bscale, DropCfg bd,
                     hipStream_t st) {
  const unsigned nb = (unsigned)cdiv(rows, LN_ROWS_PER_BLOCK);
#define LNB(TR, TDX, TGB)                                                                     \
  ln_bwd_kernel<NPL, TX, TD, TR, TDX, TGB><<<nb, LnbCfg<NPL>::WAVES * 64, 0, st>>>(          \
      (const TX*)x, (const TD*)dy, rows, gamma, mean, rstd, (const TR*)dres, (TDX*)dx, part, \
      (TGB*)gb, bscale, bd)
  const bool rf = dresdt == LASR_F32, xf = dxdt == LASR_F32, gf = gbdt == LASR_F32;
  if (rf && xf && gf) LNB(float, float, float);
  else if (rf && xf) LNB(float, float, bf16_t);
  else if (rf && gf) LNB(float, bf16_t, float);
  else if (rf) LNB(float, bf16_t, bf16_t);
  else if (xf && gf) LNB(bf16_t, float, float);
  else if (xf) LNB(bf16_t, float, bf16_t);
  else if (gf) LNB(bf16_t, bf16_t, float);
  else LNB(bf16_t, bf16_t, bf16_t);
#undef LNB
}
template <int NPL>
static void ln_bwd_npl(const void* x, int xdt, const void* dy, int dydt, int64_t rows,
                       const float* gamma, const float* mean, const float* rstd, const void* dres,
                       int dresdt, void* dx, int dxdt, float* part, void* gb, int gbdt,
                       float bscale, DropCfg bd, hipStream_t st) {
  if (xdt == LASR_F32 && dydt == LASR_F32) ln_bwd_3<NPL, float, float>(x, dy, rows, gamma, mean, rstd, dres, dresdt, dx, dxdt, part, gb, gbdt, bscale, bd, st);
  else if (xdt == LASR_F32) ln_bwd_3<NPL, float, bf16_t>(x, dy, rows, gamma, mean, rstd, dres, dresdt, dx, dxdt, part, gb, gbdt, bscale, bd, st);
  else if (dydt == LASR_F32) ln_bwd_3<NPL, bf16_t, float>(x, dy, rows, gamma, mean, rstd, dres, dresdt, dx, dxdt, part, gb, gbdt, bscale, bd, st);
  else ln_bwd_3<NPL, bf16_t, bf16_t>(x, dy, rows, gamma, mean, rstd, dres, dresdt, dx, dxdt, part, gb, gbdt, bscale, bd, st);
}

extern "C" int lasr_layernorm_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype,
                                  int64_t rows, int D, const float* gamma, const float* mean,
                                  const float* rstd, const void* dres, int dres_dtype, void* dx,
                                  int dx_dtype, float* dgamma, float* dbeta, float* workspace,
                                  int64_t ws_floats, void* gb, int gb_dtype, float bscale,
                                  float bp, uint64_t bseed, void* stream) {
  LASR_CHECK_ARG(D % 64 == 0 && D >= 64 && D <= 1024, "lasr_layernorm_bwd: D=%d unsupported", D);
  LASR_CHECK_ARG(ln_aligned(x, D, x_dtype) && ln_aligned(dy, D, dy_dtype) &&
                     ln_aligned(dres, D, dres_dtype) && ln_aligned(dx, D, dx_dtype) &&
                     ln_aligned(gb, D, gb_dtype) && ln_aligned(gamma, D, LASR_F32),
                 "lasr_layernorm_bwd: misaligned row pointer");
  if (rows <= 0) return LASR_OK;
  const int64_t nblk = cdiv(rows, LN_ROWS_PER_BLOCK);
  LASR_CHECK_ARG(ws_floats >= nblk * 2 * D, "lasr_layernorm_bwd: workspace too small (%lld < %lld)",
                 (long long)ws_floats, (long long)(nblk * 2 * D));
  DropCfg bd = mkdrop(bp, bseed);
  hipStream_t st = (hipStream_t)stream;
  switch (D / 64) {
#define CASE(n) case n: ln_bwd_npl<n>(x, x_dtype, dy, dy_dtype, rows, gamma, mean, rstd, dres, dres_dtype, dx, dx_dtype, workspace, gb, gb_dtype, bscale, bd, st); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
    default: lasr_set_error("lasr_layernorm_bwd: D=%d unsupported", D); return LASR_ERR_INVALID;
  }
  int rc = lasr_check_launch("layernorm_bwd");
  if (rc) return rc;
  if (dgamma && dbeta) {
    rc = lasr_reduce_cols(workspace, (int)nblk, 2 * D, dgamma, dbeta, D, 1, st);
  } else if (dgamma || dbeta) {
    ln_param_reduce_kernel<<<(unsigned)cdiv(D, 256), 256, 0, st>>>(workspace, (int)nblk, D, dgamma, dbeta);
    rc = lasr_check_launch("layernorm_bwd/reduce");
  }
  return rc;
}

// ----------------------------- branch grad ----------------------------------------
template <typename TI, typename TO>
__global__ void branch_grad_kernel(const TI* dx, int64_t n, TO* gb, float scale, DropCfg d) {
  const uint32_t key = drop_key_if(d);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gb[i] = from_f<TO>(scale * drop_mul_if(d, key, (uint64_t)i) * to_f(dx[i]));
}

extern "C" int lasr_branch_grad(const void* dx, int dx_dtype, int64_t n, void* gb, int gb_dtype,
                                float scale, float p, uint64_t seed, void* stream) {
  if (n <= 0) return LASR_OK;
  DropCfg d = mkdrop(p, seed);
  hipStream_t st = (hipStream_t)stream;
  const unsigned nb = (unsigned)std::min<int64_t>(cdiv(n, 256), 8192);
  if (dx_dtype == LASR_F32 && gb_dtype == LASR_F32) branch_grad_kernel<float, float><<<nb, 256, 0, st>>>((const float*)dx, n, (float*)gb, scale, d);
  else if (dx_dtype == LASR_F32) branch_grad_kernel<float, bf16_t><<<nb, 256, 0, st>>>((const float*)dx, n, (bf16_t*)gb, scale, d);
  else if (gb_dtype == LASR_F32) branch_grad_kernel<bf16_t, float><<<nb, 256, 0, st>>>((const bf16_t*)dx, n, (float*)gb, scale, d);
  else branch_grad_kernel<bf16_t, bf16_t><<<nb, 256, 0, st>>>((const bf16_t*)dx, n, (bf16_t*)gb, scale, d);
  return lasr_check_launch("branch_grad");
}

// ----------------------------- column sums ----------------------------------------
// Column sums (bias gradients): blocks of 32 column-octets x 8 row groups sum a chunk of
// rows with 16-B loads, combine the 8 groups in LDS (fixed order) and emit one partial
// row per chunk; at most CS_MAXCHUNK chunks, so the final reduce_cols stays short.
constexpr int CS_MAXCHUNK = 128;
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* X, int64_t M, int64_t N,
                                                             int64_t ldx, int64_t rpc, float* part) {
  __shared__ float sh[8][256 + 4];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t n = ((int64_t)blockIdx.x * 32 + tx) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rpc;
  const int64_t r1 = r0 + rpc < M ? r0 + rpc : M;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    for (int64_t r = r0 + ty; r < r1; r += 8) {
      float v[8];
      if (VEC) {
        ld8(X + r * ldx + n, v);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = n + q < N ? to_f(X[r * ldx + n + q]) : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += v[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) sh[ty][tx * 8 + q] = s[q];
  __syncthreads();
  // 256 columns of this block: thread t finishes column t
  const int c = threadIdx.x;
  const int64_t nc = (int64_t)blockIdx.x * 256 + c;
  if (nc < N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += sh[g][c];
    part[(int64_t)blockIdx.y * N + nc] = t;
  }
}

static int64_t colsum_chunks(int64_t M) { return std::min<int64_t>(cdiv(M, 64), CS_MAXCHUNK); }

extern "C" int lasr_colsum(const void* X, int dtype, int64_t M, int64_t N, int64_t ldx, float* out,
                           int accumulate, float* workspace, int64_t ws_floats, void* stream) {
  if (N <= 0) return LASR_OK;
  const int64_t nchunk = M > 0 ? colsum_chunks(M) : 1;
  const int64_t rpc = M > 0 ? cdiv(M, nchunk) : 0;
  LASR_CHECK_ARG(ws_floats >= nchunk * N, "lasr_colsum: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  dim3 g1((unsigned)cdiv(N, 256), (unsigned)nchunk);
  const bool vec = N % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)X & 15) == 0;
  if (M > 0) {
    if (dtype == LASR_F32) {
      if (vec) colsum_partial_kernel<float, true><<<g1, 256, 0, st>>>((const float*)X, M, N, ldx, rpc, workspace);
      else colsum_partial_kernel<float, false><<<g1, 256, 0, st>>>((const float*)X, M, N, ldx, rpc, workspace);
    } else {
      if (vec) colsum_partial_kernel<bf16_t, true><<<g1, 256, 0, st>>>((const bf16_t*)X, M, N, ldx, rpc, workspace);
      else colsum_partial_kernel<bf16_t, false><<<g1, 256, 0, st>>>((const bf16_t*)X, M, N, ldx, rpc, workspace);
    }
  } else {
    if (hipMemsetAsync(workspace, 0, N * sizeof(float), st) != hipSuccess) return lasr_check_launch("colsum/memset");
  }
  int rc = lasr_check_launch("colsum");
  if (rc) return rc;
  return lasr_reduce_cols(workspace, (int)nchunk, N, out, nullptr, N, accumulate, st);
}

// (liteasr/nets/conformer_layer.py:130 / :147 backward across a layer boundary; see
// ln2_bwd_kernel.)  dy1 fp32 or bf16, gb2 fp32 / bf16 / none; part1 / part2 [nblk][2][D] each,
// nblk = ceil(rows / 16), reduced by the caller (lasr_reduce_multi) like lasr_layernorm_bwd's.
extern "C" int lasr_layernorm2_bwd(const float* x1, const void* dy1, int dy1_dtype, const float* dres1, int64_t rows,
                                   int D, const float* g1, const float* mean1, const float* rstd1, float* part1,
                                   const float* x2, const float* g2, const float* mean2, const float* rstd2,
                                   float* dx2, float* part2, void* gb2, int gb2_dtype, float bscale, float bp,
                                   uint64_t bseed, void* stream) {
  LASR_CHECK_ARG(D == 256 || D == 512 || D == 128 || D == 64, "lasr_layernorm2_bwd: D=%d unsupported", D);
  LASR_CHECK_ARG(x1 && dy1 && dres1 && g1 && mean1 && rstd1 && part1 && x2 && g2 && mean2 && rstd2 && dx2 && part2,
                 "lasr_layernorm2_bwd: null operand");
  LASR_CHECK_ARG(dy1_dtype == LASR_F32 || dy1_dtype == LASR_BF16, "lasr_layernorm2_bwd: dy1 dtype");
  LASR_CHECK_ARG(!gb2 || gb2_dtype == LASR_F32 || gb2_dtype == LASR_BF16, "lasr_layernorm2_bwd: gb2 dtype");
  LASR_CHECK_ARG(ln_aligned(x1, D, LASR_F32) && ln_aligned(dy1, D, dy1_dtype) && ln_aligned(dres1, D, LASR_F32) &&
                     ln_aligned(x2, D, LASR_F32) && ln_aligned(dx2, D, LASR_F32) &&
                     (!gb2 || ln_aligned(gb2, D, gb2_dtype)), "lasr_layernorm2_bwd: misaligned row pointer");
  if (rows <= 0) return LASR_OK;
  const unsigned nb = (unsigned)cdiv(rows, LN_ROWS_PER_BLOCK);
  DropCfg bd = mkdrop(bp, bseed);
  hipStream_t st = (hipStream_t)stream;
#define L2B(NPL, TD, TGB)                                                                                        \
  ln2_bwd_kernel<NPL, TD, TGB><<<nb, LnbCfg<NPL>::WAVES * 64, 0, st>>>(x1, (const TD*)dy1, dres1, g1, mean1, rstd1, \
                                                                      part1, x2, g2, mean2, rstd2, dx2, part2,     \
                                                                      (TGB*)gb2, rows, bscale, bd)
#define L2D(NPL)                                                                    \
  if (dy1_dtype == LASR_BF16 && gb2_dtype != LASR_F32) L2B(NPL, bf16_t, bf16_t);    \
  else if (dy1_dtype == LASR_BF16) L2B(NPL, bf16_t, float);                         \
  else if (gb2_dtype != LASR_F32) L2B(NPL, float, bf16_t);                          \
  else L2B(NPL, float, float);
  switch (D / 64) {
    case 1: { L2D(1) } break;
    case 2: { L2D(2) } break;
    case 4: { L2D(4) } break;
    default: { L2D(8) } break;
  }
#undef L2D
#undef L2B
  return lasr_check_launch("layernorm2_bwd");
}
