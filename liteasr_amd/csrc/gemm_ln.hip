// Split-K GEMM reductions fused with the LayerNorm that consumes the GEMM's rows.
//
// The decoder runs its K = ff GEMMs on B*(L+1) = 1312 rows, a grid too small to fill the chip,
// so lasr_gemm splits K and reduces the fp32 partials in a second launch; the next LayerNorm
// was a third.  Here the reduction launch also does the norm, one wave per row:
//   lasr_gemm_ln_fwd: C = epilogue(sum of the partials) (fp32: the FFN's fc2 with its residual
//     + dropout, liteasr/nets/transformer_layer.py:211-221), then y = LN(C row) + mean / rstd
//     (the next layer's first norm, :196, or the decoder's after_norm, transformer_decoder.py:92);
//   lasr_gemm_ln_bwd: C = dln (the fc1 input gradient, bf16), then the LayerNorm backward of
//     the norm in front of the FFN (dx, the branch gradient gb, and the dgamma / dbeta partial
//     rows in lasr_layernorm_bwd's workspace layout).
// Every value is computed as the separate launches compute it: the partials summed in slice
// order (splitk_reduce_kernel), the same epilogue (epi_store4), the stored C rounding, then the
// norm arithmetic of ln_math.h in the lane layout of ln_fwd_kernel / ln_bwd_kernel (norm.hip)
// -- bit-identical (tests/test_fusions_gpu.py).  When the plan does not split K the entries run
// the GEMM and the norm as two launches.
//
// lasr_gemm_qbias_bwd: the encoder attention's positional-projection gradient dp (a K = B*T'
// GEMM per head, split over K) has its split-K reduction blocks and the independent
// positional-bias gradient blocks (lasr_qbias_bwd: dq = dqu + dqv and the du / dv partial rows,
// liteasr/nets/attention.py:131-135) in one launch.
#include "gemm_kernel.h"
#include "ln_math.h"
#include "qbias.h"

namespace {

// norm.hip's geometry (the partial-row layout and the wave combine order must match it)
constexpr int LNF_WAVES = 4;       // ln_fwd_kernel: one row per wave, 4 rows per block
constexpr int LNB_ROWS = 16;       // ln_bwd_kernel: LN_ROWS_PER_BLOCK
template <int NPL>
constexpr int lnb_waves() { return NPL <= 8 ? 16 : 8; }  // LnbCfg<NPL>::WAVES

struct LnFwdPost {
  const float* gamma;
  const float* beta;
  float eps;
  void* y;
  int y_dtype;
  float* mean;
  float* rstd;
};

struct LnBwdPost {
  const void* x;
  int x_dtype;
  const float* gamma;
  const float* mean;
  const float* rstd;
  const void* dres;
  int dres_dtype;
  void* dx;
  int dx_dtype;
  float* part;
  void* gb;
  int gb_dtype;
  float bscale;
  DropCfg bd;
};

// The row's NPL columns of lane `lane` (c0 = lane * NPL) as the split-K reduction leaves
// them: partials summed in slice order, epilogue, stored to C; v = the stored values.
template <int NPL, typename TC>
LASR_DEV void reduce_row(const GemmP& p, uint32_t dkey, float al, int64_t row, int c0, float* v) {
  const int64_t MN = (int64_t)p.M * p.N;
#pragma unroll
  for (int g4 = 0; g4 < NPL; g4 += 4) {
    const float* src = p.ws + row * p.N + c0 + g4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int sl = 0;
    for (; sl + 4 <= p.split_k; sl += 4) {
      f32x4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = *(const f32x4*)(src + (int64_t)(sl + u) * MN);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += t[u][e];
    }
    for (; sl < p.split_k; ++sl) {
      const f32x4 t = *(const f32x4*)(src + (int64_t)sl * MN);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += t[e];
    }
    epi_store4<TC, true>(p, dkey, 0, 0, 0, (int)row, c0 + g4, 4, acc, al, v + g4);
  }
}

template <int NPL, typename TY>
__global__ __launch_bounds__(256) void splitk_reduce_ln_fwd_kernel(GemmP p, LnFwdPost q) {
  constexpr int D = NPL * 64;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * LNF_WAVES + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const int c0 = lane * NPL;
  float v[NPL], g[NPL], b[NPL];
  reduce_row<NPL, float>(p, epi_key(p), alpha_of(p), row, c0, v);
  ldv<NPL>(q.gamma + c0, g);
  ldv<NPL>(q.beta + c0, b);
  float o[NPL], mu, rs;
  ln_fwd_row<D, NPL>(v, g, b, q.eps, o, mu, rs);
  if (lane == 0) { q.mean[row] = mu; q.rstd[row] = rs; }
  stv<NPL>((TY*)q.y + row * D + c0, o);
}

template <int NPL, typename TC, typename TX, typename TR, typename TDX, typename TGB>
__global__ __launch_bounds__(1024) void splitk_reduce_ln_bwd_kernel(GemmP p, LnBwdPost q) {
  constexpr int D = NPL * 64, WAVES = lnb_waves<NPL>(), RPW = LNB_ROWS / WAVES;
  __shared__ float sp[WAVES][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = lane * NPL;
  const float al = alpha_of(p);
  const uint32_t dkey = epi_key(p);
  float pg[NPL], pb[NPL], gm[NPL];
  ldv<NPL>(q.gamma + c0, gm);
#pragma unroll
  for (int i = 0; i < NPL; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const uint32_t key = (q.gb && q.bd.p > 0.f) ? drop_key(q.bd) : 0u;
  const TX* x = (const TX*)q.x;
  const TR* dres = (const TR*)q.dres;
  TDX* dx = (TDX*)q.dx;
  TGB* gb = (TGB*)q.gb;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = (int64_t)blockIdx.x * LNB_ROWS + w * RPW + rr;
    if (row < p.M) {
      const float mu = q.mean[row], rs = q.rstd[row];
      float xv[NPL], d[NPL];
      reduce_row<NPL, TC>(p, dkey, al, row, c0, d);
      ldv<NPL>(x + row * D + c0, xv);
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
        if (q.bd.p > 0.f) drop_mul_n<NPL>(q.bd, key, (uint64_t)(row * D + c0), dm);
#pragma unroll
        for (int i = 0; i < NPL; ++i) o[i] *= q.bscale * (q.bd.p > 0.f ? dm[i] : 1.f);
        stv<NPL>(gb + row * D + c0, o);
      }
    }
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < NPL; ++i) sp[w][c0 + i] = pass == 0 ? pg[i] : pb[i];
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < WAVES; ++k) a += sp[k][c];
      q.part[(int64_t)blockIdx.x * 2 * D + pass * D + c] = a;
    }
    __syncthreads();
  }
}

// the fused reductions take: batch 1, 4-wide partial rows, no bias rowsum, D = N in 256 / 512
bool fusable(const GemmP& p) {
  return p.batch == 1 && p.v4 && !p.rs_ws && (p.N == 256 || p.N == 512) && p.ldc % 4 == 0;
}

int launch_fwd(const GemmP& p, const void* ctx, hipStream_t st) {
  const LnFwdPost& q = *(const LnFwdPost*)ctx;
  if (!fusable(p)) return 0;
  const unsigned nb = (unsigned)cdiv(p.M, LNF_WAVES);
  const bool yb = q.y_dtype == LASR_BF16;
  if (p.N == 256) {
    if (yb) splitk_reduce_ln_fwd_kernel<4, bf16_t><<<nb, 256, 0, st>>>(p, q);
    else splitk_reduce_ln_fwd_kernel<4, float><<<nb, 256, 0, st>>>(p, q);
  } else {
    if (yb) splitk_reduce_ln_fwd_kernel<8, bf16_t><<<nb, 256, 0, st>>>(p, q);
    else splitk_reduce_ln_fwd_kernel<8, float><<<nb, 256, 0, st>>>(p, q);
  }
  return 1;
}

// the decoder's instance: bf16 dln, fp32 x / dres / dx, bf16 gb (or none); other dtype
// combinations run the two launches
int launch_bwd(const GemmP& p, const void* ctx, hipStream_t st) {
  const LnBwdPost& q = *(const LnBwdPost*)ctx;
  if (!fusable(p) || q.x_dtype != LASR_F32 || q.dx_dtype != LASR_F32 || (q.dres && q.dres_dtype != LASR_F32) ||
      (q.gb && q.gb_dtype != LASR_BF16))
    return 0;
  const unsigned nb = (unsigned)cdiv(p.M, LNB_ROWS);
  if (p.N == 256) {
    splitk_reduce_ln_bwd_kernel<4, bf16_t, float, float, float, bf16_t><<<nb, 64 * lnb_waves<4>(), 0, st>>>(p, q);
  } else {
    splitk_reduce_ln_bwd_kernel<8, bf16_t, float, float, float, bf16_t><<<nb, 64 * lnb_waves<8>(), 0, st>>>(p, q);
  }
  return 1;
}

struct QbiasPost {
  const void* dqu;
  const void* dqv;
  int dt;
  int64_t rows;
  int D;
  void* dqkv;
  int64_t ld;
  float* part;
  int gx, gy;  // lasr_qbias_bwd's grid
};

// blocks [0, nred): the split-K reduction with nred blocks; [nred, nred + gx*gy): qbias blocks
template <typename TC, typename TQ>
__global__ __launch_bounds__(256) void splitk_reduce_qbias_kernel(GemmP p, int nred, QbiasPost q) {
  const int b = blockIdx.x;
  if (b < nred) {
    splitk_reduce_body<TC>(p, b, nred);
    return;
  }
  const int k = b - nred;
  qbias_bwd_body<TQ>((const TQ*)q.dqu, (const TQ*)q.dqv, q.rows, q.D, (TQ*)q.dqkv, q.ld, q.part, k % q.gx, k / q.gx);
}

// the reduction's block count as lasr_gemm sizes it
int reduce_blocks(const GemmP& p) {
  const int64_t total = (int64_t)p.M * p.N * p.batch;
  return (int)std::min<int64_t>(cdiv(p.v4 ? total / 4 : total, 256), 4096);
}

int launch_qbias(const GemmP& p, const void* ctx, hipStream_t st) {
  const QbiasPost& q = *(const QbiasPost*)ctx;
  const int nred = reduce_blocks(p);
  const unsigned nb = (unsigned)(nred + q.gx * q.gy);
  if (q.dt == LASR_BF16) splitk_reduce_qbias_kernel<bf16_t, bf16_t><<<nb, 256, 0, st>>>(p, nred, q);
  else splitk_reduce_qbias_kernel<float, float><<<nb, 256, 0, st>>>(p, nred, q);
  return 1;
}

}  // namespace

extern "C" int lasr_gemm_qbias_bwd(const lasr_gemm_args* a, const void* dqu, const void* dqv, int dt, int B, int T,
                                   int H, int dk, void* dqkv, int64_t ld, float* ws, int64_t ws_floats, void* stream) {
  LASR_CHECK_ARG(a && dqu && dqv && dqkv && ws, "lasr_gemm_qbias_bwd: null argument");
  LASR_CHECK_ARG(dt == a->c_dtype && (dt == LASR_F32 || dt == LASR_BF16), "lasr_gemm_qbias_bwd: C and dq dtypes differ");
  const int64_t rows = (int64_t)B * T;
  const int D = H * dk;
  const int64_t nchunk = cdiv(rows, QB_ROWS);
  LASR_CHECK_ARG(ws_floats >= nchunk * 2 * D && nchunk <= 65535, "lasr_gemm_qbias_bwd: workspace / rows");
  LASR_CHECK_ARG(D % 2 == 0 && ld % 2 == 0, "lasr_gemm_qbias_bwd: D and ld must be even");
  QbiasPost q = {dqu, dqv, dt, rows, D, dqkv, ld, ws, (int)cdiv(D, 2 * QB_CP), (int)nchunk};
  GemmRowPost post = {launch_qbias, &q, 0};
  const int rc = gemm_run(a, stream, &post);
  if (rc || post.done) return rc;
  return lasr_qbias_bwd(dqu, dqv, dt, B, T, H, dk, dqkv, ld, nullptr, nullptr, ws, ws_floats, stream);
}

extern "C" int lasr_gemm_ln_fwd(const lasr_gemm_args* a, const float* gamma, const float* beta, float eps, void* y,
                                int y_dtype, float* mean, float* rstd, void* stream) {
  LASR_CHECK_ARG(a && gamma && beta && y && mean && rstd, "lasr_gemm_ln_fwd: null argument");
  LASR_CHECK_ARG(a->c_dtype == LASR_F32 && (a->batch <= 1) && a->ldc == a->N && !a->rowsum,
                 "lasr_gemm_ln_fwd: fp32 C with contiguous rows, batch 1, no rowsum");
  LASR_CHECK_ARG(y_dtype == LASR_F32 || y_dtype == LASR_BF16, "lasr_gemm_ln_fwd: bad y_dtype");
  LnFwdPost q = {gamma, beta, eps, y, y_dtype, mean, rstd};
  GemmRowPost post = {launch_fwd, &q, 0};
  const int rc = gemm_run(a, stream, &post);
  if (rc || post.done) return rc;
  return lasr_layernorm_fwd(a->C, LASR_F32, a->M, a->N, gamma, beta, eps, y, y_dtype, mean, rstd, nullptr, 0, 0.f, 0,
                            stream);
}

extern "C" int lasr_gemm_ln_bwd(const lasr_gemm_args* a, const void* x, int x_dtype, const float* gamma,
                                const float* mean, const float* rstd, const void* dres, int dres_dtype, void* dx,
                                int dx_dtype, float* part, int64_t part_floats, void* gb, int gb_dtype, float bscale,
                                float bp, uint64_t bseed, void* stream) {
  LASR_CHECK_ARG(a && x && gamma && mean && rstd && dx && part, "lasr_gemm_ln_bwd: null argument");
  LASR_CHECK_ARG((a->batch <= 1) && a->ldc == a->N && !a->rowsum,
                 "lasr_gemm_ln_bwd: C with contiguous rows, batch 1, no rowsum");
  const int64_t nblk = cdiv(a->M, LNB_ROWS);
  LASR_CHECK_ARG(part_floats >= nblk * 2 * a->N, "lasr_gemm_ln_bwd: partial rows need %lld floats",
                 (long long)(nblk * 2 * a->N));
  LnBwdPost q = {x, x_dtype, gamma, mean, rstd, dres, dres_dtype, dx, dx_dtype, part, gb, gb_dtype, bscale,
                 mkdrop(bp, bseed)};
  GemmRowPost post = {a->c_dtype == LASR_BF16 ? launch_bwd : nullptr, &q, 0};
  if (!post.launch) post.launch = [](const GemmP&, const void*, hipStream_t) { return 0; };
  const int rc = gemm_run(a, stream, &post);
  if (rc || post.done) return rc;
  return lasr_layernorm_bwd(x, x_dtype, a->C, a->c_dtype, a->M, a->N, gamma, mean, rstd, dres, dres_dtype, dx,
                            dx_dtype, nullptr, nullptr, part, part_floats, gb, gb_dtype, bscale, bp, bseed, stream);
}
