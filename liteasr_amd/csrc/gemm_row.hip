// Full-row GEMM tiles with the LayerNorm in the epilogue (lasr_linear_res_ln,
// lasr_linear_dx_ln_bwd; include/liteasr_hip.h).
//
// A Conformer layer's residual projections (FFN fc2, attention linear_out, pointwise_conv2:
// liteasr/nets/conformer_layer.py:37-78, feed_forward.py:19, attention.py:58,
// conformer_convolution.py:55) write the d-wide residual stream, and the very next op is the
// following sub-block's LayerNorm over that row (layer_norm.py:20).  Their backward mirror is
// the input-gradient GEMM of each sub-block's first projection, followed by that LayerNorm's
// backward.  A tile that owns whole rows (RB rows x all D = N columns) can finish the norm in
// its own epilogue: the separate LayerNorm launch and its re-read of the row disappear.
//
// Tile: RB = 32 rows x D (256 or 512) columns, 512 threads = 8 waves (wave w owns rows
// 16 (w / 4) .. +15 and columns [(w % 4) D/4, +D/4): each output is accumulated by ONE wave
// over k in order, as in the generic GEMM), v_mfma_f32_16x16x32_bf16 with the operands
// swapped (acc = C^T fragments, as gemm_glds_tile), operands streamed HBM -> LDS by
// global_load_lds_dwordx4 into an S-stage ring of 64-deep stages (two 32-deep sub-tiles with
// the images, swizzles and fragment reads of tile.h), one counted vmcnt + barrier per stage.
// One workgroup per CU (M = 7968 -> 249 workgroups); two waves per SIMD overlap one wave's
// LDS-DMA issue and waits with the other's fragment reads and MFMAs.
//
// Epilogue: the fp32 tile is staged in LDS; each wave then finishes 4 rows, one row per
// step with lane l owning columns [l D/64, (l+1) D/64) -- the lane layout of ln_fwd_kernel /
// ln_bwd_kernel (norm.hip) -- so every output is BIT-IDENTICAL to the two-launch path:
//  forward:  out = res + s * dropout(acc + bias) (gemm epilogue order), y1 = LN1(out) with
//            ln_fwd's arithmetic, optionally z = LN2(y1) with ln2_fwd's;
//  backward: dln = bf16(acc) (the dX GEMM's bf16 output), then ln_bwd's arithmetic per row
//            (dx = dres + LN'(dln), gb = bscale * dropout(dx)), and the gamma / beta partial
//            rows in ln_bwd's block layout ([cdiv(M,16)][2D], each 16-row block summed in row
//            order), so the caller's deferred reduction is unchanged.
#include "gemm_kernel.h"
#include "ln_math.h"

namespace {

constexpr int RB = 32;  // rows per workgroup
constexpr int BK = 32;  // k depth of one sub-tile image
constexpr int KS = 2;   // sub-tiles per ring stage (64-deep stages)

template <int D>
struct RowCfg {
  static constexpr int NT = 512;          // 8 waves: 2 (row halves) x 4 (column quarters)
  static constexpr int WN = D / 4;        // columns per wave
  static constexpr int FN = WN / 16;      // 16-column fragments per wave (one 16-row fragment)
  static constexpr int NPL = D / 64;      // epilogue columns per lane
  static constexpr int RW = RB / 8;       // epilogue rows per wave (row it * 8 + wave)
  static constexpr int TILE = (RB + D) * BK;   // elements of one 32-deep sub-tile (A then B)
  static constexpr int STAGE = KS * TILE;
  static constexpr int S = D == 256 ? 4 : 2;   // ring stages (LDS: 144 / 136 KiB)
  // glds per thread per stage: B = KS * D * 4 16-B units over all 512 threads; A = KS * RB * 4
  // = 256 units, one per thread of waves 0-3
  static constexpr int GLB = KS * D * 4 / NT;
  static constexpr int GLA = GLB + 1;
  static constexpr int LDC = D + 4;       // fp32 staging row stride
  // rows per wave of ln_bwd_kernel (norm.hip LnbCfg: 16 waves x 1 row up to D = 512): its
  // dgamma/dbeta block partials sum per-wave row groups in order
  static constexpr int RPW = NPL <= 8 ? 1 : 2;
  static constexpr int SMEM = S * STAGE * 2;
  static_assert(SMEM >= (RB * LDC + RB * D) * 4, "epilogue staging must fit the ring");
};

struct RowP {
  int M, K;
  const bf16_t* A;
  int64_t lda;
  const bf16_t* W;
  int64_t ldw;
  const float* g1;
  const float* b1;
  float eps;
  float* mean1;
  float* rstd1;
  // forward
  const float* bias;
  const float* res;
  float res_scale;
  DropCfg drop;
  float* out;
  void* y1;
  const float* g2;
  const float* b2;
  bf16_t* y2;
  float* mean2;
  float* rstd2;
  // backward
  const float* x;
  const float* dres;
  float* dx;
  bf16_t* gb;
  float bscale;
  DropCfg bd;
  float* part;
};

// A tile (32 rows x 64 k, K-contiguous) of one ring stage: one 16-B unit per thread of waves
// 0-3, the two 32-deep sub-tile images of glds_tile<32, true> (unit P of sub-tile u at
// u*TILE + P*8).
template <int D>
LASR_DEV void issue_a(const RowP& p, int m0, int k0, bf16_t* stage, int tid) {
  const int u = tid >> 7, P = tid & 127, r = P >> 2, c = (P & 3) ^ swz(r);
  const int gr = min(m0 + r, p.M - 1);
  const bf16_t* src = p.A + (int64_t)gr * p.lda + k0 + u * BK + c * 8;
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(stage + u * RowCfg<D>::TILE + (P & ~63) * 8), 16, 0,
                                   0);
}

// glds_tile (tile.h) issued by 512 threads: the same image, unit P = i * 512 + tid.
template <int R_TILE, bool KC>
LASR_DEV void glds_tile512(const bf16_t* base, int64_t ld, int R, int k0, bf16_t* dst, int tid) {
  constexpr int PER = R_TILE * 4 / 512;
  const int wid = tid >> 6;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int P = i * 512 + tid;
    const bf16_t* src;
    if (KC) {
      const int r = P >> 2, c = (P & 3) ^ swz(r);
      src = base + (int64_t)min(r, R - 1) * ld + k0 + c * 8;
    } else {
      constexpr int CPR = R_TILE / 8;
      const int k = P / CPR, ps = P % CPR;
      const int ls = ((((ps >> 1) ^ htr<R_TILE>(k))) << 1) | (ps & 1);
      src = base + (int64_t)(k0 + k) * ld + min(ls * 8, ((R + 7) & ~7) - 8);
    }
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (i * 512 + wid * 64) * 8), 16, 0, 0);
  }
}

template <int D, bool BKC>
LASR_DEV void row_mainloop(const RowP& p, int m0, bf16_t* smem) {
  using Cf = RowCfg<D>;
  constexpr int FN = Cf::FN, S = Cf::S;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  f32x4 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    bf16_t* dst = smem + (t % S) * Cf::STAGE;
    const int k0 = t * (KS * BK);
    if (wid < 4) issue_a<D>(p, m0, k0, dst, tid);
#pragma unroll
    for (int u = 0; u < KS; ++u) glds_tile512<D, BKC>(p.W, p.ldw, D, k0 + u * BK, dst + u * Cf::TILE + RB * BK, tid);
  };
  auto compute = [&](const bf16_t* cur) {
    bf16x8 bfr[FN];
    v2i rb[2 * FN];
    const bf16x8 af = frag<RB, true>(cur, wr * 16, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BKC) bfr[j] = frag<D, true>(cur + RB * BK, wc * Cf::WN + j * 16, lane);
      else frag_tr_raw<D>(cur + RB * BK, wc * Cf::WN + j * 16, lane, rb + 2 * j);
    }
    if constexpr (!BKC) {
      tie_lgkm<2 * FN>(rb);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_from_raw(rb + 2 * j);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[j], 0, 0, 0);
  };

  const int nst = p.K / (KS * BK);  // host-checked: K % 64 == 0
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nst) issue(t);
  for (int kt = 0; kt < nst; ++kt) {
    const int after = min(S - 2, nst - 1 - kt);
    if (wid < 4) wait_ring<S, Cf::GLA>(after);  // waves 0-3 also carry the A tile
    else wait_ring<S, Cf::GLB>(after);
    lds_barrier();
    if (kt + S - 1 < nst) issue(kt + S - 1);
#pragma unroll
    for (int u = 0; u < KS; ++u) compute(smem + (kt % S) * Cf::STAGE + u * Cf::TILE);
  }
  __syncthreads();  // every wave is done with the ring: the epilogue reuses it
  // stage the tile (fp32, row stride LDC): C^T fragment j of lane l is row wr*16 + (l & 15),
  // columns j*16 + 4 (l >> 4) .. +3 of the wave's column block
  float* cs = reinterpret_cast<float*>(smem);
  const int cl = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < FN; ++j) *(f32x4*)(cs + (wr * 16 + cl) * Cf::LDC + wc * Cf::WN + j * 16 + rq) = acc[j];
  __syncthreads();
}

template <int D, typename TY1>
__global__ __launch_bounds__(512, 1) void row_res_ln_kernel(RowP p) {
  using Cf = RowCfg<D>;
  constexpr int NPL = Cf::NPL, RW = Cf::RW;  // epilogue rows per wave: it * 8 + wid
  __shared__ __attribute__((aligned(16))) char smem_raw[Cf::SMEM];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  const int m0 = blockIdx.x * RB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c0 = lane * NPL;
  // the epilogue's per-row inputs do not depend on the GEMM: load them before the main loop
  // (one wave per SIMD: a load issued per epilogue row would expose its full latency)
  float rv[RW][NPL];
#pragma unroll
  for (int it = 0; it < RW; ++it) ldv<NPL>(p.res + (int64_t)min(m0 + it * 8 + wid, p.M - 1) * D + c0, rv[it]);
  float bv[NPL], g1[NPL], b1[NPL], g2[NPL], b2[NPL];
  if (p.bias) ldv<NPL>(p.bias + c0, bv);
  else
#pragma unroll
    for (int q = 0; q < NPL; ++q) bv[q] = 0.f;
  ldv<NPL>(p.g1 + c0, g1);
  ldv<NPL>(p.b1 + c0, b1);
  if (p.g2) {
    ldv<NPL>(p.g2 + c0, g2);
    ldv<NPL>(p.b2 + c0, b2);
  }
  row_mainloop<D, true>(p, m0, smem);

  const float* cs = reinterpret_cast<const float*>(smem_raw);
  const bool drop = p.drop.p > 0.f;
  const uint32_t key = drop ? drop_key(p.drop) : 0u;
#pragma unroll
  for (int it = 0; it < RW; ++it) {
    const int r = it * 8 + wid, m = m0 + r;
    if (m < p.M) {
      float v[NPL];
#pragma unroll
      for (int q = 0; q < NPL; ++q) v[q] = cs[r * Cf::LDC + c0 + q] * 1.f + bv[q];
      // epi_core's order: dropout (one draw per column pair), then the residual
      if (drop) {
        const uint32_t km = drop_keep_mask<NPL>(p.drop, key, (uint64_t)m * D + c0);
#pragma unroll
        for (int q = 0; q < NPL; ++q) v[q] *= (km >> q) & 1u ? p.drop.scale : 0.f;
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q) v[q] = rv[it][q] + p.res_scale * v[q];
      stv<NPL>(p.out + (int64_t)m * D + c0, v);
      float o[NPL], mu, rs;
      ln_fwd_row<D, NPL>(v, g1, b1, p.eps, o, mu, rs);
      if (lane == 0) { p.mean1[m] = mu; p.rstd1[m] = rs; }
      stv<NPL>((TY1*)p.y1 + (int64_t)m * D + c0, o);
      if (p.g2) {  // ln2_fwd_kernel's second pass on the fp32 y1 row
        float z[NPL];
        ln_fwd_row<D, NPL>(o, g2, b2, p.eps, z, mu, rs);
        if (lane == 0) { p.mean2[m] = mu; p.rstd2[m] = rs; }
        stv<NPL>(p.y2 + (int64_t)m * D + c0, z);
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(512, 1) void row_dx_ln_bwd_kernel(RowP p) {
  using Cf = RowCfg<D>;
  constexpr int NPL = Cf::NPL, RPW = Cf::RPW, LDC = Cf::LDC, NG = Cf::RW;  // rows per wave: it * 8 + wid
  static_assert(RPW == 1, "row groups of more than one row: D > 512 is not instantiated");
  __shared__ __attribute__((aligned(16))) char smem_raw[Cf::SMEM];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  const int m0 = blockIdx.x * RB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c0 = lane * NPL;
  // per-row inputs first (see row_res_ln_kernel): x, dres, mean, rstd of the wave's rows
  float xv[NG][NPL], rv[NG][NPL], mu[NG], rs[NG];
#pragma unroll
  for (int it = 0; it < NG; ++it) {
    const int m = min(m0 + it * 8 + wid, p.M - 1);
    ldv<NPL>(p.x + (int64_t)m * D + c0, xv[it]);
    if (p.dres) ldv<NPL>(p.dres + (int64_t)m * D + c0, rv[it]);
    mu[it] = p.mean1[m];
    rs[it] = p.rstd1[m];
  }
  float gm[NPL];
  ldv<NPL>(p.g1 + c0, gm);
  row_mainloop<D, false>(p, m0, smem);

  // dgamma rows overwrite the staged rows they came from (only the wave that read a row
  // writes it); dbeta rows go to pb
  float* cs = reinterpret_cast<float*>(smem_raw);
  float* pb = cs + RB * LDC;
  const bool bdrop = p.gb && p.bd.p > 0.f;
  const uint32_t key = bdrop ? drop_key(p.bd) : 0u;
#pragma unroll
  for (int it = 0; it < NG; ++it) {
    const int r = it * 8 + wid, m = m0 + r;  // one row = one wave of ln_bwd_kernel
    float pg[NPL], pbv[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) { pg[i] = 0.f; pbv[i] = 0.f; }
    if (m < p.M) {
      float d[NPL], o[NPL];
#pragma unroll
      for (int i = 0; i < NPL; ++i) d[i] = bf2f(f2bf(cs[r * LDC + c0 + i]));  // the dX GEMM's bf16 dln
      if (p.dres) ln_bwd_row<D, NPL, true>(xv[it], d, gm, mu[it], rs[it], rv[it], pg, pbv, o);
      else ln_bwd_row<D, NPL, false>(xv[it], d, gm, mu[it], rs[it], rv[it], pg, pbv, o);
      stv<NPL>(p.dx + (int64_t)m * D + c0, o);
      if (p.gb) {
        float dm[NPL];
        if (bdrop) drop_mul_n<NPL>(p.bd, key, (uint64_t)(m * D + c0), dm);
#pragma unroll
        for (int i = 0; i < NPL; ++i) o[i] *= p.bscale * (bdrop ? dm[i] : 1.f);
        stv<NPL>(p.gb + (int64_t)m * D + c0, o);
      }
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      cs[r * LDC + c0 + i] = pg[i];
      pb[r * D + c0 + i] = pbv[i];
    }
  }
  __syncthreads();
  // ln_bwd_kernel's block partials: each 16-row block's rows summed in order from 0
  // thread t: half h = t / D (D = 256), or both halves (D = 512), column t % D
#pragma unroll
  for (int hh = 0; hh < RB / 16 * D / Cf::NT; ++hh) {
    const int h = D == 256 ? (int)(threadIdx.x >> 8) : hh, c = threadIdx.x % D;
    if (m0 + h * 16 >= p.M) continue;
    float* dst = p.part + (int64_t)(m0 / 16 + h) * 2 * D;
    {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        a += cs[(h * 16 + k) * LDC + c];
        b += pb[(h * 16 + k) * D + c];
      }
      dst[c] = a;
      dst[D + c] = b;
    }
  }
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

}  // namespace

static int row_common(const lasr_row_ln_args* a, RowP& p, const char* who) {
  LASR_CHECK_ARG(a != nullptr, "%s: null args", who);
  LASR_CHECK_ARG(a->D == 256 || a->D == 512, "%s: D=%d (256 or 512)", who, a->D);
  LASR_CHECK_ARG(a->M >= 0 && a->K > 0 && a->K % 64 == 0, "%s: K=%d must be a positive multiple of 64", who, a->K);
  LASR_CHECK_ARG(a->A && a->W && al16(a->A) && al16(a->W) && a->lda % 8 == 0 && a->ldw % 8 == 0 &&
                     a->lda >= a->K,
                 "%s: A / W must be 16-B aligned with row strides a multiple of 8", who);
  LASR_CHECK_ARG(a->gamma1 && a->mean1 && a->rstd1 && al16(a->gamma1), "%s: gamma1 / mean1 / rstd1 required", who);
  p = RowP{};
  p.M = a->M; p.K = a->K;
  p.A = (const bf16_t*)a->A; p.lda = a->lda;
  p.W = (const bf16_t*)a->W; p.ldw = a->ldw;
  p.g1 = a->gamma1; p.b1 = a->beta1; p.eps = a->eps; p.mean1 = a->mean1; p.rstd1 = a->rstd1;
  return LASR_OK;
}

extern "C" int lasr_linear_res_ln(const lasr_row_ln_args* a, void* stream) {
  RowP p;
  int rc = row_common(a, p, "lasr_linear_res_ln");
  if (rc) return rc;
  LASR_CHECK_ARG(a->ldw >= a->K, "lasr_linear_res_ln: W is [D, K] (ldw >= K)");
  LASR_CHECK_ARG(a->res && a->out && a->y1 && a->beta1 && al16(a->res) && al16(a->out) && al16(a->y1) &&
                     al16(a->beta1) && (!a->bias || al16(a->bias)),
                 "lasr_linear_res_ln: res / out / y1 / beta1 required, 16-B aligned");
  LASR_CHECK_ARG(a->y1_dtype == LASR_BF16 || a->y1_dtype == LASR_F32, "lasr_linear_res_ln: y1 bf16 or fp32");
  LASR_CHECK_ARG(!a->gamma2 || (a->y1_dtype == LASR_F32 && a->beta2 && a->y2 && a->mean2 && a->rstd2 &&
                                al16(a->gamma2) && al16(a->beta2) && al16(a->y2)),
                 "lasr_linear_res_ln: the chained norm needs an fp32 y1 and gamma2 / beta2 / y2 / mean2 / rstd2");
  if (a->M == 0) return LASR_OK;
  p.bias = a->bias; p.res = a->res; p.res_scale = a->res_scale;
  p.drop = mkdrop(a->drop_p, a->drop_seed);
  p.out = a->out; p.y1 = a->y1;
  p.g2 = a->gamma2; p.b2 = a->beta2; p.y2 = (bf16_t*)a->y2; p.mean2 = a->mean2; p.rstd2 = a->rstd2;
  const dim3 grid((unsigned)cdiv(a->M, RB));
  hipStream_t st = (hipStream_t)stream;
  if (a->D == 256) {
    if (a->y1_dtype == LASR_F32) row_res_ln_kernel<256, float><<<grid, 512, 0, st>>>(p);
    else row_res_ln_kernel<256, bf16_t><<<grid, 512, 0, st>>>(p);
  } else {
    if (a->y1_dtype == LASR_F32) row_res_ln_kernel<512, float><<<grid, 512, 0, st>>>(p);
    else row_res_ln_kernel<512, bf16_t><<<grid, 512, 0, st>>>(p);
  }
  return lasr_check_launch("lasr_linear_res_ln");
}

extern "C" int lasr_linear_dx_ln_bwd(const lasr_row_ln_args* a, void* stream) {
  RowP p;
  int rc = row_common(a, p, "lasr_linear_dx_ln_bwd");
  if (rc) return rc;
  LASR_CHECK_ARG(a->ldw >= a->D, "lasr_linear_dx_ln_bwd: W is [K, D] (ldw >= D)");
  LASR_CHECK_ARG(!a->dgamma == !a->dbeta, "lasr_linear_dx_ln_bwd: dgamma and dbeta together (or neither)");
  LASR_CHECK_ARG(a->x && a->dx && a->part && al16(a->x) && al16(a->dx) && al16(a->part) &&
                     (!a->dres || al16(a->dres)) && (!a->gb || al16(a->gb)),
                 "lasr_linear_dx_ln_bwd: x / dx / part required, 16-B aligned");
  if (a->M == 0) return LASR_OK;
  p.x = a->x; p.dres = a->dres; p.dx = a->dx; p.gb = (bf16_t*)a->gb; p.bscale = a->bscale;
  p.bd = mkdrop(a->bp, a->bseed);
  p.part = a->part;
  const dim3 grid((unsigned)cdiv(a->M, RB));
  hipStream_t st = (hipStream_t)stream;
  if (a->D == 256) row_dx_ln_bwd_kernel<256><<<grid, 512, 0, st>>>(p);
  else row_dx_ln_bwd_kernel<512><<<grid, 512, 0, st>>>(p);
  rc = lasr_check_launch("lasr_linear_dx_ln_bwd");
  if (rc || !a->dgamma) return rc;
  // lasr_layernorm_bwd's own reduction of the same partial rows
  return lasr_reduce_cols(a->part, (int)cdiv(a->M, 16), 2 * a->D, a->dgamma, a->dbeta, a->D, 1, st);
}
