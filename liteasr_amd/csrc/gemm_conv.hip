// Subsampling conv2 as implicit GEMMs (lasr_conv2_gemm): the gather instances of the LDS-DMA
// kernel (gemm_kernel.h) and their host launcher.
#include "gemm_kernel.h"

// ========================= subsampling conv2, implicit GEMM ======================
// (lasr_conv2_gemm, include/liteasr_hip.h) Same LDS-DMA kernel, gather instances G_FWD /
// G_DW / G_DX: im2col(y1) is never materialised, and the data gradient is scattered straight
// into dy1 per output parity class (no dcol, no col2im).  Replaces the reference's
// nn.Conv2d(C, C, 3, 2) forward and backward (liteasr/nets/subsampling.py:31-47).
static GemmP conv_params(const lasr_conv2_args* a) {
  GemmP p;
  memset(&p, 0, sizeof(p));
  p.batch = 1;
  p.batch_div = 1;
  p.alpha = 1.f;
  p.res_scale = 1.f;
  p.split_k = 1;
  p.drop = mkdrop(0.f, 0);
  ConvG& g = p.cv;
  g.B = a->B; g.T1 = a->T1; g.F1 = a->F1; g.C = a->C;
  g.T2 = (a->T1 - 3) / 2 + 1;
  g.F2 = (a->F1 - 3) / 2 + 1;
  g.M2 = g.B * g.T2 * g.F2;
  g.q32 = 32 / g.F2;
  g.r32 = 32 % g.F2;
  return p;
}

// The weight gradient on 256 x 256 tiles with 8 waves and 64-deep ring stages
// (gemm_bf16_glds_kernel NW = 8) when C % 256 == 0: one 512-thread workgroup per CU, K split
// so the 9 tiles fill the 256 CUs once (28 slices at config 2), half the LDS-DMA ingest per
// MFMA of the 4-wave 128 x 128 tiles: 365 -> 236 us standalone, 352 -> 186 us in the step
// (tools/conv2_bench.py, profiles/r03).  Forward and data gradient stay on the 4-wave
// 128 x 256 tiles: their 8-wave variants (256 x 256 with 64- or 32-deep stages, 256 x 128)
// took 265-299 / 523-529 us against 262 / 468 (their 592-tile grids run 2.3 rounds of one
// workgroup per CU).
// The data gradient's four output parity classes in ONE launch: class i owns the blocks
// [start[i], start[i+1]) (starts multiples of 8: the XCD remap stays exact inside a class),
// heaviest class (4 taps) first.  One launch of ~4.9k workgroups instead of four of ~1.2k
// (each 2.3-2.4 rounds of the 512 resident workgroups, so every class paid its own
// partially filled last round).  Same tiles, same k order per output as the per-class
// launches it replaced (profiles/r03/conv2_dx_ab.json: hashes equal).
struct DxClasses {
  int start[5];
  int M[4], K[4];
  int rb[4];  // DX_W1: first conv1 partial row of each class (its 128-row tiles in order)
};

template <int BN, int EPI = EPI_RT>
__global__ __launch_bounds__(256, 2) void conv2_dx_kernel(GemmP p, DxClasses c) {
  const int blk = blockIdx.x;
  int i = 0;
  for (int j = 1; j < 4; ++j)
    if (blk >= c.start[j]) i = j;
  GemmP q = p;
  q.cv.cls = i;
  q.M = c.M[i];
  q.K = c.K[i];
  q.kchunk = c.K[i];
  q.cv.w1rb = c.rb[i];
  const int ntx = p.N / BN, nty = (q.M + 127) / 128, ntile = ntx * nty;
  const int local = blk - c.start[i];
  if (local >= ntile) return;  // alignment padding
  const int wg = xcd_remap(local, ntile);
  gemm_glds_tile<128, BN, true, false, bf16_t, 3, G_DX, 1, 4, EPI>(q, wg % ntx, wg / ntx, 0);
}

// The conv1 weight-gradient partials of LASR_CONV2_DX_W1 ([rows][10][C], one row per 128-row
// tile of the four classes) summed in fixed order: groups of W1_GROUP rows here (coalesced
// 1-KB row reads, ~800 workgroups), then the group sums by lasr_reduce_cols.
constexpr int W1_GROUP = 64;
__global__ __launch_bounds__(256) void w1_group_sum_kernel(const float* __restrict__ part, int P, int N,
                                                           float* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
  if (n >= N) return;
  const int p0 = g * W1_GROUP, p1 = min(P, p0 + W1_GROUP);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  for (int p = p0; p < p1; p += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p + k < p1 ? part[(int64_t)(p + k) * N + n] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += v[k];
  }
  out[(int64_t)g * N + n] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

static int64_t dx_tile_rows(int B, int T1, int F1) {
  int64_t rows = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int pt = cls >> 1, pf = cls & 1;
    rows += cdiv((int64_t)B * ((T1 - pt + 1) >> 1) * ((F1 - pf + 1) >> 1), 128);
  }
  return rows;
}

// partials [P][10C], group sums [cdiv(P, W1_GROUP)][10C], total [10C]
extern "C" int64_t lasr_conv2_dx_w1_workspace(int B, int T1, int F1, int C) {
  if (B <= 0 || T1 < 3 || F1 < 3 || C <= 0) return 0;
  const int64_t P = dx_tile_rows(B, T1, F1);
  return (P + cdiv(P, W1_GROUP) + 1) * 10 * (int64_t)C * 4;
}

extern "C" int lasr_conv2_gemm(const lasr_conv2_args* a, void* stream) {
  LASR_CHECK_ARG(a != nullptr, "lasr_conv2_gemm: null args");
  LASR_CHECK_ARG(a->mode == LASR_CONV2_FWD || a->mode == LASR_CONV2_DW || a->mode == LASR_CONV2_DX ||
                 a->mode == LASR_CONV2_DX_W1, "lasr_conv2_gemm: bad mode");
  LASR_CHECK_ARG(a->B > 0 && a->T1 >= 3 && a->F1 >= 3 && a->C > 0 && a->C % 128 == 0,
                 "lasr_conv2_gemm: needs B > 0, T1, F1 >= 3 and C % 128 == 0");
  LASR_CHECK_ARG((int64_t)a->B * a->T1 * a->F1 * a->C < (1LL << 31) && 9LL * a->C * a->C < (1LL << 31),
                 "lasr_conv2_gemm: tensors past 2^31 elements");
  const bool w1 = a->mode == LASR_CONV2_DX_W1;
  LASR_CHECK_ARG(a->y1 && aligned16(a->y1) && (w1 || (a->out && aligned16(a->out))), "lasr_conv2_gemm: y1/out");
  GemmP p = conv_params(a);
  const ConvG& g = p.cv;
  const int C = a->C;
  const int64_t kpad = cdiv(g.M2, 32) * 32;
  if (a->mode != LASR_CONV2_FWD)
    LASR_CHECK_ARG(a->dy2 && aligned16(a->dy2) && a->dy2_rows >= kpad && a->dy2_rows >= g.M2 + 1,
                   "lasr_conv2_gemm: dy2 needs >= max(roundup32(M2), M2 + 1) rows, the tail zero");
  if (a->mode != LASR_CONV2_DW)
    LASR_CHECK_ARG(a->w2p && aligned16(a->w2p), "lasr_conv2_gemm: w2p");
  hipStream_t st = (hipStream_t)stream;
  const int BN = C % 256 == 0 ? 256 : 128;
  const bool wide = BN == 256;
  p.c_vec = 1;
  if (a->mode == LASR_CONV2_FWD) {
    LASR_CHECK_ARG(a->bias && aligned16(a->bias), "lasr_conv2_gemm: bias");
    p.M = g.M2; p.N = C; p.K = 9 * C; p.kchunk = p.K;
    p.A = a->y1; p.lda_m = 9 * C; p.lda_k = 1;
    p.B = a->w2p; p.ldb_n = 9 * C; p.ldb_k = 1;
    p.C = a->out; p.ldc = C;
    p.bias = a->bias; p.bias_vec = 1; p.act = LASR_ACT_RELU;
    p.epi_mode = 0;
    // (64 x 256 tiles, 2366 of them: 355 vs 279 us, profiles/r03/conv2_dx_ab.json)
    dim3 grid((unsigned)(C / BN), (unsigned)cdiv(p.M, 128), 1);
    LASR_CHECK_ARG(grid.y <= 65535, "lasr_conv2_gemm: grid too large");
    if (BN == 256 && epi_code(p) == EPI_RELU)
      gemm_bf16_glds_kernel<128, 256, true, true, bf16_t, 3, 2, G_FWD, 1, 4, EPI_RELU><<<grid, 256, 0, st>>>(p);
    else if (BN == 256) gemm_bf16_glds_kernel<128, 256, true, true, bf16_t, 3, 2, G_FWD><<<grid, 256, 0, st>>>(p);
    else gemm_bf16_glds_kernel<128, 128, true, true, bf16_t, 3, 3, G_FWD><<<grid, 256, 0, st>>>(p);
    return lasr_check_launch("lasr_conv2_gemm/fwd");
  }
  if (a->mode == LASR_CONV2_DW) {
    p.M = C; p.N = 9 * C; p.K = (int)kpad;
    p.A = a->dy2; p.lda_m = 1; p.lda_k = C;
    p.B = a->y1; p.ldb_n = 1; p.ldb_k = 9 * C;
    p.C = a->out; p.ldc = 9 * C;
    p.epi_mode = 0; p.ws_vec = 1; p.v4 = 1;
    const int TM = wide ? 256 : 128, TN = wide ? 256 : 128;
    const int64_t tiles = (int64_t)(C / TM) * (9 * C / TN);
    int split = 1;
    const int kt = (int)(kpad / 32);
    if (wide)  // one 512-thread workgroup per CU: fill the 256 CUs once, no second round
      split = (int)std::max<int64_t>(1, std::min<int64_t>(256 / tiles, kt / 16));
    else while (tiles * split < 512 && kt / (split * 2) >= 16 && split * 2 <= 64) split *= 2;
    // fewer K slices when the workspace holds fewer partial slabs (never silently one slice)
    const int64_t per = ((int64_t)C * 9 * C + (a->rowsum ? C : 0)) * 4;
    const int64_t fit = a->workspace && aligned16(a->workspace) ? a->workspace_bytes / per : 0;
    if (split > fit) split = (int)std::max<int64_t>(1, fit);
    p.split_k = split;
    p.kchunk = split > 1 ? (int)(cdiv(cdiv(kpad, split), wide ? 64 : 32) * (wide ? 64 : 32)) : (int)kpad;
    if (split > 1) split = (int)cdiv(kpad, p.kchunk);  // no empty slice
    p.split_k = split;
    p.ws = (float*)a->workspace;
    p.rowsum = a->rowsum;
    if (a->rowsum && split > 1) p.rs_ws = p.ws + (int64_t)split * C * 9 * C;
    dim3 grid((unsigned)(9 * C / TN), (unsigned)(C / TM), (unsigned)split);
    if (wide) gemm_bf16_glds_kernel<256, 256, false, false, float, 2, 1, G_DW, 2, 8><<<grid, 512, 0, st>>>(p);
    else gemm_bf16_glds_kernel<128, 128, false, false, float, 3, 3, G_DW><<<grid, 256, 0, st>>>(p);
    int rc = lasr_check_launch("lasr_conv2_gemm/dw");
    if (!rc && split > 1) {
      const int64_t total = (int64_t)C * 9 * C;
      const int nblk = (int)std::min<int64_t>(cdiv(total / 4, 256), 4096);
      splitk_reduce_kernel<float><<<nblk, 256, 0, st>>>(p);
      rc = lasr_check_launch("lasr_conv2_gemm/dw_reduce");
    }
    return rc;
  }
  // LASR_CONV2_DX: the four output parity classes in one launch, heaviest (4 taps) first
  p.N = C;
  p.A = a->dy2; p.lda_m = C; p.lda_k = 1;
  p.B = a->w2p; p.ldb_n = 1; p.ldb_k = 9 * C;
  p.C = a->out; p.ldc = C;
  p.aux = a->y1; p.aux_dtype = LASR_BF16; p.ldaux = C; p.aux_act = LASR_ACT_RELU; p.aux_vec = 1;
  p.epi_mode = 1;
  p.cv.zero = (const bf16_t*)a->dy2 + (int64_t)g.M2 * C;
  DxClasses dc = {};
  int nb = 0, rows = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int pt = cls >> 1, pf = cls & 1;
    const int nI = (g.T1 - pt + 1) >> 1, nJ = (g.F1 - pf + 1) >> 1;
    dc.M[cls] = g.B * nI * nJ;
    dc.K[cls] = (pt ? 1 : 2) * (pf ? 1 : 2) * C;
    dc.start[cls] = nb;
    dc.rb[cls] = rows;
    rows += (int)cdiv(dc.M[cls], 128);
    nb += (int)(cdiv(cdiv(dc.M[cls], 128) * (C / BN), 8) * 8);
  }
  dc.start[4] = nb;
  if (w1) {
    // the conv1 weight gradient in the epilogue (conv1: x [B, T, F] -> y1, 3x3 stride 2)
    // (its own epilogue: the LASR_EPI_SPEC switch, which only selects between equal-result
    // store epilogues, does not apply)
    LASR_CHECK_ARG(BN == 256, "lasr_conv2_gemm/dx_w1: needs C %% 256 == 0");
    LASR_CHECK_ARG(a->x && a->dw1 && a->db1 && a->T >= 3 && a->F >= 3 && (a->T - 3) / 2 + 1 == g.T1 &&
                   (a->F - 3) / 2 + 1 == g.F1, "lasr_conv2_gemm/dx_w1: x [B, T, F] must give y1's T1 / F1");
    LASR_CHECK_ARG((int64_t)g.B * a->T * a->F < (1LL << 31), "lasr_conv2_gemm/dx_w1: x past 2^31 elements");
    const int64_t need = lasr_conv2_dx_w1_workspace(g.B, g.T1, g.F1, C);
    LASR_CHECK_ARG(a->workspace && aligned16(a->workspace) && a->workspace_bytes >= need,
                   "lasr_conv2_gemm/dx_w1: workspace needs %lld bytes", (long long)need);
    p.cv.x = a->x; p.cv.T0 = a->T; p.cv.F0 = a->F;
    p.cv.w1part = (float*)a->workspace;
    conv2_dx_kernel<256, EPI_AUX_RELU_W1><<<nb, 256, 0, st>>>(p, dc);
    if (int rc = lasr_check_launch("lasr_conv2_gemm/dx_w1")) return rc;
    const int N10 = 10 * C, ng = (int)cdiv(rows, W1_GROUP);
    float* grp = p.cv.w1part + (int64_t)rows * N10;
    float* tot = grp + (int64_t)ng * N10;
    w1_group_sum_kernel<<<dim3((unsigned)cdiv(N10, 256), (unsigned)ng), 256, 0, st>>>(p.cv.w1part, rows, N10, grp);
    if (int rc = lasr_check_launch("lasr_conv2_gemm/dx_w1_groups")) return rc;
    if (int rc = lasr_reduce_cols(grp, ng, N10, tot, nullptr, N10, 0, st)) return rc;
    return lasr_scatter_kc(tot, 9, C, 9, a->dw1, a->db1, st);
  }
  if (BN == 256 && epi_code(p) == EPI_AUX_RELU) conv2_dx_kernel<256, EPI_AUX_RELU><<<nb, 256, 0, st>>>(p, dc);
  else if (BN == 256) conv2_dx_kernel<256><<<nb, 256, 0, st>>>(p, dc);
  else conv2_dx_kernel<128><<<nb, 256, 0, st>>>(p, dc);
  return lasr_check_launch("lasr_conv2_gemm/dx");
}
