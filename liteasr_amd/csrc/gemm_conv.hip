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

extern "C" int lasr_conv2_gemm(const lasr_conv2_args* a, void* stream) {
  LASR_CHECK_ARG(a != nullptr, "lasr_conv2_gemm: null args");
  LASR_CHECK_ARG(a->mode == LASR_CONV2_FWD || a->mode == LASR_CONV2_DW || a->mode == LASR_CONV2_DX,
                 "lasr_conv2_gemm: bad mode");
  LASR_CHECK_ARG(a->B > 0 && a->T1 >= 3 && a->F1 >= 3 && a->C > 0 && a->C % 128 == 0,
                 "lasr_conv2_gemm: needs B > 0, T1, F1 >= 3 and C % 128 == 0");
  LASR_CHECK_ARG((int64_t)a->B * a->T1 * a->F1 * a->C < (1LL << 31) && 9LL * a->C * a->C < (1LL << 31),
                 "lasr_conv2_gemm: tensors past 2^31 elements");
  LASR_CHECK_ARG(a->y1 && a->out && aligned16(a->y1) && aligned16(a->out), "lasr_conv2_gemm: y1/out");
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
  p.c_vec = 1;
  if (a->mode == LASR_CONV2_FWD) {
    LASR_CHECK_ARG(a->bias && aligned16(a->bias), "lasr_conv2_gemm: bias");
    p.M = g.M2; p.N = C; p.K = 9 * C; p.kchunk = p.K;
    p.A = a->y1; p.lda_m = 9 * C; p.lda_k = 1;
    p.B = a->w2p; p.ldb_n = 9 * C; p.ldb_k = 1;
    p.C = a->out; p.ldc = C;
    p.bias = a->bias; p.bias_vec = 1; p.act = LASR_ACT_RELU;
    p.epi_mode = 0;
    dim3 grid((unsigned)(C / BN), (unsigned)cdiv(p.M, 128), 1);
    LASR_CHECK_ARG(grid.y <= 65535, "lasr_conv2_gemm: grid too large");
    if (BN == 256) gemm_bf16_glds_kernel<128, 256, true, true, bf16_t, 3, 2, G_FWD><<<grid, 256, 0, st>>>(p);
    else gemm_bf16_glds_kernel<128, 128, true, true, bf16_t, 3, 3, G_FWD><<<grid, 256, 0, st>>>(p);
    return lasr_check_launch("lasr_conv2_gemm/fwd");
  }
  if (a->mode == LASR_CONV2_DW) {
    p.M = C; p.N = 9 * C; p.K = (int)kpad;
    p.A = a->dy2; p.lda_m = 1; p.lda_k = C;
    p.B = a->y1; p.ldb_n = 1; p.ldb_k = 9 * C;
    p.C = a->out; p.ldc = 9 * C;
    p.epi_mode = 0; p.ws_vec = 1; p.v4 = 1;
    const bool big = g_tile_m == 256 && C % 256 == 0;
    const int TM = big ? 256 : 128, TN = big ? 256 : 128;
    const int64_t tiles = (int64_t)(C / TM) * (9 * C / TN);
    int split = 1;
    const int kt = (int)(kpad / 32);
    if (g_split > 0) split = g_split;
    else while (tiles * split < 512 && kt / (split * 2) >= 16 && split * 2 <= 64) split *= 2;
    const int64_t need = ((int64_t)split * C * 9 * C + (a->rowsum ? (int64_t)split * C : 0)) * 4;
    if (split > 1 && (!a->workspace || a->workspace_bytes < need || !aligned16(a->workspace))) split = 1;
    p.split_k = split;
    p.kchunk = split > 1 ? (int)(cdiv(cdiv(kpad, split), 32) * 32) : (int)kpad;
    p.ws = (float*)a->workspace;
    p.rowsum = a->rowsum;
    if (a->rowsum && split > 1) p.rs_ws = p.ws + (int64_t)split * C * 9 * C;
    dim3 grid((unsigned)(9 * C / TN), (unsigned)(C / TM), (unsigned)split);
    if (big) gemm_bf16_glds_kernel<256, 256, false, false, float, 3, 1, G_DW><<<grid, 256, 0, st>>>(p);
    else if (g_stages >= 4) gemm_bf16_glds_kernel<128, 128, false, false, float, 4, 2, G_DW><<<grid, 256, 0, st>>>(p);
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
  // LASR_CONV2_DX: one launch per output parity class, heaviest (4 taps) first
  p.N = C;
  p.A = a->dy2; p.lda_m = C; p.lda_k = 1;
  p.B = a->w2p; p.ldb_n = 1; p.ldb_k = 9 * C;
  p.C = a->out; p.ldc = C;
  p.aux = a->y1; p.aux_dtype = LASR_BF16; p.ldaux = C; p.aux_act = LASR_ACT_RELU; p.aux_vec = 1;
  p.epi_mode = 1;
  p.cv.zero = (const bf16_t*)a->dy2 + (int64_t)g.M2 * C;
  for (int cls = 0; cls < 4; ++cls) {
    const int pt = cls >> 1, pf = cls & 1;
    const int nI = (g.T1 - pt + 1) >> 1, nJ = (g.F1 - pf + 1) >> 1;
    p.cv.cls = cls;
    p.M = g.B * nI * nJ;
    p.K = (pt ? 1 : 2) * (pf ? 1 : 2) * C;
    p.kchunk = p.K;
    dim3 grid((unsigned)(C / BN), (unsigned)cdiv(p.M, 128), 1);
    LASR_CHECK_ARG(grid.y <= 65535, "lasr_conv2_gemm: grid too large");
    if (BN == 256) gemm_bf16_glds_kernel<128, 256, true, false, bf16_t, 3, 2, G_DX><<<grid, 256, 0, st>>>(p);
    else gemm_bf16_glds_kernel<128, 128, true, false, bf16_t, 3, 3, G_DX><<<grid, 256, 0, st>>>(p);
    const int rc = lasr_check_launch("lasr_conv2_gemm/dx");
    if (rc) return rc;
  }
  return LASR_OK;
}
