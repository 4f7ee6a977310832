// Batched GEMM with fused epilogues (lasr_gemm, include/liteasr_hip.h).
//
// bf16 path: 256-thread workgroups (4 waves, 2x2), BMxBNx32 tiles, register-staged
// double-buffered LDS, v_mfma_f32_16x16x32_bf16, fp32 accumulation.  LDS tiles are
// stored K-contiguous ([rows][32] bf16, 64-B rows) with a 16-B-chunk XOR swizzle
// chunk' = chunk ^ H[(row>>2)&3], H = {0,2,3,1}: for the ds_read_b128 lane groups of
// gfx950 every 16-lane group then covers all 16 slots of a 256-B bank row (no
// conflicts).  Operands that are not K-contiguous in HBM (the dW "TN" GEMMs, the dX "NN"
// GEMMs, the attention P.V / dS^T products) keep their HBM orientation in LDS ([k][rows])
// and are read with the gfx950 transposed read ds_read_b64_tr_b16 (TileLoader below).
// fp32 path (parity build): 64x64x16 tiles on v_mfma_f32_16x16x4f32 (exact fp32 FMA
// chain), element-wise staging; correctness first.
//
// Replaces aten addmm/mm/bmm at liteasr/nets/feed_forward.py:18-19,
// attention.py:35-37,58,69,145,149, subsampling.py:34,47, conformer_convolution.py:48,55,
// ctc.py:29, transformer_decoder.py:91 (and their autograd backward GEMMs).
#include "gemm_kernel.h"
#include <algorithm>

// ================================ host launcher ==================================
// The launcher keeps no process-wide state: tile / stage-depth overrides are per-call fields of
// lasr_gemm_args (tile_m, tile_n, ksub; 0 = the planner's choice).

// bf16 launch table: gemm_launch.h, instantiated per operand layout in gemm_l{0..3}.hip
template <bool AKC, bool BKC, typename TC>
void launch_bf16(const GemmP& p, int BM, int BN, int ks, int nw, bool glds, dim3 grid, hipStream_t st);
#define LASR_EXTERN_LAUNCH(ak, bk)                                                                         \
  extern template void launch_bf16<ak, bk, float>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t); \
  extern template void launch_bf16<ak, bk, bf16_t>(const GemmP&, int, int, int, int, bool, dim3, hipStream_t);
LASR_EXTERN_LAUNCH(true, true)
LASR_EXTERN_LAUNCH(true, false)
LASR_EXTERN_LAUNCH(false, true)
LASR_EXTERN_LAUNCH(false, false)
#undef LASR_EXTERN_LAUNCH

template <typename TC>
static void dispatch(const GemmP& p, bool akc, bool bkc, int bf16in, int BM, int BN, int ks, int nw, bool glds,
                     dim3 grid, hipStream_t st) {
  if (bf16in) {
    if (akc && bkc) launch_bf16<true, true, TC>(p, BM, BN, ks, nw, glds, grid, st);
    else if (akc) launch_bf16<true, false, TC>(p, BM, BN, ks, nw, glds, grid, st);
    else if (bkc) launch_bf16<false, true, TC>(p, BM, BN, ks, nw, glds, grid, st);
    else launch_bf16<false, false, TC>(p, BM, BN, ks, nw, glds, grid, st);
  } else {
    if (akc && bkc) gemm_f32_kernel<true, true, TC><<<grid, 256, 0, st>>>(p);
    else if (akc) gemm_f32_kernel<true, false, TC><<<grid, 256, 0, st>>>(p);
    else if (bkc) gemm_f32_kernel<false, true, TC><<<grid, 256, 0, st>>>(p);
    else gemm_f32_kernel<false, false, TC><<<grid, 256, 0, st>>>(p);
  }
}

static int narrow_n_tiles = 1;  // (lasr_gemm_narrow_tiles: A/B runs)
extern "C" int lasr_gemm_narrow_tiles(int on) {
  narrow_n_tiles = on != 0;
  return LASR_OK;
}

// Tile and split-K choice for one call (shared by lasr_gemm and lasr_gemm_plan).  nwo: 8 for
// an 8-wave instance (none planned today; see below), else 4.
static void gemm_plan(const lasr_gemm_args* a, int* BMo, int* BNo, int* splito, int* kso = nullptr,
                      int* nwo = nullptr) {
  int nw = 4;
  const int batch = a->batch > 0 ? a->batch : 1;
  const bool bf = a->in_dtype == LASR_BF16;
  int BM = 64, BN = 64;
  int split = a->split_k > 0 ? a->split_k : 1;
  const bool plain = !a->act && !a->zout && !a->aux && !a->res && a->drop_p <= 0.f;
  // split_k <= 0 asks for an automatic split; with an epilogue (the small-grid long-K GEMMs,
  // kernels.gemm) the fixed-order split-K reduction applies it (splitk_reduce_kernel:
  // bias, activation, aux, dropout, residual, beta -- the same per-element arithmetic)
  const bool autosplit = a->split_k <= 0 && !a->zout && a->workspace;
  const int kt = (int)cdiv(a->K, 32);
  if (bf && autosplit && kt >= 16) {
    // long-K (weight-gradient) GEMMs: big tiles, fill the chip with K slices instead
    // dW shapes of the step (K = B*T' ~ 8k): 64-wide tiles and >= 512 workgroups
    // (tools/dw_sweep.py: 15-25 % faster than 128 x 128 at 256 blocks); 64 x 64 up to
    // 768 x 256 outputs, else 64 along the longer side.  Very long K (the subsampling
    // conv2 weight gradient, K ~ 151k) keeps 128 x 128 and 256 workgroups.
    const bool very_long = kt >= 2048;
    BM = BN = 64;
    if (very_long) {
      BM = a->M >= 96 ? 128 : 64;
      BN = a->N >= 96 ? 128 : 64;
    } else if ((int64_t)a->M * a->N > 768 * 256) {
      BM = a->M >= a->N ? 64 : 128;
      BN = a->M >= a->N ? 128 : 64;
    }
    const int64_t nb = cdiv(a->M, BM) * cdiv(a->N, BN) * (int64_t)batch;
    // K-contiguous A: the small-grid long-K data GEMMs kernels.gemm splits (the decoder's
    // K = 2048 / V projections at B*(L+1) rows): ~128+ workgroups -- fewer fp32 slabs to
    // reduce beats filling the chip (tools/tile_ab.py at M 1312: split 4 12.5 / 13.3 us vs
    // split 8 15.8 / 15.4 us); the weight gradients (M-contiguous A) fill one round or two
    const int64_t target = a->lda_k == 1 ? 128 : (very_long || !plain ? 256 : 512);
    while (nb * split < target && split * 2 <= 64 && kt / (split * 2) >= 8) split *= 2;
  } else if (bf) {
    const int cfg[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};
    // narrow outputs (N <= 64; the per-head d_k-wide attention GEMMs, e.g. dqv = dBD p over
    // B*H batches, K = T'): 64 x 64 -- a 128-wide tile leaves half or more of its columns
    // idle, and the short k loops want the most row tiles (dqv at config 4, d_k 32: 34.0 ->
    // 19.2 us; config 2: 8.8 -> 6.1; long: 20.6 -> 15.9; profiles/r06/attn_gemm_tiles.jsonl)
    const int c0 = a->N <= 64 && narrow_n_tiles ? 3 : 0;
    for (int c = c0; c < 4; ++c) {
      const int64_t nb = cdiv(a->M, cfg[c][0]) * cdiv(a->N, cfg[c][1]) * (int64_t)batch;
      BM = cfg[c][0]; BN = cfg[c][1];
      // >= 480: the N = 512 GEMMs of config 4 (M 7968) take 128 x 64 at 504 tiles instead of
      // 64 x 64 at 1000 (2 rounds): fc2 forward 42.4 -> 32.8 us, fc1 dX 38.4 -> 29.3 us in the
      // graph-replayed sweep, whole large step 19.91 -> 19.38 ms with small unchanged
      // (profiles/r06/tile_ab_large_n512.jsonl, step_ab_tile_threshold.jsonl)
      if (nb >= 480) break;
    }
    // very large outputs with long K (subsampling conv2: M 151k, N 256, K 2304): the
    // 128x256 tile halves the A re-reads (tile sweep: 237 vs 266 us)
    if (BM == 128 && BN == 128 && a->N >= 256 && a->K >= 1024 && cdiv(a->M, 128) * batch >= 1024) BN = 256;
    // heavy epilogues over wide outputs (FFN fc1 forward: pre-activation copy + Swish +
    // dropout; FFN dX fc2: activation-gradient aux + dropout; N 2048): 128x256 halves the
    // per-output epilogue bookkeeping (cold-cache sweep: 32 vs 38 us, 40.2 vs 44.6 us)
    // (also the gate-free fc1 forward: bias + Swish + dropout without zout)
    if (BM == 128 && BN == 128 && (a->zout || a->aux || (a->act && a->drop_p > 0.f)) && a->N >= 1024) BN = 256;
    // (FFN fc2 forward, M 7968 N 256 K 2048: 64 x 128 wins the cold-operand sweep, 24.2 vs
    // 27.6 us, but loses inside the step, 33.5 vs 24 us per launch: kept at 64 x 64)
    // (the 8-wave 256 x 256 tile, one workgroup per CU, for the FFN fc1 forward / fc2 input
    // gradient at K = 256: 40.8 / 38.5 vs 37.8 / 38.4 us in the step, 11.70 vs 11.59 ms/step --
    // their time is the epilogue, which a second co-resident 4-wave workgroup overlaps)
  }
  if (!bf && autosplit) {
    const int64_t nb = cdiv(a->M, BM) * cdiv(a->N, BN) * (int64_t)batch;
    while (nb * split < 512 && split * 2 <= 32 && kt / (split * 2) >= 4) split *= 2;
  }
  if (bf && a->tile_m) {  // per-call override (A/B tools, bit-identity tests)
    BM = a->tile_m;
    BN = a->tile_n;
    nw = 4;
  }
  if (a->split_k <= -2 && plain && a->workspace) split = -a->split_k;  // explicit partials-only
  const int64_t rs_floats = a->rowsum ? (int64_t)split * a->M : 0;
  // an explicit split (split_k >= 2) may carry any epilogue but the pre-activation copy: the
  // split-K reduction applies it (tools/splitk_sweep.py)
  if (split > 1 && ((!plain && !autosplit && (a->split_k < 2 || a->zout)) || !a->workspace ||
                    a->workspace_bytes < ((int64_t)split * batch * a->M * a->N + rs_floats) * 4))
    split = 1;
  // ring depth of the LDS-DMA kernel: 64-deep stages (two 32-deep sub-tiles per counted
  // wait + barrier) for 64 x 64 tiles and long k loops; 32-deep for the wide 128 x 256 tiles
  // (their 64-deep ring fits only 2 stages) and short-K big tiles (tools/ksub_sweep.py)
  if (kso) {
    const int64_t kc = split > 1 ? cdiv(a->K, split) : a->K;
    const bool small = BM * BN <= 64 * 128;
    *kso = (bf && BM < 256 && BN < 256 && ((BM == 64 && BN == 64) || kc >= 1024 || (kc >= 512 && small))) ? 2 : 1;
    if (nw == 8) *kso = 2;
    else if (a->ksub) *kso = a->ksub;
  }
  if (nwo) *nwo = nw;
  *BMo = BM;
  *BNo = BN;
  *splito = split;
}

// LDS-DMA eligibility: bf16, 16-B aligned rows/columns; for a non-K-contiguous operand the
// row stride covers the extent rounded up to 8 (a 16-B chunk never leaves its row; the
// padding columns only feed discarded outputs).
static bool gemm_uses_glds(const lasr_gemm_args* a) {
  if (a->in_dtype != LASR_BF16) return false;
  const bool akc = (a->lda_k == 1), bkc = (a->ldb_k == 1);
  const int64_t s_a = akc ? a->lda_m : a->lda_k;
  const int64_t s_b = bkc ? a->ldb_n : a->ldb_k;
  const bool a_vec = aligned16(a->A) && s_a % 8 == 0 && a->sa1 % 8 == 0 && a->sa2 % 8 == 0;
  const bool b_vec = aligned16(a->B) && s_b % 8 == 0 && a->sb1 % 8 == 0 && a->sb2 % 8 == 0;
  const int64_t M8 = cdiv(a->M, 8) * 8, N8 = cdiv(a->N, 8) * 8;
  return a_vec && b_vec && (akc || a->lda_k >= M8) && (bkc || a->ldb_k >= N8);
}

static bool tile_ok(int tm, int tn) {
  return (tm == 0 && tn == 0) || ((tm == 64 || tm == 128 || tm == 256) && (tn == 64 || tn == 128 || tn == 256) &&
                                  (tm < 256 || tn >= 128) && (tn < 256 || tm >= 128));
}

extern "C" int lasr_gemm_plan(const lasr_gemm_args* a, int* tile_m, int* tile_n, int* split_k, int* flags) {
  LASR_CHECK_ARG(a && tile_m && tile_n && split_k, "lasr_gemm_plan: null argument");
  int ks = 1, nw = 4;
  gemm_plan(a, tile_m, tile_n, split_k, &ks, &nw);
  const bool glds = gemm_uses_glds(a);
  if (!glds) {  // as lasr_gemm: 256-wide tiles exist only in the LDS-DMA kernel
    *tile_m = std::min(*tile_m, 128);
    *tile_n = std::min(*tile_n, 128);
    nw = 4;
  }
  if (flags) {
    *flags = (glds ? LASR_PLAN_GLDS : 0) | (a->rowsum && glds && a->lda_k != 1 ? LASR_PLAN_ROWSUM_FUSED : 0) |
             (glds && ks == 2 && (*tile_m < 256 || nw == 8) ? LASR_PLAN_KSUB2 : 0) |
             (glds && nw == 8 ? LASR_PLAN_WIDE : 0);
  }
  return LASR_OK;
}

extern "C" int lasr_gemm(const lasr_gemm_args* a, void* stream) { return gemm_run(a, stream, nullptr); }

int gemm_run(const lasr_gemm_args* a, void* stream, GemmRowPost* post) {
  LASR_CHECK_ARG(a != nullptr, "lasr_gemm: null args");
  LASR_CHECK_ARG(a->M >= 0 && a->N >= 0 && a->K >= 0, "lasr_gemm: negative size");
  LASR_CHECK_ARG(a->in_dtype == LASR_F32 || a->in_dtype == LASR_BF16, "lasr_gemm: bad in_dtype");
  LASR_CHECK_ARG(a->c_dtype == LASR_F32 || a->c_dtype == LASR_BF16, "lasr_gemm: bad c_dtype");
  LASR_CHECK_ARG(a->lda_m == 1 || a->lda_k == 1, "lasr_gemm: A needs a unit stride");
  LASR_CHECK_ARG(a->ldb_n == 1 || a->ldb_k == 1, "lasr_gemm: B needs a unit stride");
  LASR_CHECK_ARG(a->A && a->B && a->C, "lasr_gemm: null operand");
  LASR_CHECK_ARG(a->zout_mode == 0 || a->zout_mode == 1, "lasr_gemm: zout_mode must be 0 or 1");
  LASR_CHECK_ARG(a->act != LASR_ACT_GATE && (!a->aux || a->aux_act != LASR_ACT_NONE),
                 "lasr_gemm: act GATE is only an aux_act; aux needs an aux_act");
  LASR_CHECK_ARG(tile_ok(a->tile_m, a->tile_n) && a->ksub >= 0 && a->ksub <= 2,
                 "lasr_gemm: tile override must be 64/128/256 x 64/128/256 (256 only beside >= 128) or 0 x 0, "
                 "ksub 0, 1 or 2");
  if (a->M == 0 || a->N == 0 || a->batch == 0) return LASR_OK;
  const int batch = a->batch > 0 ? a->batch : 1;
  const int bdiv = a->batch_div > 0 ? a->batch_div : 1;
  LASR_CHECK_ARG(batch == 1 || (!a->aux && !a->res && !a->zout && !a->rowsum),
                 "lasr_gemm: aux/res/zout/rowsum only supported for batch == 1");
  LASR_CHECK_ARG(!a->rowsum || a->lda_m == 1, "lasr_gemm: rowsum needs an M-contiguous A");

  GemmP p;
  p.M = a->M; p.N = a->N; p.K = a->K; p.batch = batch; p.batch_div = bdiv;
  p.A = a->A; p.lda_m = a->lda_m; p.lda_k = a->lda_k; p.sa1 = a->sa1; p.sa2 = a->sa2;
  p.B = a->B; p.ldb_n = a->ldb_n; p.ldb_k = a->ldb_k; p.sb1 = a->sb1; p.sb2 = a->sb2;
  p.C = a->C; p.ldc = a->ldc; p.sc1 = a->sc1; p.sc2 = a->sc2;
  p.alpha = a->alpha; p.alpha_dev = a->alpha_dev; p.beta = a->beta;
  p.bias = a->bias; p.act = a->act; p.zout = a->zout; p.zout_mode = a->zout_mode;
  p.aux = a->aux; p.aux_dtype = a->aux_dtype; p.ldaux = a->ldaux; p.aux_act = a->aux_act;
  p.drop = mkdrop(a->drop_p, a->drop_seed);
  p.res = a->res; p.res_dtype = a->res_dtype; p.ldres = a->ldres; p.res_scale = a->res_scale;

  const bool akc = (a->lda_k == 1);
  const bool bkc = (a->ldb_k == 1);
  const bool bf = a->in_dtype == LASR_BF16;
  {
    const int64_t s_a = akc ? a->lda_m : a->lda_k;
    const int64_t s_b = bkc ? a->ldb_n : a->ldb_k;
    p.a_vec = bf && aligned16(a->A) && s_a % 8 == 0 && a->sa1 % 8 == 0 && a->sa2 % 8 == 0;
    p.b_vec = bf && aligned16(a->B) && s_b % 8 == 0 && a->sb1 % 8 == 0 && a->sb2 % 8 == 0;
  }
  p.c_vec = aligned16(a->C) && a->ldc % 8 == 0 && a->sc1 % 8 == 0 && a->sc2 % 8 == 0 &&
            (!a->zout || aligned16(a->zout));
  p.aux_vec = a->aux && aligned16(a->aux) && a->ldaux % 8 == 0;
  p.res_vec = a->res && aligned16(a->res) && a->ldres % 8 == 0;
  p.ws_vec = a->N % 8 == 0;
  p.bias_vec = a->bias && aligned16(a->bias);
  {
    // 4-wide accesses of the direct epilogue: every row start 4-element aligned and the
    // bases aligned to 4 elements' bytes (8 B bf16, 16 B fp32)
    auto al4 = [](const void* q, int dtp) {
      return ((uintptr_t)q & (dtp == LASR_F32 ? 15 : 7)) == 0;
    };
    const int cdt = a->c_dtype;
    p.v4 = a->N % 4 == 0 && a->ldc % 4 == 0 && a->sc1 % 4 == 0 && a->sc2 % 4 == 0 && al4(a->C, cdt) &&
           (!a->zout || al4(a->zout, cdt)) && (!a->bias || aligned16(a->bias)) &&
           (!a->aux || (a->ldaux % 4 == 0 && al4(a->aux, a->aux_dtype))) &&
           (!a->res || (a->ldres % 4 == 0 && al4(a->res, a->res_dtype))) &&
           (!a->workspace || aligned16(a->workspace));
  }
  {
    const int nsrc = (a->aux ? 1 : 0) + (a->res ? 1 : 0);
    const bool base_ok = p.c_vec && a->beta == 0.f;
    const bool src_ok = nsrc == 1 && a->N % 8 == 0 && (a->aux ? p.aux_vec : p.res_vec);
    p.epi_mode = !base_ok ? 2 : nsrc == 0 ? 0 : src_ok ? 1 : 2;
  }

  int BM, BN, split, ks, nw;
  gemm_plan(a, &BM, &BN, &split, &ks, &nw);
  p.split_k = split;
  const int kstep = bf ? 32 : 16;
  p.kchunk = split > 1 ? (int)(cdiv(cdiv(a->K, split), kstep) * kstep) : a->K;
  p.ws = (float*)a->workspace;
  p.rowsum = nullptr;
  p.rs_ws = nullptr;

  hipStream_t st = (hipStream_t)stream;
  // LDS-DMA path: 16-B aligned rows/columns; for a non-K-contiguous operand the row stride
  // covers the extent rounded up to 8 (a 16-B chunk never leaves its row; the padding
  // columns only feed discarded outputs).
  const bool glds = gemm_uses_glds(a);
  if (!glds) {  // 256-wide tiles exist only in the LDS-DMA kernel
    BM = std::min(BM, 128);
    BN = std::min(BN, 128);
    nw = 4;
  }
  dim3 grid((unsigned)cdiv(a->N, BN), (unsigned)cdiv(a->M, BM), (unsigned)(batch * split));
  LASR_CHECK_ARG(grid.y <= 65535 && grid.z <= 65535, "lasr_gemm: grid too large");
  // fused bias gradient: in the LDS-DMA kernel when A is M-contiguous, else a column sum
  const bool rs_fused = a->rowsum && glds && !akc;
  if (rs_fused) {
    p.rowsum = a->rowsum;
    if (split > 1) p.rs_ws = p.ws + (int64_t)split * batch * a->M * a->N;
  }
  if (a->c_dtype == LASR_F32) dispatch<float>(p, akc, bkc, bf, BM, BN, ks, nw, glds, grid, st);
  else dispatch<bf16_t>(p, akc, bkc, bf, BM, BN, ks, nw, glds, grid, st);
  int rc = lasr_check_launch("lasr_gemm");
  if (!rc && split > 1 && a->split_k >= 0 && post) {  // a row post-op may take over the reduction
    const int r = post->launch(p, post->ctx, st);
    if (r < 0) return r;
    post->done = r;
    if (r) {
      rc = lasr_check_launch("lasr_gemm/splitk_reduce_post");
      if (rc || !a->rowsum || rs_fused) return rc;
    }
  }
  if (!rc && split > 1 && a->split_k >= 0 && !(post && post->done)) {
    const int64_t total = (int64_t)a->M * a->N * batch;
    const int nblk = (int)std::min<int64_t>(cdiv(p.v4 ? total / 4 : total, 256), 4096);
    if (a->c_dtype == LASR_F32) splitk_reduce_kernel<float><<<nblk, 256, 0, st>>>(p);
    else splitk_reduce_kernel<bf16_t><<<nblk, 256, 0, st>>>(p);
    rc = lasr_check_launch("lasr_gemm/splitk_reduce");
  }
  if (rc || !a->rowsum || rs_fused) return rc;
  // unfused: rowsum of A[M, K] (lda_m == 1) = column sums of the [K, M] matrix, ld lda_k.
  // Its scratch starts after the split-K partials (which a partials-only call leaves in the
  // workspace for the caller's reduction: they must not be overwritten).
  const int64_t used = split > 1 ? (int64_t)split * batch * a->M * a->N : 0;
  LASR_CHECK_ARG(a->workspace && a->workspace_bytes / 4 > used, "lasr_gemm: no workspace left for the rowsum");
  return lasr_colsum(a->A, a->in_dtype, a->K, a->M, a->lda_k, a->rowsum, 1, (float*)a->workspace + used,
                     a->workspace_bytes / 4 - used, stream);
}


// ---------------------------------------------------------------------------------------
// Grouped split-K weight gradients (partials only): the deferred dW GEMMs of one backward
// node in one launch.  Every problem must be what lasr_gemm would run as a partials-only
// (split_k = -1) LDS-DMA launch with 64-deep stages, A M-contiguous and B N-contiguous
// (dW = dY^T X), and all must share the planned tile; the partials (+ fused rowsum partials)
// land exactly where lasr_gemm would put them, bit for bit.
int launch_dw_group(const DwGroupP& g, int BM, int BN, int blocks, hipStream_t st);
static int dw_group_lpt = 1;  // (lasr_gemm_dw_group_order: tests and A/B runs)
extern "C" int lasr_gemm_dw_group_order(int longest_first) {
  dw_group_lpt = longest_first != 0;
  return LASR_OK;
}

extern "C" int lasr_gemm_dw_group(const lasr_gemm_args* args, int n, void* stream) {
  LASR_CHECK_ARG(args && n >= 1 && n <= LASR_DW_GROUP_MAX, "lasr_gemm_dw_group: 1..%d problems", LASR_DW_GROUP_MAX);
  DwGroupP g = {};
  g.n = n;
  // Problems are laid out longest K slice first.  The hardware deals blocks out in index
  // order and a CU takes the next block when its current one ends, so a group queued in
  // backward order (a layer's first FFN last) started its longest blocks in the last round
  // and they set the launch's tail; longest-first ends the launch about when the chip's
  // total work does.  Block order does not change any block's k range or destination: the
  // partials are bit-identical.
  int ord[LASR_DW_GROUP_MAX];
  int64_t work[LASR_DW_GROUP_MAX];
  for (int i = 0; i < n; ++i) {
    const lasr_gemm_args* a = args + i;
    int bm, bn, sp, ks;
    gemm_plan(a, &bm, &bn, &sp, &ks);
    // the K slice each block runs (the exact split is settled below; the group's tile is
    // shared, so the slice length orders the blocks by their work)
    work[i] = a->split_k == 1 || sp <= 1 ? a->K : cdiv(a->K, sp);
    ord[i] = i;
  }
  if (dw_group_lpt)
    std::stable_sort(ord, ord + n, [&](int x, int y) { return work[x] > work[y]; });
  int BM0 = 0, BN0 = 0, blocks = 0;
  for (int i = 0; i < n; ++i) {
    const lasr_gemm_args* a = args + ord[i];
    LASR_CHECK_ARG(a->in_dtype == LASR_BF16 && a->c_dtype == LASR_F32, "lasr_gemm_dw_group: bf16 in, fp32 partials");
    LASR_CHECK_ARG(a->lda_m == 1 && a->lda_k != 1 && a->ldb_n == 1 && a->ldb_k != 1,
                   "lasr_gemm_dw_group: A M-contiguous and B N-contiguous (dW = dY^T X)");
    const bool direct = a->split_k == 1;  // full-K tiles writing C itself (beta 0 / 1), no slab
    LASR_CHECK_ARG((direct || (a->split_k < 0 && a->workspace)) && (a->batch <= 1) && a->M > 0 && a->N > 0 &&
                       a->K > 0,
                   "lasr_gemm_dw_group: partials-only problems with a workspace, or direct (split_k 1) ones");
    LASR_CHECK_ARG(!direct || (a->C && a->ldc >= a->N && (a->beta == 0.f || a->beta == 1.f) && a->alpha == 1.f &&
                               !a->alpha_dev),
                   "lasr_gemm_dw_group: a direct problem needs C, ldc >= N, beta 0 or 1, alpha 1");
    LASR_CHECK_ARG(i == 0 || direct == (g.direct[0] != 0), "lasr_gemm_dw_group: direct and split problems mixed");
    LASR_CHECK_ARG(!a->act && !a->zout && !a->aux && !a->res && a->drop_p <= 0.f && !a->bias,
                   "lasr_gemm_dw_group: no epilogue");
    LASR_CHECK_ARG(gemm_uses_glds(a), "lasr_gemm_dw_group: operands not LDS-DMA eligible");
    int BM, BN, split, ks;
    gemm_plan(a, &BM, &BN, &split, &ks);
    if (direct) split = 2;  // (plan-shape checks below; the launch uses one K slice)
    // the group kernel runs 64-deep ring stages; a lone 32-deep launch gives the same bits
    // (the sub-tiles keep their images and order: test_gemm_ksub2_bit_identical), so a
    // short-K plan (e.g. the decoder's FFN weights, K = B*(L+1)) groups too
    LASR_CHECK_ARG(split > 1, "lasr_gemm_dw_group: plan is not a split-K launch");
    // the FFN-sized problems (64 x 128 / 128 x 64 plans) run on 128 x 128 group tiles: a
    // third less LDS-DMA ingest per output, and a tile's shape does not change any output's
    // summation order (k order within the slice); the group's many problems and K slices
    // keep the chip full (grouped FFN dW of a layer: 77 -> 57 us per launch)
    if (((BM == 128 && BN == 64) || (BM == 64 && BN == 128)) && a->M >= 128 && a->N >= 128) {
      BM = BN = 128;
      // 256 x 128 tiles on 8 waves, one workgroup per CU, the same K slices (one tile for
      // the whole group): 0.25 fewer LDS-DMA bytes per MFMA than the 4-wave 128 x 128 tile;
      // 11.84 -> 11.63-11.70 ms/step on two boxes (profiles/r03/dw_group_ab.json; 256 x 256
      // with twice the slices, and a 2-stage ring, measured no better).
      if (a->M >= 256 && a->N >= 256 && !direct) {  // (direct groups keep 128 x 128: twice the tiles)
        BM = 256;
        BN = 128;
      }
    }
    LASR_CHECK_ARG(i == 0 || (BM == BM0 && BN == BN0), "lasr_gemm_dw_group: problems plan different tiles");
    BM0 = BM;
    BN0 = BN;
    if (direct) split = 1;
    g.M[i] = a->M; g.N[i] = a->N; g.K[i] = a->K;
    g.split[i] = split;
    g.kchunk[i] = direct ? a->K : (int)(cdiv(cdiv(a->K, split), 32) * 32);
    g.direct[i] = direct;
    g.C[i] = (float*)a->C; g.ldc[i] = a->ldc; g.beta[i] = a->beta; g.rowsum[i] = a->rowsum;
    g.v4[i] = a->N % 4 == 0 && aligned16(direct ? a->C : a->workspace);
    g.A[i] = a->A; g.lda[i] = a->lda_k;
    g.B[i] = a->B; g.ldb[i] = a->ldb_k;
    g.ws[i] = (float*)a->workspace;
    g.rs_ws[i] = a->rowsum && !direct ? (float*)a->workspace + (int64_t)split * a->M * a->N : nullptr;
    g.start[i] = blocks;
    const int64_t nb = cdiv(a->M, BM) * cdiv(a->N, BN) * (int64_t)split;
    LASR_CHECK_ARG(blocks + nb + 8 < (1ll << 31), "lasr_gemm_dw_group: too many blocks");
    blocks += (int)cdiv(nb, 8) * 8;
  }
  g.start[n] = blocks;
  static const int slice_xcd = [] { const char* e = getenv("LASR_DW_SLICE_XCD"); return e && e[0] ? atoi(e) : 1; }();
  g.slice_xcd = slice_xcd;
  LASR_CHECK_ARG(launch_dw_group(g, BM0, BN0, blocks, (hipStream_t)stream) == 0,
                 "lasr_gemm_dw_group: no grouped instance for tile %dx%d", BM0, BN0);
  return lasr_check_launch("lasr_gemm_dw_group");
}
