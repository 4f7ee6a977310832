/*
 * liteasr_hip.h — C ABI of libliteasr_hip.so, the MI355X (gfx950) kernels behind
 * the U2 / Conformer + hybrid CTC-attention training step.
 *
 * The reference (Nazukixv/LiteASR) is pure PyTorch: every op on its hot path is an
 * aten kernel reached from a liteasr.nets module.  Each entry point below replaces
 * one of those aten call sites; the citation names the reference file:line whose
 * behaviour it reproduces (paths relative to the reference repo root).
 *
 * Conventions
 *   - Plain pointers + sizes; no framework types.  Caller owns every buffer; the
 *     library keeps no device allocations (scratch is caller-provided workspace).
 *   - dtype codes: LASR_F32 / LASR_BF16 for activation storage; arithmetic is fp32.
 *   - Every call is stream-ordered on `stream` (a hipStream_t passed as void*),
 *     never synchronises, and is safe to capture into a hipGraph.
 *   - Return 0 on success, a negative LASR_ERR_* on failure; lasr_last_error()
 *     returns a thread-local message for the last failure.
 *   - Dropout: (p, seed) pairs.  The keep-mask is a pure function of
 *     (seed, logical element index) so backward regenerates it.
 *   - Reductions use fixed orders (no float atomics) => bitwise deterministic.
 */
#ifndef LITEASR_HIP_H
#define LITEASR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { LASR_F32 = 0, LASR_BF16 = 1, LASR_I32 = 2, LASR_I64 = 3, LASR_U8 = 4 };
enum { LASR_OK = 0, LASR_ERR_INVALID = -1, LASR_ERR_LAUNCH = -2 };
enum { LASR_ACT_NONE = 0, LASR_ACT_RELU = 1, LASR_ACT_SWISH = 2,
       LASR_ACT_GATE = 3 /* aux_act only: multiply by the aux value itself */,
       LASR_ACT_TANH = 4 /* act: tanh; aux_act: multiply by 1 - aux^2 (aux = a stored tanh
                            output: the Transducer joint, liteasr/models/transducer.py:202) */ };

const char* lasr_last_error(void);
int lasr_version(void);
/* Register a device uint64 step counter mixed into every dropout seed at kernel run
 * time (so graph replays draw fresh masks); NULL disables.  lasr_counter_add bumps it
 * on the stream (called once per training forward). */
int lasr_set_dropout_counter(const uint64_t* dev_counter);
int lasr_counter_add(uint64_t* dev_counter, uint64_t v, void* stream);

/* ------------------------------------------------------------------------
 * Batched GEMM with fused epilogue.
 *   C[z][m,n] = epilogue( alpha * sum_k A[z][m,k] * B[z][k,n] )
 * Replaces the aten addmm/mm/bmm behind nn.Linear and the attention matmuls:
 *   liteasr/nets/feed_forward.py:18-19, liteasr/nets/attention.py:35-37,58,69,145,149,
 *   liteasr/nets/subsampling.py:34,47, liteasr/nets/conformer_convolution.py:48,55,
 *   liteasr/nets/ctc.py:29, liteasr/nets/transformer_decoder.py:91.
 * Element strides are free (one of lda_m/lda_k must be 1, same for B).
 * z in [0,batch): z1 = z / batch_div, z2 = z % batch_div; operand offset
 *   = z1*s?1 + z2*s?2.
 * Epilogue order: v = alpha*acc (* *alpha_dev); v += bias[n]; zout = v; v = act(v);
 *   v *= act'(aux[m,n]); v *= dropmask(z*M*N + m*N + n); v = res[m,n] + res_scale*v;
 *   C = beta*C + v.
 * split_k (plain epilogues only: alpha/alpha_dev/beta/bias; otherwise 1 is used):
 *   1 = no split; > 1 = that many K slices; 0 = automatic (long-K dW GEMMs).  Slice
 *   partial sums go to `workspace` ([split][batch][M][N] fp32) and a second kernel reduces
 *   them in fixed order (deterministic).  -1 = automatic, partials only: the reduction
 *   is skipped (callers that fuse it elsewhere; profiling the GEMM kernel alone).
 *   The split (and tile) lasr_gemm would use is reported by lasr_gemm_plan.
 * ---------------------------------------------------------------------- */
typedef struct lasr_gemm_args {
  int M, N, K;
  int batch, batch_div;
  const void* A; int64_t lda_m, lda_k, sa1, sa2;
  const void* B; int64_t ldb_n, ldb_k, sb1, sb2;
  void* C; int64_t ldc, sc1, sc2;
  int in_dtype;  /* dtype of A and B */
  int c_dtype;
  float alpha; const float* alpha_dev;
  float beta;
  const float* bias;
  int act;
  void* zout;  /* optional (c_dtype, ld = ldc): zout_mode 0 the pre-activation copy, 1 the
               * gate act'(pre-activation) * keep (keep = the epilogue's dropout keep flag,
               * 0/1), which a later GEMM applies as aux with aux_act = LASR_ACT_GATE */
  const void* aux; int aux_dtype; int64_t ldaux; int aux_act;  /* v *= aux_act'(aux) */
  float drop_p; uint64_t drop_seed;
  const void* res; int res_dtype; int64_t ldres; float res_scale;
  int split_k;  /* 1: none, > 1: forced, 0: auto (fills the chip; needs workspace), -1: auto,
                 fp32 partials only (no reduction; the caller sums the [split] slabs),
                 <= -2: -split_k slices, fp32 partials only */
  void* workspace; int64_t workspace_bytes;
  /* optional fused bias gradient: rowsum[m] += sum_k A[m,k] (fp32, batch == 1, A
   * M-contiguous i.e. lda_m == 1: the dW = dY^T X GEMMs, rowsum = dbias).  Replaces the
   * separate column sum of dY (aten sum over rows in Linear's backward). */
  float* rowsum;
  int zout_mode;
  /* per-call plan overrides (0 = the planner's choice), for A/B measurements and the
   * bit-identity tests: the bf16 LDS-DMA tile (64/128/256 x 64/128/256) and the k depth of
   * its ring stages (1 = 32-deep, 2 = 64-deep: two 32-deep sub-tiles per counted wait).
   * A tile or stage depth never changes any output's summation order. */
  int tile_m, tile_n;
  int ksub;
} lasr_gemm_args;
int lasr_gemm(const lasr_gemm_args* args, void* stream);
/* A GEMM whose rows feed a LayerNorm (the decoder's K = ff GEMMs on B*(L+1) rows; the
 * reference's layer boundary liteasr/nets/transformer_layer.py:196-221 and the norm
 * liteasr/nets/layer_norm.py:8-28).  When the plan splits K, the split-K reduction launch also
 * runs the norm (one launch fewer, bit-identical to lasr_gemm + the norm entry); otherwise the
 * two launches run.  C must be batch 1 with contiguous rows (ldc == N), no rowsum.
 *  lasr_gemm_ln_fwd: C fp32 (the epilogue's output, e.g. res + dropout(A B)), then
 *    y = LN(C) (y_dtype) + mean / rstd per row -- lasr_layernorm_fwd(C, ...).
 *  lasr_gemm_ln_bwd: C = dln (any epilogue, stored), then lasr_layernorm_bwd(x, dln, ...) with
 *    dgamma = dbeta = NULL: dx, gb and the dgamma / dbeta partial rows in `part`
 *    ([cdiv(M, 16)][2N]; the caller reduces them). */
int lasr_gemm_ln_fwd(const lasr_gemm_args* args, const float* gamma, const float* beta, float eps, void* y,
                     int y_dtype, float* mean, float* rstd, void* stream);
int lasr_gemm_ln_bwd(const lasr_gemm_args* args, const void* x, int x_dtype, const float* gamma, const float* mean,
                     const float* rstd, const void* dres, int dres_dtype, void* dx, int dx_dtype, float* part,
                     int64_t part_floats, void* gb, int gb_dtype, float bscale, float bp, uint64_t bseed,
                     void* stream);
/* The encoder attention's positional-projection gradient GEMM (dp, split over K = B*T') and the
 * positional-bias gradient of lasr_qbias_bwd (liteasr/nets/attention.py:131-135) with its
 * partial rows left in ws (du = dv = NULL): when the GEMM's plan splits K, the split-K
 * reduction and the qbias blocks share one launch (bit-identical to lasr_gemm +
 * lasr_qbias_bwd); otherwise the two launches run.  C's dtype = dt. */
int lasr_gemm_qbias_bwd(const lasr_gemm_args* args, const void* dqu, const void* dqv, int dt, int B, int T, int H,
                        int dk, void* dqkv, int64_t ld, float* ws, int64_t ws_floats, void* stream);
/* Dropout: one 32-bit counter-hash draw per element pair, 16-bit halves against
 * thr = round(p * 65536); kept values scale by lasr_dropout_scale(p) = 65536 / (65536 - thr)
 * (E[mask * scale] = 1 exactly).  Host helper, no device work. */
float lasr_dropout_scale(float p);
/* Tile and split-K lasr_gemm would use; flags (nullable): LASR_PLAN_GLDS (LDS-DMA
 * kernel), LASR_PLAN_ROWSUM_FUSED (rowsum computed in the GEMM; with split_k = -1 and a
 * split > 1 its [split][M] partials follow the [split][batch][M][N] C partials in the
 * workspace, else it is written to rowsum directly). */
#define LASR_PLAN_GLDS 1
#define LASR_PLAN_ROWSUM_FUSED 2
#define LASR_PLAN_KSUB2 4 /* 64-deep LDS ring stages (two 32-deep sub-tiles per wait) */
#define LASR_PLAN_WIDE 8  /* 256 x 256 tile on 8 waves (512-thread workgroups) */
int lasr_gemm_plan(const lasr_gemm_args* args, int* tile_m, int* tile_n, int* split_k, int* flags);

/* Grouped split-K weight gradients (liteasr/trainer.py:142 loss.backward: the per-module
 * weight gradients of one Conformer layer / the decoder): n <= 8 independent partials-only
 * problems dW_i = A_i^T B_i (args[i] as for lasr_gemm with split_k = -1: A M-contiguous,
 * B N-contiguous, bf16, no epilogue, workspace for [split][M][N] partials + [split][M]
 * rowsum partials when rowsum is set) that plan the same tile with 64-deep stages, in one
 * launch; the partials are bit-identical to separate lasr_gemm calls.  The caller reduces
 * them (lasr_reduce_multi). */
int lasr_gemm_dw_group(const lasr_gemm_args* args, int n, void* stream);
/* Block order of later lasr_gemm_dw_group launches: 1 (default) = the problems with the
 * longest K slice first, 0 = call order; the partials are the same bits either way. */
int lasr_gemm_dw_group_order(int longest_first);
/* Planner switch for narrow outputs (N <= 64): 1 (default) = 64 x 64 tiles, 0 = the
 * fill-the-chip tile order of wider outputs; the results are the same bits. */
int lasr_gemm_narrow_tiles(int on);

/* Batched partial reductions (one launch for a backward node's deferred parameter
 * gradients): out[n] (+)= sum_p part[p*N + n], n < split -> out0[n], else out1[n-split].
 * Summation order per segment as the single-launch kernels (lasr_reduce_cols for P > 64,
 * the split-K reduce for P <= 64 with N % 4 == 0), so results are bit-identical. */
typedef struct lasr_reduce_seg {
  const float* part; int64_t N; int P; int accumulate;
  float* out0; float* out1; int64_t split;
} lasr_reduce_seg;
int lasr_reduce_multi(const lasr_reduce_seg* segs, int nseg, void* stream);

/* Column sums: out[n] (+)= sum_m X[m,n]  (bias gradients; fp32 out).
 * Two-pass deterministic; workspace >= ceil(M/rows_per_block)*N floats (see impl). */
int lasr_colsum(const void* X, int dtype, int64_t M, int64_t N, int64_t ldx,
                float* out, int accumulate, float* workspace, int64_t ws_floats, void* stream);

/* ------------------------------------------------------------------------
 * LayerNorm over the last dim, eps from caller (1e-12 in LiteASR:
 * liteasr/nets/layer_norm.py:10-21).  Row-major [rows, D].
 * fwd: y (y_dtype) = (x-mean)*rstd*gamma + beta; saves mean/rstd (fp32, [rows]).
 *      y2 (optional, y2_dtype): a second copy, with dropout (p2,seed2) applied
 *      (used for CTC's input dropout, liteasr/nets/ctc.py:29).
 * bwd: dx = LN'(dy) (+ dres if given); dgamma/dbeta accumulated into fp32 outs.
 *      Optional branch-grad output: gb = bscale * dropmask(bseed) * dx (gb_dtype),
 *      the gradient entering the preceding residual branch
 *      (liteasr/nets/conformer_layer.py:42,54,63; transformer_layer.py:48,58,173).
 * ---------------------------------------------------------------------- */
int lasr_layernorm_fwd(const void* x, int x_dtype, int64_t rows, int D, const float* gamma,
                       const float* beta, float eps, void* y, int y_dtype, float* mean,
                       float* rstd, void* y2, int y2_dtype, float p2, uint64_t seed2,
                       void* stream);
/* Two chained LayerNorms per row (a Conformer layer's final norm, then the next layer's
 * first norm: liteasr/nets/conformer_layer.py:147, :130): y = LN1(x) fp32 + (mean1, rstd1),
 * z = LN2(y) bf16 + (mean2, rstd2); bit-identical to two lasr_layernorm_fwd calls. */
int lasr_layernorm2_fwd(const float* x, int64_t rows, int D, const float* g1, const float* b1,
                        const float* g2, const float* b2, float eps, float* y, float* mean1,
                        float* rstd1, void* z, float* mean2, float* rstd2, void* stream);
int lasr_layernorm_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype, int64_t rows,
                       int D, const float* gamma, const float* mean, const float* rstd,
                       const void* dres, int dres_dtype, void* dx, int dx_dtype,
                       float* dgamma, float* dbeta, float* workspace, int64_t ws_floats,
                       void* gb, int gb_dtype, float bscale, float bp, uint64_t bseed,
                       void* stream);
/* The two LayerNorm backwards at a Conformer layer boundary in one launch (the reverse of
 * lasr_layernorm2_fwd; liteasr/nets/conformer_layer.py:130 and :147): the next layer's first
 * norm, dx1 = dres1 + LN1'(dy1) (x1 fp32, dy1 fp32 / bf16, dres1 fp32; dx1 is not stored),
 * then this layer's final norm on it, dx2 = LN2'(dx1) (x2 fp32, dx2 fp32) and the branch
 * gradient gb2 = bscale * drop(dx2) (bf16 / fp32, or NULL).  part1 / part2: each norm's
 * [ceil(rows/16)][2][D] gamma / beta partial rows, as lasr_layernorm_bwd's workspace holds
 * them, for the caller's reduction.  Bit-identical to two lasr_layernorm_bwd calls with dx1
 * stored in fp32 between them. */
int lasr_layernorm2_bwd(const float* x1, const void* dy1, int dy1_dtype, const float* dres1, int64_t rows, int D,
                        const float* g1, const float* mean1, const float* rstd1, float* part1, const float* x2,
                        const float* g2, const float* mean2, const float* rstd2, float* dx2, float* part2, void* gb2,
                        int gb2_dtype, float bscale, float bp, uint64_t bseed, void* stream);
/* ------------------------------------------------------------------------
 * Full-row GEMM with the LayerNorm in its epilogue: the residual projections of a
 * Conformer layer and the following sub-block's norm (liteasr/nets/conformer_layer.py:37-78
 * residual adds, layer_norm.py:20), and their backward (the input-gradient GEMM of a
 * sub-block's first projection + that norm's backward).  Tiles of 32 rows x all D columns
 * (D = 256 or 512), K % 64 == 0, bf16 A/W with 16-B aligned rows; every [M, D] buffer
 * below is contiguous.  Outputs are bit-identical to the two-launch path they replace
 * (lasr_gemm with its res epilogue + lasr_layernorm_fwd / lasr_layernorm2_fwd; lasr_gemm
 * to a bf16 dln + lasr_layernorm_bwd).
 *  lasr_linear_res_ln:    A [M, K], W [D, K] (nn.Linear weight):
 *    out = res + res_scale * dropout(A W^T + bias)   (fp32; dropout = lasr_gemm's, one
 *                                                    draw per column pair of row-major out)
 *    y1 = LN1(out) (y1_dtype) + mean1 / rstd1; if gamma2: y1 must be fp32 and
 *    y2 = LN2(y1) (bf16) + mean2 / rstd2 (the chained norms of lasr_layernorm2_fwd).
 *  lasr_linear_dx_ln_bwd: A = dY [M, K], W [K, D]:  dln = bf16(dY W), then
 *    dx = LN1'(dln; x, gamma1, mean1, rstd1) (+ dres), gb = bscale * dropmask(bp, bseed) * dx
 *    (bf16, optional), and part = the dgamma / dbeta partial rows [cdiv(M, 16)][2 D]
 *    exactly as lasr_layernorm_bwd's workspace holds them (dgamma = columns [0, D), dbeta =
 *    [D, 2D)); with dgamma and dbeta set they are also reduced into them (+=) as
 *    lasr_layernorm_bwd does, else the caller reduces them (lasr_reduce_multi).
 * ---------------------------------------------------------------------- */
typedef struct lasr_row_ln_args {
  int M, D, K;
  const void* A; int64_t lda;
  const void* W; int64_t ldw;
  const float* gamma1; const float* beta1; float eps;
  float* mean1; float* rstd1;
  /* forward */
  const float* bias; const float* res; float res_scale; float drop_p; uint64_t drop_seed;
  float* out; void* y1; int y1_dtype;
  const float* gamma2; const float* beta2; void* y2; float* mean2; float* rstd2;
  /* backward */
  const float* x; const float* dres; float* dx; void* gb; float bscale; float bp; uint64_t bseed;
  float* part; float* dgamma; float* dbeta;
} lasr_row_ln_args;
int lasr_linear_res_ln(const lasr_row_ln_args* args, void* stream);
int lasr_linear_dx_ln_bwd(const lasr_row_ln_args* args, void* stream);

/* gb = scale * dropmask(seed) * dx  (residual-branch gradient, standalone form). */
int lasr_branch_grad(const void* dx, int dx_dtype, int64_t n, void* gb, int gb_dtype,
                     float scale, float p, uint64_t seed, void* stream);

/* ------------------------------------------------------------------------
 * CTC (blank=0, reduction=sum) fused with log_softmax over the vocab.
 * Replaces liteasr/criterions/hybrid_ctc_attn.py:67-75 (h_ctc.transpose(0,1)
 * .log_softmax(-1) -> nn.CTCLoss) and aten's ctc_loss / _ctc_loss_backward.
 * logits: [B, T, V] (batch-major; row (b,t) starts at (b*T+t)*ld, ld >= V — a padded
 *         leading dimension keeps the vocab GEMMs 16-B vectorised), dtype `ldt`;
 *         grad uses the same row stride.
 * targets: [B, Lmax] int32, padded; tlen/ilen: [B] int32.
 * fwd: writes nll[B] (fp32; +inf when infeasible), and saves lse[B*T], lp[B*T*(Lmax+1)]
 *      (log-probs of blank and each target position) and alpha[B*T*(2*Lmax+1)].
 * bwd: grad[b,t,:] = g * (softmax - gamma_t) for t < ilen[b], 0 otherwise, where
 *      g = gscale * (*gdev if gdev).  Uses beta[B*T*(2*Lmax+1)] scratch.
 * ---------------------------------------------------------------------- */
/* beta (optional, [B][T][2*Lmax+1]): when given, the forward also runs the beta
 * recursion, concurrently with alpha; pass beta_ready = 1 to lasr_ctc_bwd then.
 * 2*Lmax+1 <= 1024 (one lattice state per thread).  alpha == NULL runs only the first
 * stage (row log-sum-exp over V and the gather of the blank / target log-probs into lp);
 * lasr_ctc_lattice then runs the second (the serial-in-T alpha (+ beta) recursion over lp
 * and nll), so the two stages can be timed or scheduled apart. */
int lasr_ctc_fwd(const void* logits, int ldt, int B, int T, int V, int64_t ld, const int32_t* targets,
                 int Lmax, const int32_t* ilen, const int32_t* tlen, float* lse, float* lp,
                 float* alpha, float* beta, float* nll, void* stream);
int lasr_ctc_lattice(int B, int T, int Lmax, const int32_t* targets, const int32_t* ilen, const int32_t* tlen,
                     const float* lp, float* alpha, float* beta, float* nll, void* stream);
int lasr_ctc_bwd(const void* logits, int ldt, int B, int T, int V, int64_t ld, const int32_t* targets,
                 int Lmax, const int32_t* ilen, const int32_t* tlen, const float* lse,
                 const float* lp, const float* alpha, const float* nll, float* beta,
                 int beta_ready, void* grad, int gdt, float gscale, const float* gdev, void* stream);

/* ------------------------------------------------------------------------
 * Label-smoothed KL (liteasr/criterions/hybrid_ctc_attn.py:49-64):
 *   row loss = sum_c td_c (log td_c - log_softmax(h)_c), td = s/(V-1), 1-s at target;
 *   rows with target == ignore contribute 0.
 * fwd: loss_rows[R] fp32, lse[R]. bwd: grad = g*(softmax - td) (0 on ignored rows).
 * logits/grad rows are `ld` elements apart (ld >= V).
 * ---------------------------------------------------------------------- */
int lasr_lsm_kl_fwd(const void* logits, int ldt, int R, int V, int64_t ld, const int32_t* target,
                    int ignore, float smoothing, float* lse, float* loss_rows, void* stream);
int lasr_lsm_kl_bwd(const void* logits, int ldt, int R, int V, int64_t ld, const int32_t* target,
                    int ignore, float smoothing, const float* lse, void* grad, int gdt,
                    float gscale, const float* gdev, void* stream);
/* out[0] = wa * sum(a[0:na]) + wb * sum(b[0:nb])   (hybrid loss combine,
 * liteasr/criterions/hybrid_ctc_attn.py:63-64,75,78). */
int lasr_loss_combine(const float* a, int na, float wa, const float* b, int nb, float wb,
                      float* out, void* stream);

/* ------------------------------------------------------------------------
 * Attention pieces (materialised-score form).
 * Relative-position MHA (liteasr/nets/attention.py:120-154, rel_shift :99-118):
 *   qu = q + pos_bias_u, qv = q + pos_bias_v       (lasr_qbias_fwd)
 *   S = scale*(qu k^T + rel_shift(qv p^T)), masked_fill(mask,-1e38), softmax, dropout
 *                                                  (lasr_attn_softmax_fwd, relpos=1)
 * Scores/probs are [Z=B*H, Tq, ldS] with ldS >= Tk (padding columns written 0).
 * mask: uint8 (1 = masked) addressed mask[b*mask_sb + i*mask_sq + j], may be NULL.
 * ---------------------------------------------------------------------- */
int lasr_qbias_fwd(const void* qkv, int dt, int B, int T, int H, int dk, int64_t ld_qkv,
                   const float* bias_u, const float* bias_v, void* qu, void* qv, void* stream);
int lasr_qbias_bwd(const void* dqu, const void* dqv, int dt, int B, int T, int H, int dk,
                   void* dqkv, int64_t ld_dqkv, float* dbias_u, float* dbias_v,
                   float* workspace, int64_t ws_floats, void* stream);
/* (dbias_u = dbias_v = NULL: the [ceil(B*T/64)][2*H*dk] partials stay in workspace.) */
int lasr_attn_softmax_fwd(const float* s_ac, const float* s_bd, int relpos, int B, int H,
                          int Tq, int Tk, int ldS, const uint8_t* mask, int64_t mask_sb,
                          int64_t mask_sq, void* P, int pdt, float drop_p, uint64_t seed,
                          void* Praw, void* stream);
/* P: probabilities after dropout (the P.V operand); Praw (optional, needed only when
 * drop_p > 0): probabilities before dropout, for the backward.
 * bwd: dS = Praw * (dPd*dropmask - rowsum(Praw*dPd*dropmask)), zeroed where masked
 * (masked_fill backward); dPd = dO V^T (fp32 [Z,Tq,ldS]). */
int lasr_attn_softmax_bwd(const void* P, int pdt, const float* dPd, int B, int H, int Tq, int Tk,
                          int ldS, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq,
                          float drop_p, uint64_t seed, void* dS, int dsdt, void* stream);
/* Inverse of rel_shift: dBD[z,r,c] = dS[z,i,j] for the unique (i,j) that reads
 * BD[r,c] in attention.py:99-118, else 0. */
int lasr_relshift_bwd(const void* dS, int dt, int Z, int T, int ldS, void* dBD, void* stream);
/* Fused relative-position self-attention, bf16, d_k = 64, Tq = Tk = T, no attention
 * dropout (liteasr/nets/attention.py:120-154 with rel_shift :99-118; replaces the
 * materialised-score chain qu.k^T, qv.p^T, lasr_attn_softmax_fwd, P.V).
 *   qu, qv   [B*T, ldq]  (q + pos_bias_u / v, lasr_qbias_fwd), head h at column h*64
 *   k, v     [B*T, ldkv] (slots of the fused qkv projection)
 *   pos      [T, ldp]    (linear_pos(pos_emb))
 *   stats    [B*H*T][2]  out: row max and 1/row sum of exp (the backward recomputes P)
 *   ctx      [B*T, ldc]  out: softmax(S) V, heads concatenated
 * mask as lasr_attn_softmax_fwd.  Row strides multiples of 8 elements, 16-B aligned. */
int lasr_relattn_fwd(const void* qu, const void* qv, int64_t ldq, const void* k, const void* v,
                     int64_t ldkv, const void* pos, int64_t ldp, int B, int H, int T, int dk,
                     const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                     float* stats, void* ctx, int64_t ldc, void* stream);
/* lasr_relattn_fwd with lasr_qbias_fwd folded in (one launch fewer per Conformer layer):
 *   q        [B*T, ldqin] the q slot of the fused qkv projection
 *   bu, bv   [H*d_k] fp32 pos_bias_u / pos_bias_v (attention.py:93-96), 16-B aligned
 *   qu, qv   [B*T, ldq]   out: q + u, q + v (bf16, lasr_qbias_fwd's rounding), for the backward
 * everything else as lasr_relattn_fwd. */
int lasr_relattn_fwd_qb(const void* q, int64_t ldqin, const float* bu, const float* bv, void* qu, void* qv,
                        int64_t ldq, const void* k, const void* v, int64_t ldkv, const void* pos, int64_t ldp,
                        int B, int H, int T, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq,
                        float scale, float* stats, void* ctx, int64_t ldc, void* stream);
/* Backward of lasr_relattn_fwd (recompute; deterministic).  Outputs:
 *   Dbuf [B*H*T]        scratch: rowsum(dctx * ctx)
 *   dqu  [B*T, ldq]     dL/d(q+u)
 *   dbd  [B][H][T][ldS] dL/d(bd) before rel_shift (unscaled), as lasr_relshift_bwd writes it
 *                       ([H][B][T][ldS] when dbd_head_major: then dpos = scale sum_b dbd^T.qv
 *                       is one K = B*T GEMM per head); feeds dqv = scale dbd.p
 *   dk, dv [B*T, lddkv] dL/dk, dL/dv (may be the k / v slots of dqkv). */
int lasr_relattn_bwd(const void* qu, const void* qv, int64_t ldq, const void* k, const void* v,
                     int64_t ldkv, const void* pos, int64_t ldp, int B, int H, int T, int dk,
                     const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                     const float* stats, const void* ctx, const void* dctx, int64_t ldc,
                     float* Dbuf, void* dqu, void* dbd, int ldS, int dbd_head_major, void* dk_out,
                     void* dv_out, int64_t lddkv, void* stream);
/* Plain scaled dot-product attention on the fused kernels (no positional term), Tq queries
 * and Tk keys per utterance (liteasr/nets/attention.py:41-71, the decoder's self and source
 * attention): q [B*Tq, ldq], k / v [B*Tk, ldkv], mask[b*mask_sb + i*mask_sq + j] != 0 ->
 * masked (-1e38 before the softmax), stats / ctx as lasr_relattn_fwd.  No attention dropout. */
int lasr_attn_fwd(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                  int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                  float* stats, void* ctx, int64_t ldc, void* stream);
/* Backward of lasr_attn_fwd (recompute): dq [B*Tq, ldq], dk / dv [B*Tk, lddkv]; Dbuf
 * [B*H*Tq] scratch. */
int lasr_attn_bwd(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                  int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                  const float* stats, const void* ctx, const void* dctx, int64_t ldc, float* Dbuf, void* dq,
                  void* dk_out, void* dv_out, int64_t lddkv, void* stream);
/* The same two with the key blocks split over nsplit workgroups per query block (1 <=
 * nsplit <= ceil(Tk / 64)) and combined in a second launch, for few query blocks over long
 * key runs (the decoder's source attention).  The results are those of the one-pass entries
 * up to fp32 summation order.  work: 16-B aligned fp32 scratch of lasr_attn_split_work floats.
 * lasr_attn_split_count suggests nsplit (1 = no split) for a shape. */
int lasr_attn_fwd_split(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                        int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                        float* stats, void* ctx, int64_t ldc, int nsplit, float* work, int64_t work_floats,
                        void* stream);
int lasr_attn_bwd_split(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                        int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                        const float* stats, const void* ctx, const void* dctx, int64_t ldc, float* Dbuf, void* dq,
                        void* dk_out, void* dv_out, int64_t lddkv, int nsplit, float* work, int64_t work_floats,
                        void* stream);
int64_t lasr_attn_split_work(int B, int H, int Tq, int dk, int nsplit);
int lasr_attn_split_count(int B, int H, int Tq, int Tk);
/* dst[t, h*dk + c] = sum_b src[b,h,t,c]  (pos-projection grad reduced over batch). */
int lasr_reduce_batch(const float* src, int B, int H, int T, int dk, void* dst, int dt,
                      void* stream);

/* ------------------------------------------------------------------------
 * Conv2d subsampling (liteasr/nets/subsampling.py:31-47), channels-last layout.
 * conv1: x [B,T,F] fp32 -> y1 [B,T1,F1,C] = relu(conv3x3s2(x) + b)   (W1: [C,9])
 * conv1 bwd: dW1[C,9], db1[C] from dy1 (pre-masked by relu').
 * im2col: y1 -> col [B*T2*F2, 9*C] (k = (kh*3+kw)*C + cin).
 * col2im: dcol -> dy1 (sum of the <=4 taps), multiplied by relu'(y1).
 * ---------------------------------------------------------------------- */
int lasr_conv1_fwd(const float* x, int B, int T, int F, int C, const float* w,
                   const float* bias, void* y1, int dt, void* stream);
int lasr_conv1_bwd(const float* x, int B, int T, int F, int C, const void* dy1, int dt,
                   float* dw, float* db, float* workspace, int64_t ws_floats, void* stream);
int lasr_im2col3x3s2(const void* y1, int dt, int B, int T1, int F1, int C, void* col,
                     void* stream);
int lasr_col2im3x3s2(const void* dcol, int dt, int B, int T1, int F1, int C,
                     const void* y1, void* dy1, void* stream);
/* conv2 as implicit GEMMs on the LDS-DMA MFMA kernel (no im2col / col2im buffers):
 *  LASR_CONV2_FWD: out = y2 [M2, C] bf16 = relu(im2col(y1) W2p^T + bias)         (y1, w2p, bias)
 *  LASR_CONV2_DW : out = dW [C, 9C] fp32 = dy2^T im2col(y1); rowsum (nullable) += column
 *                  sums of dy2 (db2)                                        (dy2, y1, workspace)
 *  LASR_CONV2_DX : out = dy1 [B,T1,F1,C] bf16 = col2im(dy2 W2p) * relu'(y1)      (dy2, w2p, y1)
 * M2 = B*T2*F2 (T2 = (T1-3)/2+1, F2 = (F1-3)/2+1); W2p [C, 9C] bf16 with k = (kh*3+kw)*C + cin
 * (the im2col column order above); dy2 [dy2_rows, C] bf16 with dy2_rows >=
 * max(roundup32(M2), M2 + 1) and rows M2.. zero (the weight-gradient k padding and the taps
 * that fall outside dy2).  C % 128 == 0, every pointer 16-B aligned.  DW splits K over
 * workgroups when the workspace holds split*(9C*C + C) floats (summed in fixed order).
 *  LASR_CONV2_DX_W1: the data gradient of DX consumed in place by the conv1 weight gradient
 *                  (lasr_conv1_bwd's dW1 / db1), dy1 never stored: dw1 [C, 9] += sum over
 *                  dy1 positions of dy1 (x) the 3x3 stride-2 patch of x [B, T, F] fp32 (k = kh*3
 *                  + kw), db1 [C] += sum of dy1.  Needs C % 256 == 0 and a workspace of
 *                  lasr_conv2_dx_w1_workspace(B, T1, F1, C) bytes; out unused.
 * Replaces nn.Conv2d(C, C, 3, 2)'s forward and backward at liteasr/nets/subsampling.py:42
 * (DX_W1: also the weight gradient of the first nn.Conv2d(1, C, 3, 2) there). */
#define LASR_CONV2_FWD 0
#define LASR_CONV2_DW 1
#define LASR_CONV2_DX 2
#define LASR_CONV2_DX_W1 3
typedef struct lasr_conv2_args {
  int mode;
  int B, T1, F1, C;
  const void* y1;
  const void* w2p;
  const float* bias;
  const void* dy2; int64_t dy2_rows;
  void* out;
  float* rowsum;
  void* workspace; int64_t workspace_bytes;
  /* LASR_CONV2_DX_W1 only */
  const float* x; int T, F;
  float* dw1; float* db1;
} lasr_conv2_args;
int lasr_conv2_gemm(const lasr_conv2_args* args, void* stream);
/* Workspace bytes of a LASR_CONV2_DX_W1 call (per-tile partials of dw1 / db1). */
int64_t lasr_conv2_dx_w1_workspace(int B, int T1, int F1, int C);
/* ---- Paraformer CIF predictor (liteasr/nets/paraformer/predictor.py:24-118) ----------
 * fwd: alpha[b,t] = t < plen[b] ? sigmoid(z[b,t]) : 0; sum_alpha[b] = sum_t alpha;
 *      beta = sum_alpha / ylen - 1e-4; integrate-and-fire over t (the reference's update
 *      rules, incl. state += (beta - acc) * h on non-firing frames); fired states with a
 *      non-zero |.|-sum go to out[b, 0..] in time order (rows past U dropped), the rest of
 *      out[b] is zero.  Keeps alpha, acc (accumulated weight after t), fired (u8) and row
 *      (output row of frame t, -1 for none) for the backward; mae[b] = |sum_alpha - ylen|
 *      (nullable).  h [B,T,D] fp32, D in {64, 128, 256, 512, 1024}.
 * bwd: from gout [B,U,D] and gsum [B] (the loss gradients of out and sum_alpha, both
 *      nullable): dz [B,T] (the gradient of the predictor logits, zero past plen) and
 *      dh [B,T,D] (written). */
typedef struct lasr_cif_args {
  int B, T, D, U;
  const float* z; const int* plen; const int* ylen; const float* h;
  float* alpha; float* acc; uint8_t* fired; int* row; float* sum_alpha; float* mae; float* out;
  const float* gout; const float* gsum; float* dz; float* dh;
} lasr_cif_args;
int lasr_cif_fwd(const lasr_cif_args* args, void* stream);
int lasr_cif_bwd(const lasr_cif_args* args, void* stream);
/* Glancing sampler mix (liteasr/nets/paraformer/glancing_sampler.py:32), fp32 [rows, D],
 * replace u8 [rows]: fwd out = replace ? a : b; bwd (a = the incoming gradient)
 * out = replace ? a : 0 (embedding branch), out2 = replace ? 0 : a (CIF branch). */
int lasr_glancing_mix(int64_t rows, int D, const uint8_t* replace, const float* a, const float* b,
                      float* out, float* out2, int backward, void* stream);
/* Transpose the last two dims of [N][A][Bd] into [N][Bd][A] (fp32 -> dst dtype), or
 * (reverse=1) [N][Bd][A] -> [N][A][Bd] with optional accumulate into fp32. */
int lasr_permute_last2(const void* src, int sdt, int64_t N, int64_t A, int64_t Bd, void* dst,
                       int ddt, int reverse, int accumulate, void* stream);

/* ------------------------------------------------------------------------
 * Conformer convolution module (liteasr/nets/conformer_convolution.py:44-57),
 * channels-last [B,T,C]:  glu(pw1) -> depthwise conv (K taps, pad (K-1)/2) -> BN(train)
 * -> swish -> pw2.  pw1/pw2 are lasr_gemm calls.
 * ---------------------------------------------------------------------- */
int lasr_glu_dwconv_fwd(const void* z1, int dt, int B, int T, int C, int K, const float* w,
                        const float* bias, void* y, int ydt, float* stats_ws, void* stream);
/* number of stats partials written by lasr_glu_dwconv_fwd (3*C floats each) */
int lasr_dwconv_nparts(int B, int T);
int lasr_bn_finalize(const float* stats_ws, int nparts, int C, float eps, float momentum,
                     const float* gamma, const float* beta, float* running_mean,
                     float* running_var, int64_t* num_batches, float* mean, float* rstd,
                     float* scale, float* shift, int mode, void* stream);
/* mode: 0 batch stats, 1 batch stats + running-stat update (train), 2 running stats (eval) */
int lasr_bn_act_fwd(const void* y, int ydt, int64_t rows, int C, const float* scale,
                    const float* shift, void* h, int hdt, int act, void* stream);
/* BN+activation backward: dgamma/dbeta accumulated, dy = BN'(dh * act'(u)); act is
 * LASR_ACT_SWISH (the default conv-module activation) or LASR_ACT_RELU (encoder activation
 * "relu", liteasr/nets/transformer_encoder.py:77-80).
 * batch_stats 1: train-mode BN (mean/rstd are the batch statistics, their gradient terms
 * included); 0: eval-mode BN (mean/rstd = running statistics, constants).
 * ws >= (ceil(rows/64)+1)*2*C floats. */
int lasr_bn_act_bwd(const void* y, int ydt, const void* dh, int hdt, int64_t rows, int C,
                    const float* scale, const float* shift, const float* mean,
                    const float* rstd, const float* gamma, float* dgamma, float* dbeta,
                    void* dy, int dydt, float* ws, int64_t ws_floats, int batch_stats, int act,
                    void* stream);
int lasr_glu_dwconv_bwd(const void* z1, int dt, const void* dy, int dydt, int B, int T, int C,
                        int K, const float* w, void* dz1, float* dw, float* db, float* ws,
                        int64_t ws_floats, void* stream);
/* dw [C][K] and db [C] accumulate; with dw = db = NULL the [nparts][C*K + C] partials
 * (lasr_dwconv_nparts) stay in ws for a deferred lasr_reduce_multi. */
/* lasr_bn_act_bwd followed by lasr_glu_dwconv_bwd (liteasr/nets/conformer_convolution.py:48-57
 * backward: BatchNorm + activation, then the depthwise conv and the GLU), with dy never stored:
 * the depthwise backward computes it while loading its window.  y / dh are [B*T, C] as for
 * lasr_bn_act_bwd (bn_ws: its workspace, which must not overlap ws), z1 / dz1 / w / dw / db as
 * for lasr_glu_dwconv_bwd; the same outputs, bit for bit, one launch and 8 B per element of HBM
 * traffic fewer. */
int lasr_bn_act_glu_dwconv_bwd(const void* y, int ydt, const void* dh, int hdt, int B, int T, int C,
                               const float* scale, const float* shift, const float* mean, const float* rstd,
                               const float* gamma, float* dgamma, float* dbeta, float* bn_ws,
                               int64_t bn_ws_floats, int batch_stats, int act, const void* z1, int dt, int K,
                               const float* w, void* dz1, float* dw, float* db, float* ws, int64_t ws_floats,
                               void* stream);

/* ------------------------------------------------------------------------
 * Elementwise / embedding / positional encoding
 * ---------------------------------------------------------------------- */
int lasr_cast(const void* src, int sdt, void* dst, int ddt, int64_t n, void* stream);
int lasr_scale_add(const void* a, int adt, const void* b, int bdt, float sa, float sb,
                   void* out, int odt, int64_t n, void* stream); /* out = sa*a + sb*b */
/* Decoder embedding + absolute PE (liteasr/nets/transformer_decoder.py:77-78,
 * positional_encoding.py:49-56): y[r,:] = E[ids[r],:]*xscale + pe[r % L,:], dropout; pe may
 * be NULL (plain embedding lookup).  lasr_embed_bwd: dE[ids[r]] += the rows' gradients; a
 * row with a negative id contributes nothing (nn.Embedding padding_idx). */
int lasr_embed_pe_fwd(const int32_t* ids, int R, int L, int D, const float* E,
                      const float* pe, float xscale, float p, uint64_t seed, void* y, int ydt,
                      void* stream);
int lasr_embed_bwd(const int32_t* ids, int R, int D, const void* dy, int dydt, float xscale,
                   float p, uint64_t seed, float* dE, void* stream);
/* y = x*xscale (+ pe[t]) with dropout; rows = B*T, row r uses pe row r % T. */
int lasr_pe_fwd(const void* x, int xdt, int64_t rows, int T, int D, const float* pe,
                float xscale, float p, uint64_t seed, void* y, int ydt, void* stream);

/* ------------------------------------------------------------------------
 * Transducer (liteasr/models/transducer.py) and the RNN-T loss (liteasr/criterions/rnnt.py:
 * warp-transducer RNNTLoss(blank) / warp_rnnt.rnnt_loss(reduction="mean"), both on the raw
 * joint logits with the log-softmax fused).  Lattice rows are (b, t, u) with u fastest:
 * row = (b*T + t)*U1 + u, U1 = Lmax + 1; logits / grad rows start at row*ld (ld >= V).
 * targets [B, Lmax] int32 (labels at u < tlen[b]); ilen / tlen [B] int32.
 * fwd: lse [rows], lp [rows][2] = (log p(blank), log p(next label)), alpha / beta
 *      [B][T][U1] (log space, beta includes the node's own emission) and nll [B]
 *      (= -log P(y|x); +inf when ilen = 0).  U1 <= 1024.
 * bwd: grad[row] = g * (softmax * occ - blank / label occupancies) for rows inside
 *      (ilen[b], tlen[b] + 1), 0 elsewhere; g = gscale * (*gdev if gdev) (the batch mean:
 *      gscale = 1/B).
 * ---------------------------------------------------------------------- */
int lasr_rnnt_fwd(const void* logits, int ldt, int B, int T, int U1, int V, int64_t ld, const int32_t* targets,
                  int Lmax, const int32_t* ilen, const int32_t* tlen, int blank, float* lse, float* lp,
                  float* alpha, float* beta, float* nll, void* stream);
int lasr_rnnt_bwd(const void* logits, int ldt, int B, int T, int U1, int V, int64_t ld, const int32_t* targets,
                  int Lmax, const int32_t* ilen, const int32_t* tlen, int blank, const float* lse, const float* lp,
                  const float* alpha, const float* beta, const float* nll, void* grad, int gdt, float gscale,
                  const float* gdev, void* stream);
/* Joint (transducer.py:199-203): z[(b*T + t)*U1 + u][j] = tanh(e[b*T + t][j] + d[u*B + b][j]),
 * e = lin_enc(h_enc) [B*T][J], d = lin_dec(h_dec) [U1*B][J] (time-major rows), fp32; J % 8 == 0.
 * lasr_joint_reduce: the joint inputs' gradients from dz (the tanh input gradient, rows as
 * z): de[b*T + t] = sum_u dz, dd[u*B + b] = sum_t dz, fixed summation order. */
int lasr_joint_fwd(const float* e, const float* d, int B, int T, int U1, int J, void* z, int zdt, void* stream);
int lasr_joint_reduce(const void* dz, int dzdt, int B, int T, int U1, int J, void* de, void* dd, int odt,
                      void* stream);
/* LSTMCell gate arithmetic (liteasr/nets/rnn_decoder.py:21-24,49-67; torch gate order i, f,
 * g, o) around the per-step recurrent GEMM: gates [B][ldg >= 4H] fp32 pre-activations
 * (x W_ih^T + b_ih + h W_hh^T), plus bias [4H] (nullable: b_hh) added by the cell; c_prev
 * NULL = zero state.  fwd writes c_out [B][H] fp32 and h_out [B][ldh].  bwd: dh = dh_out
 * (+ dh_rec, fp32), dc = dc_next + ..., writes the gate pre-activation gradients dgates
 * [B][lddg] and dc_prev (nullable). */
int lasr_lstm_cell_fwd(const float* gates, int64_t ldg, const float* bias, const float* c_prev, int B, int H,
                       float* c_out, void* h_out, int hdt, int64_t ldh, void* stream);
int lasr_lstm_cell_bwd(const float* gates, int64_t ldg, const float* bias, const float* c, const float* c_prev,
                       const void* dh_out, int dhdt, int64_t lddh, const float* dh_rec, const float* dc_next, int B,
                       int H, void* dgates, int gdt, int64_t lddg, float* dc_prev, void* stream);

/* ------------------------------------------------------------------------
 * U2 bookkeeping (liteasr/models/u2.py:319-358, liteasr/utils/mask.py:8-90,
 * transformer_encoder.py:117-120): int64 in -> int32/uint8 out, bit-exact.
 *   ys_in [B, L+1]  = [sos | ys(-1 -> eos)]
 *   tgt   [B, L+1]  = [ys | -1] with tgt[b, ylen[b]] = eos
 *   tgt_ctc [B, L]  = ys (int32)
 *   dec_mask [B, L+1, L+1] = (j >= ylen[b]+1) | (j > i)
 *   enc_mask [B, T'] = key padding after the two stride-2 slicings
 *   pred_len [B]    = ((xlen-1)//2-1)//2
 *   ylen32 [B]
 * ---------------------------------------------------------------------- */
int lasr_u2_prep(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B, int Tx,
                 int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in, int32_t* tgt,
                 int32_t* tgt_ctc, uint8_t* dec_mask, uint8_t* enc_mask, int32_t* pred_len,
                 int32_t* ylen32, void* stream);
/* The same with the masks' row strides (bytes): dec_mask [B, L+1, dec_ld], and in chunk mode
 * enc_mask [B, T', enc_ld]; the columns past L+1 / T' are written 1 (masked), so the masks
 * come out with the 16-B aligned rows the attention kernels stage by LDS-DMA. */
int lasr_u2_prep_ld(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B, int Tx,
                    int L, int Tsub, int sos, int eos, int chunk, int32_t* ys_in, int32_t* tgt,
                    int32_t* tgt_ctc, uint8_t* dec_mask, int dec_ld, uint8_t* enc_mask, int enc_ld,
                    int32_t* pred_len, int32_t* ylen32, void* stream);
/* Every bookkeeping output and the streaming chunk mask in one launch (config 4's
 * dynamic-chunk mask; the reference composes it as padding_mask | triangle_mask(T', stage=c),
 * liteasr/utils/mask.py:84-89, applied through the layers' mask argument,
 * liteasr/nets/transformer_encoder.py:113-120).
 *   key_mask [B, T'] key padding (NULL: not written),
 *   chunk_mask [B, T', chunk_ld] (chunk_ld >= T'; columns past T' written 1 = masked):
 *     mask[b, i, j] = (4 j >= xlen[b]) | (j div c > i div c).
 *   chunk_mode 0: no chunk mask; 1: c = chunk (> 0); 2: c = *chunk_dev (int32, device: a
 *     captured graph replays whatever the host wrote there); 3: c drawn on the device from
 *     (chunk_seed, *ctr) -- ctr the uint64 step counter -- and written to *chunk_dev when
 *     non-NULL: r uniform in [1, T'-1]; r > T'/2 -> full context, else c = r mod chunk_max + 1
 *     (WeNet's dynamic chunk distribution).  c <= 0 or c >= T' is full context.  */
int lasr_u2_prep_chunk(const int64_t* xlens, const int64_t* ys, const int64_t* ylens, int B, int L,
                       int Tsub, int sos, int eos, int chunk_mode, int chunk, int32_t* chunk_dev,
                       const uint64_t* ctr, uint64_t chunk_seed, int chunk_max, int32_t* ys_in,
                       int32_t* tgt, int32_t* tgt_ctc, uint8_t* dec_mask, int dec_ld, uint8_t* key_mask,
                       uint8_t* chunk_mask, int chunk_ld, int32_t* pred_len, int32_t* ylen32,
                       void* stream);

/* ------------------------------------------------------------------------
 * SpecAugment (liteasr/utils/transform/spec_augment.py:14-125; applied per utterance in
 * the reference's DataLoader workers, liteasr/dataset/asr_dataset.py:118).  Replaces the
 * per-utterance SpecAugment.__call__ with one batched device call on the padded batch:
 *   x, out [B, Tmax, F] fp32 (out must not alias x), xlens [B] int64 (device),
 *   plan [B, plan_stride] int32 (device): center, warped (0 = no warp), nf, nt, then nf
 *   freq and nt time [lo, hi) ranges in draw order (host-drawn with the reference's RNG
 *   calls; liteasr_amd/utils/transform/spec_augment.py).
 * Time warp = Pillow BICUBIC float resize, bit-exact; masks fill 0 (replace_with_zero) or
 * the utterance's running mean.  Rows >= xlens[b] are copied unchanged.  ws: device
 * scratch of lasr_spec_augment_ws_bytes(B, Tmax) bytes (unused with replace_with_zero).
 * ---------------------------------------------------------------------- */
int64_t lasr_spec_augment_ws_bytes(int B, int Tmax);
int lasr_spec_augment(const float* x, float* out, const int64_t* xlens, const int32_t* plan,
                      int plan_stride, int B, int Tmax, int F, int replace_with_zero, void* ws,
                      int64_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Optimizer: clip_grad_norm_ + NaN-skip + Noam/Adam over flat fp32 buffers
 * (liteasr/trainer.py:152-171, liteasr/optims/noam.py:33-46, optims/adam.py:27-34,
 *  torch.optim.Adam semantics).  State lives on the device:
 *   state[0] = successful step count (float), state[1] = last lr, state[2] = last norm,
 *   state[3] = skipped flag of the last call.
 * lr_mode 0: constant lr; 1: Noam (factor, model_dim, warmup).
 * ---------------------------------------------------------------------- */
int lasr_sumsq_nparts(int64_t n);
int lasr_sumsq_partial(const float* g, int64_t n, float* ws, int64_t ws_floats, void* stream);
/* state[5]: [0] taken steps, [1] lr of the last step, [2] grad norm, [3] skipped flag,
 * [4] clip coefficient.  ws/nparts: the lasr_sumsq_partial output (may cover several
 * gradient buffers concatenated). param_lp: optional low-precision working copy that is
 * refreshed in the same pass.  Clip coefficient = min(max_norm / (norm + 1e-6), 1) for any
 * max_norm, as torch.nn.utils.clip_grad_norm_ (0 zeroes the step's gradient; +inf = no
 * clipping). */
int lasr_adam_step(float* param, void* param_lp, int lp_dtype, const float* grad, float* m,
                   float* v, int64_t n, const float* ws, int nparts, float* state,
                   float max_norm, int lr_mode, float lr, float factor, float model_dim,
                   float warmup, float beta1, float beta2, float eps, float weight_decay,
                   void* stream);
int lasr_fill(void* dst, int dt, int64_t n, float value, void* stream);

/* ---- decoding (inference) -------------------------------------------
 * Per row of logits [rows, V] (row stride ld, dtype F32/BF16): log_softmax, then the k
 * largest log-probs in descending order (ties -> smaller index) into topk_val/topk_idx
 * [rows, k], and optionally gathered[r] = log_softmax(row r)[gather_idx[r]] (-inf when
 * the index is outside [0, V)).  Replaces the per-frame `ctc.log_softmax` + `torch.topk`
 * of liteasr/models/u2.py:221-226 and the `log_softmax(h_attn)` gather of
 * u2.py:300-313.  V <= 16384, 0 <= k <= V. */
int lasr_logsoftmax_topk(const void* logits, int dtype, int64_t rows, int V, int64_t ld, int k,
                         const int32_t* gather_idx, float* topk_val, int32_t* topk_idx,
                         float* gathered, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LITEASR_HIP_H */
