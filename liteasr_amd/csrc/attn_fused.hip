// Fused relative-position self-attention (encoder MHSA), bf16 operands, d_k = 64 or 32.
// Reference: liteasr/nets/attention.py RelativeMultiHeadAttention.forward :120-154
// (ac = (q+u) k^T, bd = rel_shift((q+v) p^T), (ac+bd)/sqrt(d_k), masked_fill(-1e38),
// softmax, attn @ v), legacy rel_shift :99-118.
//
// Nothing T x T reaches HBM in the forward: scores are rebuilt per (64-query x 64-key)
// tile in registers and the softmax is two-pass (row max / sum first, then P = exp(S -
// max) / sum feeding P.V), so the only forward outputs are ctx and the row statistics
// (max, 1/sum: 2*B*H*T floats).
//
// rel_shift as a relative-position lookup.  With m = j - i + T - 1 (0 .. 2T-2):
//   j <= i    (m <= T-1): bd = (q_i   + v) . p[m]
//   j == i+1  (m == T)  : bd = 0
//   j >= i+2  (m >= T+1): bd = (q_i+1 + v) . p[m - T - 1]
// (the closed form of attn.hip).  For a wave's 16 query rows and a 64-key block the m
// values span an 80-wide window, so the wave computes G[r][m] = qv_{row} . p[..] for that
// window on MFMA (one 16x16 tile per 16 m, the "i+1" tiles with the query fragment
// shifted by one row), parks it in LDS and gathers the diagonal it needs.
//
// Backward (flash-attention style recompute, deterministic, no atomics):
//   relattn_bwd_q  : per (b, h, 64 queries): dS = P (dP - D), dQu = scale dS K, and dS
//                    scattered back through rel_shift into dBD (the G-space gradient that
//                    the dQv / dPos GEMMs consume, the exact output of relshift_bwd)
//   relattn_bwd_kv : per (b, h, 64 keys): loops over all query blocks, dV = P^T dO,
//                    dK = scale dS^T Qu
// D_i = rowsum(dO * O) is computed once by bwd_q and read by bwd_kv.
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {

// d_k (DK) is a template parameter: 64 (small / long configs) or 32 (large, 16 heads).  The
// LDS images stay 64 columns wide; with DK = 32 only their first 32 columns are filled/read.
constexpr int GLD = 84;       // fp32 row stride of a wave's G window (80 + 4)
constexpr int PLD = 72;       // bf16 row stride of a wave's P / dS tile (64 + 8)

struct RelAttnP {
  const bf16_t *qu, *qv, *k, *v, *pos;  // qu/qv [B*T, ldq]; k/v [B*T, ldkv]; pos [T, ldp]
  int64_t ldq, ldkv, ldp;
  const uint8_t* mask;                  // mask[b*msb + i*msq + j] != 0 -> masked
  int64_t msb, msq;
  int B, H, T;
  int Tk;                               // key rows per utterance (T: self-attention; a
                                        // different count only with an all-zero pos table)
  float scale;
  float* stats;                         // [B*H*T][2]: row max, 1/row sum
  bf16_t* ctx;                          // [B*T, ldc]
  int64_t ldc;
  // backward
  const bf16_t* dctx;                   // [B*T, ldc]
  const bf16_t* ctx_in;                 // forward ctx (for D)
  float* Dbuf;                          // [B*H*T]
  bf16_t* dqu;                          // [B*T, ldq]
  bf16_t* dbd;                          // [B][H] (or [H][B] if dbd_hb) x [T, ldS]
  int ldS, dbd_hb;
  bf16_t *dk, *dv;                      // [B*T, lddkv]
  int64_t lddkv;
};

LASR_DEV bf16x8 ldg8(const bf16_t* p) { return *(const bf16x8*)p; }
LASR_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
LASR_DEV f32x4 zero4() { return (f32x4){0.f, 0.f, 0.f, 0.f}; }
LASR_DEV void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- LDS images ---------------------------------------------------------------------
// 64 x 64 blocks (K, V, Qu, dO) live in two [32 rows][64 cols] halves with the 16-col
// groups XOR-swizzled per row (gemm.hip tr_off<64>).  The same image serves both MFMA
// operand orientations: 8 consecutive columns of one row (ds_read_b128: the operand's k is
// the column axis) and the transposed read ds_read_b64_tr_b16 (k is the row axis).
LASR_DEV int tr64(int k, int col) {
  const int h = ((k >> 1) & 1) | ((k >> 2) & 2);
  return k * 64 + ((((col >> 4) ^ h)) << 4) + (col & 15);
}
LASR_DEV int img_off(int row, int col) { return (row >> 5) * 2048 + tr64(row & 31, col); }
// operand fragment, k along the columns: row = rbase + lane%16, cols kb + 8*(lane/16) .. +8
LASR_DEV bf16x8 frag_row(const bf16_t* img, int rbase, int kb, int lane) {
  return *(const bf16x8*)(img + img_off(rbase + (lane & 15), kb + 8 * (lane >> 4)));
}
// operand fragment, k along the rows (one 32-row half): col = cbase + lane%16,
// rows 8*(lane/16) .. +8
LASR_DEV bf16x8 frag_tr(const bf16_t* img, int cbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + tr64(8 * g + q, cbase + pc)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + tr64(8 * g + 4 + q, cbase + pc)));
  const short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// 64 x 64 block: global -> registers (rows clamped below nrows; 2 x 16 B per thread) ...
// (named fields, not arrays: a private array carried across the loop is put in scratch)
struct Blk {
  uint4 x0, x1;
};
template <int DK>
LASR_DEV Blk blk_fetch(const bf16_t* src, int64_t ld, int row0, int nrows, int tid) {
  constexpr int SH = DK == 64 ? 3 : 2;  // log2(16-B chunks per row)
  Blk r;
  r.x0 = *(const uint4*)(src + (int64_t)min(row0 + (tid >> SH), nrows - 1) * ld + (tid & ((1 << SH) - 1)) * 8);
  if constexpr (DK == 64)
    r.x1 = *(const uint4*)(src + (int64_t)min(row0 + 32 + (tid >> 3), nrows - 1) * ld + (tid & 7) * 8);
  return r;
}
// ... registers -> LDS image
template <int DK>
LASR_DEV void blk_store(bf16_t* img, const Blk& r, int tid) {
  constexpr int SH = DK == 64 ? 3 : 2;
  *(uint4*)(img + img_off(tid >> SH, (tid & ((1 << SH) - 1)) * 8)) = r.x0;
  if constexpr (DK == 64) *(uint4*)(img + img_off(32 + (tid >> 3), (tid & 7) * 8)) = r.x1;
}

// Relative-position window of a (64-query, 64-key) block pair: row r <-> m = mlo + r,
// mlo = j0 - i0 + T - 64, holding p[m] (m <= T-1), 0 (m == T), p[m-T-1] (m >= T+1), 0 past
// the table.  128 rows x 64, padded row stride.
constexpr int PE_ROWS = 128, PELD = 72;
// Loads are unconditional (clamped row) and the zero rows are applied at store time, so
// no wait for the prefetch is forced before the block it overlaps with.
struct PeWin {
  uint4 x[4];
  uint32_t valid;
};
template <int DK>
LASR_DEV uint4 pe_chunk(const bf16_t* ph, int64_t ldp, int T, int mlo, int u, uint32_t& valid, int it) {
  constexpr int CPR = DK / 8;  // 16-B chunks per row
  const int m = mlo + u / CPR;
  const bool v1 = m >= 0 && m <= T - 1, v2 = m >= T + 1 && m <= 2 * T;
  const int src = v1 ? m : (v2 ? m - T - 1 : 0);
  valid |= (v1 || v2 ? 1u : 0u) << it;
  return *(const uint4*)(ph + (int64_t)src * ldp + (u % CPR) * 8);
}
template <int DK>
LASR_DEV PeWin pe_fetch(const bf16_t* ph, int64_t ldp, int T, int mlo, int tid) {
  PeWin r;
  r.valid = 0;
#pragma unroll
  for (int it = 0; it < DK / 16; ++it) r.x[it] = pe_chunk<DK>(ph, ldp, T, mlo, it * 256 + tid, r.valid, it);
  return r;
}
template <int DK>
LASR_DEV void pe_store(bf16_t* img, const PeWin& r, int tid) {
  constexpr int CPR = DK / 8;
#pragma unroll
  for (int it = 0; it < DK / 16; ++it) {
    const int u = it * 256 + tid;
    *(uint4*)(img + (u / CPR) * PELD + (u % CPR) * 8) = ((r.valid >> it) & 1u) ? r.x[it] : make_uint4(0, 0, 0, 0);
  }
}

// Key-padding mask bytes of the 4 keys a lane scores (mask rows independent of the
// query): raw loads now, bits formed when the block is scored.
struct KeyMask {
  uint32_t r0, r1, r2, r3;
};
LASR_DEV void keymask_fetch(const RelAttnP& a, int b, int j0, int lane, KeyMask& km) {
  km.r0 = km.r1 = km.r2 = km.r3 = 0u;
  if (a.mask && a.msq == 0) {
    const uint8_t* mr = a.mask + (int64_t)b * a.msb;
    const int j = j0 + (lane & 15), jm = a.Tk - 1;
    km.r0 = mr[min(j, jm)];
    km.r1 = mr[min(j + 16, jm)];
    km.r2 = mr[min(j + 32, jm)];
    km.r3 = mr[min(j + 48, jm)];
  }
}
LASR_DEV uint32_t keymask_bits(const KeyMask& km) {
  return (km.r0 ? 1u : 0u) | (km.r1 ? 2u : 0u) | (km.r2 ? 4u : 0u) | (km.r3 ? 8u : 0u);
}

// Query-dependent masks (msq != 0, e.g. the streaming chunk mask): the (64 x 64) byte tile
// of a block pair is prefetched like the operands (16 B per thread, clamped, unconditional)
// and read from LDS by the score tile.
constexpr int MLD = 80;  // LDS row stride of the mask tile (16-B aligned)
struct MaskBlk {
  uint32_t w0, w1, w2, w3;
};
LASR_DEV MaskBlk mask_fetch(const RelAttnP& a, int b, int i0, int j0, int tid) {
  const int r = tid >> 2, c16 = (tid & 3) * 16, im = a.T - 1, jm = a.Tk - 1;
  const uint8_t* mr = a.mask + (int64_t)b * a.msb + (int64_t)min(i0 + r, im) * a.msq;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int e = 0; e < 16; ++e) w[e >> 2] |= (mr[min(j0 + c16 + e, jm)] ? 1u : 0u) << (8 * (e & 3));
  return MaskBlk{w[0], w[1], w[2], w[3]};
}
LASR_DEV void mask_store(uint8_t* msh, const MaskBlk& m, int tid) {
  *(uint4*)(msh + (tid >> 2) * MLD + (tid & 3) * 16) = make_uint4(m.w0, m.w1, m.w2, m.w3);
}

// Scaled, masked scores of wave w's 16 query rows (iw = i0 + 16w ..) x the 64 keys j0 ..
// from the staged K image and relative-position window.
// s[c][q]: row iw + 4*(lane/16) + q, key j0 + 16c + lane%16.  -inf past T, -1e38 masked.
template <int DK, bool RM, bool RP = true>
LASR_DEV void score_tile(const RelAttnP& a, const bf16_t* kimg, const bf16_t* peimg, const bf16x8 (&qu)[DK / 32],
                         const bf16x8 (&qv)[DK / 32], const bf16x8 (&qv1)[DK / 32], int b, int w, int iw, int j0,
                         uint32_t mbits, const uint8_t* mtile, float* gw, f32x4 (&s)[4], int lane) {
  constexpr int KS = DK / 32;
  const int T = a.T, col = lane & 15, g = lane >> 4;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = mfma(qu[ks], frag_row(kimg, 16 * c, 32 * ks, lane), acc);
    s[c] = acc;
  }
  if constexpr (!RP) {  // plain attention: no positional term
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 4 * g + q, j = j0 + 16 * c + col;
        float v = s[c][q] * a.scale;
        bool masked = (mbits >> c) & 1u;
        if constexpr (RM) masked = mtile[(16 * w + r) * MLD + 16 * c + col] != 0;
        if (j >= a.Tk) v = -INFINITY;
        else if (masked) v = -1e38f;
        s[c][q] = v;
      }
    return;
  }
  const int mb = j0 - iw - 15 + T - 1;  // first m of the wave's 80-wide window
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int lo = mb + 16 * t, m = lo + col;
    const bool n1 = lo <= T - 1 && lo + 15 >= 0;      // any m in [0, T-1]
    const bool n2 = lo + 15 >= T + 1 && lo <= 2 * T;  // any m in [T+1, 2T]
    const bf16_t* pr = peimg + (48 - 16 * w + 16 * t + col) * PELD + 8 * g;
    f32x4 g1 = zero4(), g2 = zero4();
    if (n1) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) g1 = mfma(qv[ks], *(const bf16x8*)(pr + 32 * ks), g1);
    }
    if (n2) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) g2 = mfma(qv1[ks], *(const bf16x8*)(pr + 32 * ks), g2);
    }
    const bool v1 = m >= 0 && m <= T - 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) gw[(4 * g + q) * GLD + 16 * t + col] = v1 ? g1[q] : g2[q];
  }
  lds_fence();
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * g + q, i = iw + r, j = j0 + 16 * c + col;
      float v = (s[c][q] + gw[r * GLD + 16 * c + col - r + 15]) * a.scale;
      bool masked = (mbits >> c) & 1u;
      if constexpr (RM) masked = mtile[(16 * w + r) * MLD + 16 * c + col] != 0;
      if (j >= a.Tk) v = -INFINITY;
      else if (masked) v = -1e38f;
      s[c][q] = v;
    }
  lds_fence();  // the next tile overwrites gw
}

LASR_DEV float rmax16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
LASR_DEV float rsum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Query-side fragments of 16 rows from global (A operands: row = lane%16, k = 8*(lane/16)).
template <int DK>
LASR_DEV void load_qfrags(const RelAttnP& a, int b, int h, int iw, int lane, bf16x8 (&qu)[DK / 32],
                          bf16x8 (&qv)[DK / 32], bf16x8 (&qv1)[DK / 32]) {
  constexpr int KS = DK / 32;
  const int T = a.T, col = lane & 15, g = lane >> 4;
  const int r = min(iw + col, T - 1), r1 = min(iw + col + 1, T - 1);
  const int64_t base = (int64_t)b * T;
  const bf16_t* pu = a.qu + (base + r) * a.ldq + h * DK + 8 * g;
  const bf16_t* pv = a.qv + (base + r) * a.ldq + h * DK + 8 * g;
  const bf16_t* pv1 = a.qv + (base + r1) * a.ldq + h * DK + 8 * g;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qu[ks] = ldg8(pu + 32 * ks);
    qv[ks] = ldg8(pv + 32 * ks);
    qv1[ks] = ldg8(pv1 + 32 * ks);
  }
}

// P and dS of one (16 x 64) tile: P as the forward normalised it (a fully masked row is
// uniform, attention.py:54-55), dS = P (dP - D), zero where masked (masked_fill backward),
// past T or past the rows.  dP = dO V^T with V from its staged image.
template <int DK>
LASR_DEV void dscore_tile(const RelAttnP& a, const bf16_t* vimg, const bf16x8 (&dof)[DK / 32], const f32x4 (&s)[4],
                          const float (&mx)[4], const float (&il)[4], const float (&D)[4], int iw,
                          int lane, f32x4 (&p)[4], f32x4 (&ds)[4]) {
  constexpr int KS = DK / 32;
  const int T = a.T, g = lane >> 4;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x4 dp = zero4();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) dp = mfma(dof[ks], frag_row(vimg, 16 * c, 32 * ks, lane), dp);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = iw + 4 * g + q;
      const float pv = (i < T && s[c][q] != -INFINITY) ? __expf(s[c][q] - mx[q]) * il[q] : 0.f;
      p[c][q] = pv;
      ds[c][q] = s[c][q] > -1e38f ? pv * (dp[q] - D[q]) : 0.f;
    }
  }
}

// dK, dV of one key block: loops over the query blocks; per block the Qu / dO images (A of
// the scores, B of dK / dV), query stats and the position window are staged (next block
// prefetched), the K / V fragments of the block stay in registers.
// LDS: the G windows (score_tile) and the P / dS images live in one union region (a
// barrier separates the last G read from the first P / dS write), so a workgroup takes
// <= 80 KB and two fit on a CU: the 512-workgroup grid of the small config runs in one round
// (d_k 64 with a query-dependent mask needs > 256 VGPRs: one wave per SIMD there).
template <int DK, bool RM, bool RP>
__global__ __launch_bounds__(256, (DK == 64 && RM) ? 1 : 2) void relattn_bwd_kv_kernel(RelAttnP a) {
  constexpr int KS = DK / 32;
  constexpr int GBYTES = 4 * 16 * GLD * 4, PBYTES = 2 * 64 * 64 * 2;
  __shared__ __attribute__((aligned(16))) char ush[GBYTES > PBYTES ? GBYTES : PBYTES];
  bf16_t* pimg = reinterpret_cast<bf16_t*>(ush);  // P  [i][j]
  bf16_t* simg = pimg + 64 * 64;                  // dS [i][j]
  __shared__ __attribute__((aligned(16))) bf16_t oimg[64 * 64];  // dO [i][c]
  __shared__ __attribute__((aligned(16))) bf16_t qimg[64 * 64];  // Qu [i][c]
  __shared__ __attribute__((aligned(16))) bf16_t ksh[64 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t vsh[64 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t pesh[PE_ROWS * PELD];
  __shared__ __attribute__((aligned(16))) uint8_t msh[RM ? 64 * MLD : 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z, T = a.T;
  const int j0 = blockIdx.x * 64, Tk = a.Tk;
  const int64_t base = (int64_t)b * T, kbase = (int64_t)b * Tk, zrow = ((int64_t)b * a.H + h) * T;
  const bf16_t* ph = a.pos + h * DK;
  const bf16_t* quh = a.qu + base * a.ldq + h * DK;
  const bf16_t* doh = a.dctx + base * a.ldc + h * DK;
  float* gw = reinterpret_cast<float*>(ush) + w * 16 * GLD;
  KeyMask km;
  keymask_fetch(a, b, j0, lane, km);
  const uint32_t mbits = keymask_bits(km);
  blk_store<DK>(ksh, blk_fetch<DK>(a.k + kbase * a.ldkv + h * DK, a.ldkv, j0, Tk, tid), tid);
  blk_store<DK>(vsh, blk_fetch<DK>(a.v + kbase * a.ldkv + h * DK, a.ldkv, j0, Tk, tid), tid);
  Blk rq = blk_fetch<DK>(quh, a.ldq, 0, T, tid), ro = blk_fetch<DK>(doh, a.ldc, 0, T, tid);
  PeWin rp{};
  if constexpr (RP) rp = pe_fetch<DK>(ph, a.ldp, T, j0 + T - 64, tid);
  MaskBlk mk{};
  if constexpr (RM) mk = mask_fetch(a, b, 0, j0, tid);

  f32x4 dk[DK / 16], dv[DK / 16];
#pragma unroll
  for (int t = 0; t < DK / 16; ++t) { dk[t] = zero4(); dv[t] = zero4(); }
  f32x4 s[4], p[4], ds[4];
  for (int i0 = 0; i0 < T; i0 += 64) {
    const int iw = i0 + 16 * w;
    __syncthreads();  // images of the previous query block consumed
    blk_store<DK>(qimg, rq, tid);
    blk_store<DK>(oimg, ro, tid);
    if constexpr (RP) pe_store<DK>(pesh, rp, tid);
    if constexpr (RM) mask_store(msh, mk, tid);
    // per-row operands of this wave's 16 queries (global; qv / qv1 are not staged)
    bf16x8 qu[KS], qv[KS], qv1[KS], dof[KS];
    {
      const int r = min(iw + col, T - 1), r1 = min(iw + col + 1, T - 1);
      const bf16_t* pv = a.qv + (base + r) * a.ldq + h * DK + 8 * g;
      const bf16_t* pv1 = a.qv + (base + r1) * a.ldq + h * DK + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qv[ks] = ldg8(pv + 32 * ks);
        qv1[ks] = ldg8(pv1 + 32 * ks);
      }
    }
    float mx[4], il[4], D[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = min(iw + 4 * g + q, T - 1);
      mx[q] = a.stats[2 * (zrow + i)];
      il[q] = a.stats[2 * (zrow + i) + 1];
      D[q] = a.Dbuf[zrow + i];
    }
    __syncthreads();
    rq = blk_fetch<DK>(quh, a.ldq, i0 + 64, T, tid);  // next block (unconditional, clamped)
    ro = blk_fetch<DK>(doh, a.ldc, i0 + 64, T, tid);
    if constexpr (RP) rp = pe_fetch<DK>(ph, a.ldp, T, j0 - (i0 + 64) + T - 64, tid);
    if constexpr (RM) mk = mask_fetch(a, b, i0 + 64, j0, tid);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qu[ks] = frag_row(qimg, 16 * w, 32 * ks, lane);
      dof[ks] = frag_row(oimg, 16 * w, 32 * ks, lane);
    }
    score_tile<DK, RM, RP>(a, ksh, pesh, qu, qv, qv1, b, w, iw, j0, mbits, msh, gw, s, lane);
    dscore_tile<DK>(a, vsh, dof, s, mx, il, D, iw, lane, p, ds);
    __syncthreads();  // every wave's G window consumed: the P / dS images overwrite them
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int off = img_off(16 * w + 4 * g + q, 16 * c + col);
        pimg[off] = f2bf(p[c][q]);
        simg[off] = f2bf(ds[c][q]);
      }
    __syncthreads();
    // wave w: keys j0 + 16w .. (A = P^T / dS^T rows), k = the 64 queries
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = frag_tr(pimg + ks * 2048, 16 * w, lane);
      const bf16x8 sa = frag_tr(simg + ks * 2048, 16 * w, lane);
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) {
        dv[t] = mfma(pa, frag_tr(oimg + ks * 2048, 16 * t, lane), dv[t]);
        dk[t] = mfma(sa, frag_tr(qimg + ks * 2048, 16 * t, lane), dk[t]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = j0 + 16 * w + 4 * g + q;
    if (j >= Tk) continue;
    bf16_t* pk = a.dk + (kbase + j) * a.lddkv + h * DK + col;
    bf16_t* pv = a.dv + (kbase + j) * a.lddkv + h * DK + col;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
      pk[16 * t] = f2bf(dk[t][q] * a.scale);
      pv[16 * t] = f2bf(dv[t][q]);
    }
  }
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <bool RP>
void launch_bwd_kv(const RelAttnP& a, int dk, bool rm, hipStream_t st) {
  const dim3 gk((unsigned)cdiv(a.Tk, 64), (unsigned)a.H, (unsigned)a.B);
  if (dk == 64 && rm) relattn_bwd_kv_kernel<64, true, RP><<<gk, 256, 0, st>>>(a);
  else if (dk == 64) relattn_bwd_kv_kernel<64, false, RP><<<gk, 256, 0, st>>>(a);
  else if (rm) relattn_bwd_kv_kernel<32, true, RP><<<gk, 256, 0, st>>>(a);
  else relattn_bwd_kv_kernel<32, false, RP><<<gk, 256, 0, st>>>(a);
}

}  // namespace

// Key-side backward (dK, dV over all query blocks), after the query-side kernel of
// attn_flash.hip has written D = rowsum(dO * O) to Dbuf.  Argument checks: the callers
// (lasr_relattn_bwd / lasr_attn_bwd).
int lasr_attn_bwd_kv_launch(const void* qu, const void* qv, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                            const void* pos, int64_t ldp, int B, int H, int T, int Tk, int dk, const uint8_t* mask,
                            int64_t mask_sb, int64_t mask_sq, float scale, const float* stats, const void* dctx,
                            int64_t ldc, const float* Dbuf, void* dk_out, void* dv_out, int64_t lddkv, bool rp,
                            void* stream) {
  RelAttnP a = {};
  a.qu = (const bf16_t*)qu; a.qv = (const bf16_t*)qv; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.pos = (const bf16_t*)pos;
  a.ldq = ldq; a.ldkv = ldkv; a.ldp = ldp;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = T; a.Tk = Tk; a.scale = scale;
  a.stats = (float*)stats; a.ldc = ldc;
  a.dctx = (const bf16_t*)dctx; a.Dbuf = (float*)Dbuf;
  a.dk = (bf16_t*)dk_out; a.dv = (bf16_t*)dv_out; a.lddkv = lddkv;
  const bool rm = mask && mask_sq != 0;
  if (rp) launch_bwd_kv<true>(a, dk, rm, (hipStream_t)stream);
  else launch_bwd_kv<false>(a, dk, rm, (hipStream_t)stream);
  return lasr_check_launch("attn_bwd_kv");
}
