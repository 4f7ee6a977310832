// Fused relative-position / plain attention, transposed-score formulation (gfx950), bf16
// operands, d_k 64 or 32.  Reference: liteasr/nets/attention.py RelativeMultiHeadAttention
// .forward :120-154 (ac = (q+u) k^T, bd = rel_shift((q+v) p^T), (ac+bd)/sqrt(d_k),
// masked_fill(-1e38), softmax, attn @ v), legacy rel_shift :99-118; MultiHeadedAttention
// :24-73 for the plain (decoder) case.
//
// Layout of the work.  A workgroup of NW waves owns 16*NW queries of one (b, h); wave w owns
// the 16 queries iw = i0 + 16w ..  Key blocks of 64 stream through a 2-stage LDS ring filled by
// LDS-DMA (global_load_lds_dwordx4, no register staging): K, V, the relative-position window
// and (query-dependent masks) the mask tile of the block pair.  Scores are formed TRANSPOSED,
// S^T[key][query] = K . Qu^T on v_mfma_f32_16x16x32_bf16, so a lane owns ONE query (its
// column) and 4 consecutive keys per 16-key tile:
//   * the online softmax is per lane: a block max needs two cross-lane steps (the 4 lane
//     groups of a query), the running sum none until the end;
//   * P^T never leaves the registers: it is the B operand of O^T = V^T P^T as it stands, with
//     the k slots of a 32-key sub-block ordered {4g..4g+3 of tile 2ks, 4g..4g+3 of tile
//     2ks+1} and the V^T operand read in that same key order by ds_read_b64_tr_b16.
// rel_shift as a relative-position lookup (the closed form of attn.hip): with m = j - i + T - 1
//   j <= i   : bd = (q_i + v) . p[m]        j == i+1 : bd = 0
//   j >= i+2 : bd = (q_{i+1} + v) . p[m - T - 1]
// i.e. bd = G1[i][m] (m <= T-1) or G2[i][m] (m >= T) over the window table W[m] = p[m]
// (0 <= m < T), 0 (m = T), p[m-T-1] (T < m <= 2T); G1/G2 = (qv_i / qv_{i+1}) . W[m].  A wave's
// 16 queries x 64 keys span an 80-row window of W: G'[m][query] for it is 5 MFMA tiles, parked
// in the wave's LDS scratch as [query][m] (one 16-B write per tile and lane) and read back
// along the diagonal m = (j - j0) - (i - iw) + 15.
#include "common.h"
#include "tile.h"

// compile-time ablation knob (measurement builds only; 0 in the product): bit 1 drops the
// query-side backward's dBD stores, bit 2 the key-side backward's positional term
#ifndef LASR_ATTN_EXP
#define LASR_ATTN_EXP 0
#endif

namespace {

constexpr int KB = 64;   // keys per block
// A wave's G' scratch: [16 queries][80 m] fp32, query row `col` starting at float gro(col).
// The row starts are chosen so that both the parking writes (ds_write_b128 of 4 consecutive m,
// 8-lane groups) and the diagonal reads (ds_read_b32, lane (g, col) at gro(col) - col + 4g +
// const) are bank-conflict free: gro(col) = 16-B aligned, gro(col) - col over the 16 rows
// takes 16 residues mod 32 whose +4 shifts are the other 16, and each 8-row write group
// starts its rows on 8 distinct 4-bank groups (a stride of 84 was 2-way conflicted on
// every diagonal read).
constexpr int GWAVE = 1500;  // floats per wave (gro(15) + 80)
LASR_DEV int gro(int col) {
  constexpr int t[16] = {0, 100, 188, 280, 364, 464, 552, 660, 760, 860, 948, 1040, 1124, 1224, 1312, 1420};
  return t[col];
}
// The lane's two G' scratch addresses (bytes), computed once per kernel: the parking writes
// (+64t) and the diagonal reads (+4(16c + e)).  (Inside the block loop the table lookup would be
// re-issued as a global load behind every asm memory clobber, and its wait would drain the
// LDS-DMA ring.)
struct GAddr {
  uint32_t wq, diag;
};
LASR_DEV GAddr gaddr(uint32_t gq, int lane) {
  const int g = lane >> 4, col = lane & 15, r = gro(col);
  return GAddr{gq + 4u * (uint32_t)(r + 4 * g), gq + 4u * (uint32_t)(r - col + 4 * g + 15)};
}

struct FlashP {
  const bf16_t *qu, *qv, *k, *v, *pos;  // qu/qv [B*T, ldq]; k/v [B*Tk, ldkv]; pos [T, ldp]
  int64_t ldq, ldkv, ldp;
  const uint8_t* mask;                  // mask[b*msb + i*msq + j] != 0 -> masked
  int64_t msb, msq;
  int B, H, T, Tk;
  float scale;
  float* stats;                         // [B*H*T][2]: row max (scaled-score units), 1/row sum
  bf16_t* ctx;
  int64_t ldc;
  // backward (query side)
  const bf16_t* dctx;                   // [B*T, ldc]
  const bf16_t* ctx_in;                 // forward output (for D = rowsum(dO * O))
  float* Dbuf;                          // [B*H*T]
  bf16_t* dqu;                          // [B*T, ldq]
  bf16_t* dbd;                          // [B][H] (or [H][B] if dbd_hb) x [T, ldS]
  int ldS, dbd_hb;
  // plain attention only: the key blocks split over nsplit workgroups per query block (few
  // query blocks, long key runs: the decoder's source attention); each writes its partial
  // O (forward; dQ in the backward) to opart [nsplit][B*H*T][DK] fp32 and its (max, sum) to
  // mpart [nsplit][B*H*T][2], combined in split order by a second launch
  int nsplit;
  float *opart, *mpart;
  // forward with the positional biases folded in (lasr_relattn_fwd_qb): q rows [B*T, ldqin]
  // (the fused projection's q slot) and pos_bias_u / v [H*d_k] fp32; the kernel forms
  // qu = q + u and qv = q + v in registers and stores them to qu / qv (ldq) for the backward
  const bf16_t* qin;
  int64_t ldqin;
  const float *bu, *bv;
};

// bf16 zero row: the relative-position window's rows outside the table (m == T, past 2T)
__device__ __attribute__((aligned(16))) bf16_t g_zero_row[64];

// One image layout serves both MFMA operand orientations: row r of DK bf16, its 16-column
// (32-B) slots XOR-swizzled by hq(r).  A row fragment (8 consecutive columns of one row,
// ds_read_b128: 16 rows per lane group) and the transposed read (4 consecutive rows of one
// column, ds_read_b64_tr_b16: 8 rows x one 32-B slot per 32-lane group) are both bank-conflict
// free on it.  d_k 64 (two rows per 256 B): the slot of the 4 same-parity rows of any 8
// consecutive rows must differ, so hq = (r >> 1) & 3 (the round-4 form, bit 1 | bit 3 << 1,
// was 2-way conflicted on every transposed read).
template <int DK>
LASR_DEV int hq(int r) {
  if constexpr (DK == 64) return (r >> 1) & 3;
  else return (r >> 2) & 1;
}
template <int DK>
LASR_DEV int toff(int r, int c) {
  return r * DK + ((((c >> 4) ^ hq<DK>(r))) << 4) + (c & 15);
}
// image chunk P (16 B) of a row-major [rows][DK] image -> (row, logical first column)
template <int DK>
LASR_DEV void chunk_rc(int P, int& r, int& col) {
  constexpr int CPR = DK / 8;
  r = P / CPR;
  const int ps = P % CPR;
  col = (((ps >> 1) ^ hq<DK>(r)) << 4) | ((ps & 1) << 3);
}

LASR_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
LASR_DEV f32x4 zero4() { return (f32x4){0.f, 0.f, 0.f, 0.f}; }

// LDS reads in inline asm: invisible to hipcc's waitcnt pass, which would otherwise drain the
// LDS-DMA ring (vmcnt(0)) before every read it cannot prove disjoint from the DMA.  Callers
// wait with lgkm_wait<>() before using the results.
LASR_DEV v4i lds_b128(uint32_t addr) {
  v4i r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
LASR_DEV v2i lds_tr(uint32_t addr) {
  v2i r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
LASR_DEV void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// wait until at most N of the wave's LDS operations are outstanding (they retire in order)
template <int N>
LASR_DEV void lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt is 4 bits");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
// After lgkm0(): route every asm-read register through an empty asm so its consumers depend on
// a statement ordered after the wait (volatile asm statements keep their relative order).
template <typename T>
LASR_DEV void keep(T& x) { asm volatile("" : "+v"(x)); }

LASR_DEV uint32_t ldsa(const void* p) { return (uint32_t)(uintptr_t)(lptr_t)p; }

// row fragment (A or B operand with k along the image columns): rows rbase + lane%16,
// columns kb + 8*(lane/16) .. +8
template <int DK>
LASR_DEV uint32_t frag_row_addr(uint32_t img, int rbase, int kb, int lane) {
  return img + 2u * (uint32_t)toff<DK>(rbase + (lane & 15), kb + 8 * (lane >> 4));
}
// transposed fragment half: image rows k0 .. k0+3 of column cbase + lane%16 (the lane's own
// address is row k0 + (lane>>2)&3, columns cbase + 4*(lane&3) .. +3)
template <int DK>
LASR_DEV uint32_t frag_tr_addr(uint32_t img, int k0, int cbase, int lane) {
  return img + 2u * (uint32_t)toff<DK>(k0 + ((lane >> 2) & 3), cbase + (lane & 3) * 4);
}
LASR_DEV bf16x8 as_frag(v4i r) { return __builtin_bit_cast(bf16x8, r); }
LASR_DEV bf16x8 as_frag(v2i lo, v2i hi) {
  const v4i v = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8, v);
}
LASR_DEV bf16x8 pack8(const f32x4& a, const f32x4& b) {
  const v4i v = {(int)pk_bf16(a[0], a[1]), (int)pk_bf16(a[2], a[3]), (int)pk_bf16(b[0], b[1]),
                 (int)pk_bf16(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, v);
}

LASR_DEV float xmax16_32(float v) {  // max over the 4 lane groups of a column (lanes l, l^16, l^32, l^48)
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
LASR_DEV float xsum16_32(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// ---- stage geometry -------------------------------------------------------------------
// A ring stage is [K image | V image | W window | mask tile], contiguous, filled by one
// linear LDS-DMA sweep: every thread issues GL 16-B pieces; region boundaries are multiples
// of 64 pieces so a wave instruction never straddles two regions.
template <int DK, int NW, bool RP, bool RM>
struct Geo {
  static constexpr int NT = NW * 64, QB = 16 * NW, CPR = DK / 8;
  static constexpr int K_CH = KB * CPR, V_CH = KB * CPR;
  static constexpr int W_ROWS0 = RP ? KB + QB : 0;  // >= 64 + 16 NW - 1 rows of the window
  static constexpr int M_CH = RM ? QB * (KB / 16) : 0;
  static constexpr int BASE = K_CH + V_CH + M_CH;
  // pad the window so the stage is a whole number of sweeps
  static constexpr int W_CH0 = W_ROWS0 * CPR;
  static constexpr int TOT = ((BASE + W_CH0 + NT - 1) / NT) * NT;
  static constexpr int W_CH = TOT - BASE;
  static constexpr int W_ROWS = W_CH / CPR;
  static constexpr int GL = TOT / NT;
  static constexpr int STAGE_BYTES = TOT * 16;
  // region starts (pieces)
  static constexpr int K0 = 0, V0 = K_CH, W0 = K_CH + V_CH, M0 = W0 + W_CH;
  static_assert(K_CH % 64 == 0 && V_CH % 64 == 0 && M_CH % 64 == 0 && W_CH % 64 == 0, "wave-aligned regions");
  static_assert(!RP || W_ROWS >= KB + QB - 1, "window rows");
  static_assert(RP || W_CH == 0, "no window without the positional term");
};

// LDS-DMA of one region of a stage: CH pieces (a multiple of 64), piece p of the region from
// src(p); thread tid issues pieces tid, tid + NT, ... (wave-uniform: a wave instruction covers
// 64 consecutive pieces).  The ring waits use vmcnt(0), so waves may issue different counts.
template <int CH, int NT, typename Src>
LASR_DEV void dma_region(char* st, int base, int tid, Src src) {
  const int wid = tid >> 6;
#pragma unroll
  for (int k = 0; k < (CH + NT - 1) / NT; ++k) {
    const int p = k * NT + tid;
    if (CH % NT == 0 || k * NT + wid * 64 < CH)
      __builtin_amdgcn_global_load_lds((gptr_t)src(p), (lptr_t)(st + (size_t)(base + k * NT + wid * 64) * 16), 16, 0, 0);
  }
}

// relative-position window row r of a block pair whose row 0 is m = mlo (zero rows outside the table)
LASR_DEV const void* wrow(const FlashP& a, int h, int DK, int m, int c) {
  const int T = a.T;
  const int src_row = m >= 0 && m <= T - 1 ? m : (m >= T + 1 && m <= 2 * T ? m - T - 1 : -1);
  return src_row >= 0 ? (const void*)(a.pos + (int64_t)src_row * a.ldp + h * DK + c) : (const void*)(g_zero_row + c);
}

// One block pair's LDS-DMA sweep into stage `st` (shared by the forward and the query-side
// backward).
template <int DK, int NW, bool RP, bool RM>
LASR_DEV void issue_stage(const FlashP& a, int b, int h, int i0, int j0, char* st, int tid) {
  using Gm = Geo<DK, NW, RP, RM>;
  const int T = a.T, Tk = a.Tk;
  const int64_t kb = (int64_t)b * Tk;
  const bf16_t* kh = a.k + kb * a.ldkv + h * DK;
  const bf16_t* vh = a.v + kb * a.ldkv + h * DK;
  // (uniform branches) a block whose 64 key rows all exist, and a window that lies on one side
  // of m = T, take a uniform base plus the thread's loop-invariant 32-bit offset per piece;
  // only the last key block and the window straddling m = T clamp / select per piece
  if (j0 + KB <= Tk) {
    const bf16_t* kj = kh + (int64_t)j0 * a.ldkv;
    const bf16_t* vj = vh + (int64_t)j0 * a.ldkv;
    dma_region<Gm::K_CH, Gm::NT>(st, Gm::K0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return (const void*)(kj + (uint32_t)(r * a.ldkv + c));
    });
    dma_region<Gm::V_CH, Gm::NT>(st, Gm::V0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return (const void*)(vj + (uint32_t)(r * a.ldkv + c));
    });
  } else {
    dma_region<Gm::K_CH, Gm::NT>(st, Gm::K0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return (const void*)(kh + (int64_t)min(j0 + r, Tk - 1) * a.ldkv + c);
    });
    dma_region<Gm::V_CH, Gm::NT>(st, Gm::V0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return (const void*)(vh + (int64_t)min(j0 + r, Tk - 1) * a.ldkv + c);
    });
  }
  if constexpr (RP) {
    const int mb = j0 - i0 + T - Gm::QB;  // m of window row 0
    const bool lo_side = mb >= 0 && mb + Gm::W_ROWS <= T;              // rows p[m]
    const bool hi_side = mb >= T + 1 && mb + Gm::W_ROWS <= 2 * T + 1;  // rows p[m - T - 1]
    if (lo_side || hi_side) {
      const bf16_t* wb = a.pos + (int64_t)(lo_side ? mb : mb - T - 1) * a.ldp + h * DK;
      dma_region<Gm::W_CH, Gm::NT>(st, Gm::W0, tid, [&](int p) {
        int r, c;
        chunk_rc<DK>(p, r, c);
        return (const void*)(wb + (uint32_t)(r * a.ldp + c));
      });
    } else {
      dma_region<Gm::W_CH, Gm::NT>(st, Gm::W0, tid, [&](int p) {
        int r, c;
        chunk_rc<DK>(p, r, c);
        return wrow(a, h, DK, mb + r, c);
      });
    }
  }
  if constexpr (RM)
    // mask tile [query r][64 keys] bytes: rows 16-B aligned (host-checked); a piece starting
    // past the row stride holds only keys >= Tk (masked anyway): clamped
    dma_region<Gm::M_CH, Gm::NT>(st, Gm::M0, tid, [&](int p) {
      const int r = p >> 2;
      const int64_t col = min<int64_t>(j0 + (p & 3) * 16, a.msq - 16);
      return (const void*)(a.mask + (int64_t)b * a.msb + (int64_t)min(i0 + r, T - 1) * a.msq + col);
    });
}

// Query-side fragments of the lane's query (B operands: n = lane%16, k = 8*(lane/16) ..).
template <int DK>
LASR_DEV void load_q(const bf16_t* base, int64_t ld, int row, int h, int lane, bf16x8 (&f)[DK / 32]) {
  const bf16_t* p = base + (int64_t)row * ld + h * DK + 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < DK / 32; ++ks) f[ks] = *(const bf16x8*)(p + 32 * ks);
}

// q + bias for one query fragment (8 columns): the fp32 sum rounded to bf16 (RNE), exactly
// lasr_qbias_fwd's arithmetic
LASR_DEV bf16x8 qbias_frag(bf16x8 q, const float* bias) {
  const v4i qi = __builtin_bit_cast(v4i, q);
  const float4 b0 = *(const float4*)bias, b1 = *(const float4*)(bias + 4);
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  v4i r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __builtin_bit_cast(float, (uint32_t)qi[i] << 16) + bb[2 * i];
    const float hi = __builtin_bit_cast(float, (uint32_t)qi[i] & 0xffff0000u) + bb[2 * i + 1];
    r[i] = (int)pk_bf16(lo, hi);
  }
  return __builtin_bit_cast(bf16x8, r);
}

// LDS of the forward: 2 ring stages, the waves' G' scratch (RP), the key-padding bytes (!RM)
constexpr int KMASK_BYTES = 8192;  // Tk <= 8192 (host-checked)
template <int DK, int NW, bool RP, bool RM>
constexpr int fwd_lds() {
  return 2 * Geo<DK, NW, RP, RM>::STAGE_BYTES + (RP ? NW * GWAVE * 4 : 0) + (RM ? 0 : KMASK_BYTES);
}

// ---- forward, pipelined -------------------------------------------------------------------
// Per-lane LDS byte offsets of a block's fragment reads relative to its stage (computed once):
// every read of a block is base + a compile-time immediate (rows +16 keep the swizzle), so the
// address arithmetic per block is one add per base for the stage.
template <int DK, int NW, bool RP, bool RM>
struct FragOffs {
  uint32_t k[DK / 32];   // K row fragments: key rows lane%16 (+16c), columns 32ks + 8(lane/16)
  uint32_t w[DK / 32];   // the wave's window rows wb + lane%16 (+16t)
  uint32_t v[DK / 16];   // transposed fragments of a [64][DK] image (V^T, K^T): rows 4(lane/16) + (lane/4)%4
                         // (+32ks +16h), column slot t; relative to the image (region offset as immediate)
};
template <int DK, int NW, bool RP, bool RM>
LASR_DEV FragOffs<DK, NW, RP, RM> frag_offs(int w, int lane) {
  using Gm = Geo<DK, NW, RP, RM>;
  FragOffs<DK, NW, RP, RM> o;
  const int wb = 16 * (NW - 1 - w);
#pragma unroll
  for (int ks = 0; ks < DK / 32; ++ks) {
    o.k[ks] = 2u * (uint32_t)toff<DK>(lane & 15, 32 * ks + 8 * (lane >> 4));
    o.w[ks] = Gm::W0 * 16u + 2u * (uint32_t)toff<DK>(wb + (lane & 15), 32 * ks + 8 * (lane >> 4));
  }
#pragma unroll
  for (int t = 0; t < DK / 16; ++t)
    o.v[t] = 2u * (uint32_t)toff<DK>(4 * (lane >> 4) + ((lane >> 2) & 3), 16 * t + (lane & 3) * 4);
  return o;
}

// A block's score-side fragments in registers: K (A operand of S^T), the window (A operand of
// G'^T), the mask words of the lane's 4 keys per 16-key tile.
template <int DK, bool RP>
struct KWFrags {
  v4i rk[4][DK / 32];
  v4i rw[RP ? 5 : 1][DK / 32];
  uint32_t mw[4];
};

// Issue (no wait) every score-side LDS read of the block in stage `sb` (LDS byte address):
// 4*KS K fragments, then 5*KS window fragments (RP), then the 4 mask words -- in that order, so
// counted lgkm waits release K first.  km: the key-padding byte image (!RM), row-relative.
template <int DK, int NW, bool RP, bool RM>
LASR_DEV void issue_kw(uint32_t sb, const FragOffs<DK, NW, RP, RM>& o, uint32_t kmaddr, int w, int lane,
                       KWFrags<DK, RP>& f) {
  using Gm = Geo<DK, NW, RP, RM>;
  constexpr int KS = DK / 32;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const uint32_t a = sb + o.k[ks];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.rk[c][ks]) : "v"(a), "i"(c * 16 * DK * 2));
  }
  if constexpr (RP) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint32_t a = sb + o.w[ks];
#pragma unroll
      for (int t = 0; t < 5; ++t)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.rw[t][ks]) : "v"(a), "i"(t * 16 * DK * 2));
    }
  }
  const int g = lane >> 4, col = lane & 15;
  const uint32_t mimg = RM ? sb + Gm::M0 * 16u + (uint32_t)((16 * w + col) * KB + 4 * g) : kmaddr + (uint32_t)(4 * g);
#pragma unroll
  for (int c = 0; c < 4; ++c) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(f.mw[c]) : "v"(mimg), "i"(16 * c));
}

// One relative-position window tile G'^T (16 m x 16 queries) against qv (rows m <= T) or qv1
// (rows m >= T): the window's row m = T is a zero row, so a tile on one side of it needs one
// operand; the tile that straddles it takes both and selects per element.
template <int KS>
LASR_DEV f32x4 gtile(const v4i (&rw)[KS], const bf16x8 (&qv)[KS], const bf16x8 (&qv1)[KS], int lo, int T, int g) {
  f32x4 r;
  if (lo + 15 <= T) {
    r = mfma(as_frag(rw[0]), qv[0], zero4());
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) r = mfma(as_frag(rw[ks]), qv[ks], r);
  } else if (lo >= T) {
    r = mfma(as_frag(rw[0]), qv1[0], zero4());
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) r = mfma(as_frag(rw[ks]), qv1[ks], r);
  } else {
    f32x4 g1 = mfma(as_frag(rw[0]), qv[0], zero4()), g2 = mfma(as_frag(rw[0]), qv1[0], zero4());
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) {
      g1 = mfma(as_frag(rw[ks]), qv[ks], g1);
      g2 = mfma(as_frag(rw[ks]), qv1[ks], g2);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = lo + 4 * g + e <= T - 1 ? g1[e] : g2[e];
  }
  return r;
}

// Scaled + masked transposed scores (log2 units) of the lane's query against the block's 64
// keys from fragments already in registers (issue_kw): s[c][e] for key j0 + 16c + 4(lane/16) + e.
// Returns whether a per-element select was
// needed (masked key or the last block).
template <int DK, int NW, bool RP, bool RM>
LASR_DEV bool scores_kw(const FlashP& a, KWFrags<DK, RP>& f, GAddr ga, const bf16x8 (&qu)[DK / 32],
                        const bf16x8 (&qv)[DK / 32], const bf16x8 (&qv1)[DK / 32], int mlo, int j0, float c2,
                        int lane, f32x4 (&s)[4]) {
  constexpr int KS = DK / 32, NWT = RP ? 5 : 0;
  const int g = lane >> 4, col = lane & 15;
  lgkm<NWT * KS + 4>();  // the K fragments
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) keep(f.rk[c][ks]);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x4 acc = mfma(as_frag(f.rk[c][0]), qu[0], zero4());
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) acc = mfma(as_frag(f.rk[c][ks]), qu[ks], acc);
    s[c] = acc;
  }
  float bd[4][4];
  if constexpr (RP) {
    const int T = a.T;
    lgkm<4>();  // the window fragments
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) keep(f.rw[t][ks]);
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const f32x4 gt = gtile<KS>(f.rw[t], qv, qv1, mlo + 16 * t, T, g);
      // G'[query col][m - mlo = 16t + 4g + e]
      asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(ga.wq), "v"(gt), "i"(64 * t) : "memory");
    }
    // diagonal: bd(query col, key 16c + 4g + e) = G'[col][16c + 4g + e - col + 15] (the wave's
    // own writes above retire first: LDS operations of a wave complete in order)
    const uint32_t base = ga.diag;
    float v[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v[4 * c + e]) : "v"(base), "i"(4 * (16 * c + e)));
    lgkm0();
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        keep(v[4 * c + e]);
        bd[c][e] = v[4 * c + e];
      }
  } else {
    lgkm0();
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) bd[c][e] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) keep(f.mw[c]);
  const lasr_f2 c2v = {c2, c2};
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < 4; e += 2) {
      lasr_f2 x = {s[c][e], s[c][e + 1]};
      const lasr_f2 y = {bd[c][e], bd[c][e + 1]};
      x = (x + y) * c2v;
      s[c][e] = x[0];
      s[c][e + 1] = x[1];
    }
  const bool anym = __builtin_amdgcn_ballot_w64((f.mw[0] | f.mw[1] | f.mw[2] | f.mw[3]) != 0u) != 0;
  if (anym) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[c][e] = (f.mw[c] >> (8 * e)) & 0xffu ? -1e38f : s[c][e];
  }
  const bool tail = j0 + KB > a.Tk;
  if (tail) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (j0 + 16 * c + 4 * g + e >= a.Tk) s[c][e] = -INFINITY;
  }
  return anym || tail;
}

// max over the 4 lane groups of a column (lanes l, l^16, l^32, l^48) on the VALU: the gfx950
// row swaps (v_permlane16_swap: rows 0<->1, 2<->3; v_permlane32_swap: halves), no LDS round trip
LASR_DEV float xmax_rows(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = fmaxf(__builtin_bit_cast(float, (uint32_t)a[0]), __builtin_bit_cast(float, (uint32_t)a[1]));
  const uint32_t u2 = __builtin_bit_cast(uint32_t, v);
  const auto b = __builtin_amdgcn_permlane32_swap(u2, u2, false, false);
  return fmaxf(__builtin_bit_cast(float, (uint32_t)b[0]), __builtin_bit_cast(float, (uint32_t)b[1]));
}

// Forward.  A two-stage ring with the block barrier in the middle of a block: once a wave's
// reads of block j's stage are all issued and landed (the V^T fragments, read during the
// softmax), the barrier retires that stage, the DMA of block j+2 goes into it, and block j+1's
// score-side fragments are read into registers while block j's P.V products run -- the next
// block starts with its K / window / mask fragments landed.  The running max only rescales O
// and the running sum when some lane's max grew (al = 1 exactly otherwise): bit-identical.
template <int DK, int NW, bool RP, bool RM>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_fwd_kernel(FlashP a) {
  using Gm = Geo<DK, NW, RP, RM>;
  constexpr int KS = DK / 32, NT = Gm::NT;
  __shared__ __attribute__((aligned(16))) char smem[fwd_lds<DK, NW, RP, RM>()];
  char* ring = smem;                                   // 2 stages
  float* gsh = (float*)(smem + 2 * Gm::STAGE_BYTES);   // RP: NW x GWAVE floats
  uint8_t* kmask = (uint8_t*)(gsh + (RP ? NW * GWAVE : 0));  // !RM: key padding bytes
  // the wave index through readfirstlane: wave-uniform values derived from it stay in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            col = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, T = a.T, Tk = a.Tk;
  const int ns = RP ? 1 : max(a.nsplit, 1), qblk = blockIdx.x / ns, sp = blockIdx.x - qblk * ns;
  const int i0 = qblk * Gm::QB, iw = i0 + 16 * w, iq = iw + col;
  const int nb = (Tk + KB - 1) / KB;
  const int jb0 = sp * nb / ns, jb1 = (sp + 1) * nb / ns;  // this workgroup's key blocks
  const float c2 = a.scale * 1.4426950408889634f;

  issue_stage<DK, NW, RP, RM>(a, b, h, i0, jb0 * KB, ring, tid);
  if (jb0 + 1 < jb1) issue_stage<DK, NW, RP, RM>(a, b, h, i0, (jb0 + 1) * KB, ring + Gm::STAGE_BYTES, tid);
  if constexpr (!RM) {  // key padding bytes of this utterance (zeros without a mask; keys >= Tk are -inf anyway)
    const uint8_t* mr = a.mask ? a.mask + (int64_t)b * a.msb : nullptr;
    const int kpad = nb * KB;
    for (int j = tid; j < kpad; j += NT) kmask[j] = mr && j < Tk ? mr[j] : 0;
  }
  bf16x8 qu[KS], qv[KS], qv1[KS];
  if (RP && a.qin) {  // the positional biases folded in: qu / qv formed here and stored for the backward
    bf16x8 q0[KS], q1[KS];
    load_q<DK>(a.qin, a.ldqin, b * T + min(iq, T - 1), h, lane, q0);
    load_q<DK>(a.qin, a.ldqin, b * T + min(iq + 1, T - 1), h, lane, q1);
    const int cb = h * DK + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qu[ks] = qbias_frag(q0[ks], a.bu + cb + 32 * ks);
      qv[ks] = qbias_frag(q0[ks], a.bv + cb + 32 * ks);
      qv1[ks] = qbias_frag(q1[ks], a.bv + cb + 32 * ks);
    }
    if (iq < T) {
      bf16_t* du = (bf16_t*)a.qu + ((int64_t)b * T + iq) * a.ldq + cb;
      bf16_t* dv = (bf16_t*)a.qv + ((int64_t)b * T + iq) * a.ldq + cb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        *(bf16x8*)(du + 32 * ks) = qu[ks];
        *(bf16x8*)(dv + 32 * ks) = qv[ks];
      }
    }
  } else {
    load_q<DK>(a.qu, a.ldq, b * T + min(iq, T - 1), h, lane, qu);
    if constexpr (RP) {
      load_q<DK>(a.qv, a.ldq, b * T + min(iq, T - 1), h, lane, qv);
      load_q<DK>(a.qv, a.ldq, b * T + min(iq + 1, T - 1), h, lane, qv1);
    }
  }
  const FragOffs<DK, NW, RP, RM> fo = frag_offs<DK, NW, RP, RM>(w, lane);
  const uint32_t ring0 = ldsa(ring), kmaddr = ldsa(kmask);
  const GAddr ga = gaddr(ldsa(gsh + w * GWAVE), lane);
  float mrun = -INFINITY, lrun = 0.f;
  f32x4 o[DK / 16];
#pragma unroll
  for (int t = 0; t < DK / 16; ++t) o[t] = zero4();

  KWFrags<DK, RP> f;
  wait_vmcnt<0>();  // both stages' pieces and the Q loads
  lds_barrier();    // ... of every wave, and the key-padding bytes
  issue_kw<DK, NW, RP, RM>(ring0, fo, kmaddr + (uint32_t)(jb0 * KB), w, lane, f);
  for (int jb = jb0; jb < jb1; ++jb) {
    const int j0 = jb * KB;
    const int stg = (jb - jb0) & 1;
    const uint32_t sb = ring0 + (uint32_t)(stg * Gm::STAGE_BYTES);
    bool skip = false;
    if constexpr (RM) {  // (the streaming chunk mask: the blocks of future chunks)
      bool zero_byte = false;
      lgkm0();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        keep(f.mw[c]);
        zero_byte |= ((f.mw[c] - 0x01010101u) & ~f.mw[c] & 0x80808080u) != 0u;
      }
      skip = __builtin_amdgcn_ballot_w64(mrun <= -1e38f) == 0 && __builtin_amdgcn_ballot_w64(zero_byte) == 0;
    }
    f32x4 s[4];
    v2i lo[2][DK / 16], hi[2][DK / 16];
    if (!skip) {
      (void)scores_kw<DK, NW, RP, RM>(a, f, ga, qu, qv, qv1, j0 - iw + T - 16, j0, c2, lane, s);
      // V^T fragments for O^T += V^T P^T, in flight during the softmax (k slots of sub-block ks:
      // keys 32ks + 4g + e, then 32ks + 16 + 4g + e)
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) {
        const uint32_t va = sb + fo.v[t];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo[ks][t]) : "v"(va), "i"(Gm::V0 * 16 + 32 * ks * DK * 2));
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[ks][t])
                       : "v"(va), "i"(Gm::V0 * 16 + (32 * ks + 16) * DK * 2));
        }
      }
      float bm = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                       fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
      bm = fmaxf(bm, fmaxf(fmaxf(fmaxf(s[2][0], s[2][1]), fmaxf(s[2][2], s[2][3])),
                           fmaxf(fmaxf(s[3][0], s[3][1]), fmaxf(s[3][2], s[3][3]))));
      bm = xmax_rows(bm);
      const float mn = fmaxf(mrun, bm);
      float al = 1.f;
      if (__builtin_amdgcn_ballot_w64(mn > mrun) != 0) {  // some lane's max grew: rescale (al = 1 elsewhere)
        al = __builtin_amdgcn_exp2f(mrun - mn);
#pragma unroll
        for (int t = 0; t < DK / 16; ++t) o[t] *= al;
      }
      mrun = mn;
      const lasr_f2 mnv = {mn, mn};
      lasr_f2 sum2 = {0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          lasr_f2 x = {s[c][e], s[c][e + 1]};
          x -= mnv;
          x[0] = __builtin_amdgcn_exp2f(x[0]);
          x[1] = __builtin_amdgcn_exp2f(x[1]);
          s[c][e] = x[0];
          s[c][e + 1] = x[1];
          sum2 += x;
        }
      lrun = lrun * al + (sum2[0] + sum2[1]);
    }
    // mid-block: retire this block's stage, refill it with block jb+2, read block jb+1's
    // score-side fragments (landed by the next iteration)
    if (jb + 1 < jb1) {
      wait_vmcnt<0>();  // block jb+1's pieces (issued a block ago)
      lds_barrier();    // ... of every wave; every wave is done with this stage (the V^T reads landed)
      if (jb + 2 < jb1) issue_stage<DK, NW, RP, RM>(a, b, h, i0, j0 + 2 * KB, ring + stg * Gm::STAGE_BYTES, tid);
      issue_kw<DK, NW, RP, RM>(ring0 + (uint32_t)((stg ^ 1) * Gm::STAGE_BYTES), fo,
                               kmaddr + (uint32_t)(j0 + KB), w, lane, f);
    } else if (!skip) {
      lgkm0();
    }
    if (!skip) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < DK / 16; ++t) {
          keep(lo[ks][t]);
          keep(hi[ks][t]);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 pb = pack8(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
        for (int t = 0; t < DK / 16; ++t) o[t] = mfma(as_frag(lo[ks][t], hi[ks][t]), pb, o[t]);
      }
    }
  }
  // statistics in scaled-score units (max * ln 2), 1/sum: P = exp(S - max) / sum
  const float l = lrun + __shfl_xor(lrun, 16, 64);
  const float lsum = l + __shfl_xor(l, 32, 64);
  if (ns > 1) {  // a key split: unnormalised O, running max (log2 units) and sum, for the combine
    if (iq < T) {
      const int64_t row = (int64_t)sp * a.B * a.H * T + ((int64_t)b * a.H + h) * T + iq;
      if (g == 0) *(float2*)(a.mpart + 2 * row) = make_float2(mrun, lsum);
      float* op = a.opart + row * DK + 4 * g;
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) *(f32x4*)(op + 16 * t) = o[t];
    }
    return;
  }
  const float il = 1.f / lsum;
  if (iq < T) {
    if (g == 0) {  // a fully masked row keeps the masked score itself as its max (uniform P)
      float* spp = a.stats + 2 * (((int64_t)b * a.H + h) * T + iq);
      spp[0] = mrun <= -1e38f ? -1e38f : mrun * 0.6931471805599453f;
      spp[1] = il;
    }
    bf16_t* dst = a.ctx + ((int64_t)b * T + iq) * a.ldc + h * DK + 4 * g;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
      const uint2 pk = make_uint2(pk_bf16(o[t][0] * il, o[t][1] * il), pk_bf16(o[t][2] * il, o[t][3] * il));
      *(uint2*)(dst + 16 * t) = pk;
    }
  }
}

// ---- backward, query side ----------------------------------------------------------------
// Per (b, h, 16*NW queries), over the key blocks (the forward's ring, stages and transposed
// scores): P = exp(S - max) / sum from the forward's statistics, dP^T = V . dO^T, dS = P (dP - D)
// (zero where masked), dQu^T += K^T dS^T (dS^T kept in registers as the forward keeps P^T), and
// dS scattered through the inverse rel_shift into dBD, the G-space gradient the positional
// GEMMs consume (exactly relshift_bwd's output).  D_i = rowsum(dO * O) is formed here and
// stored for the key-side kernel.
template <int DK, int NW, bool RP, bool RM>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_bwd_q_kernel(FlashP a) {
  using Gm = Geo<DK, NW, RP, RM>;
  constexpr int KS = DK / 32, NT = Gm::NT;
  __shared__ __attribute__((aligned(16))) char smem[fwd_lds<DK, NW, RP, RM>()];
  char* ring = smem;
  float* gsh = (float*)(smem + 2 * Gm::STAGE_BYTES);
  uint8_t* kmask = (uint8_t*)(gsh + (RP ? NW * GWAVE : 0));
  // the wave index through readfirstlane: wave-uniform values derived from it stay in SGPRs
  // (uniform branches and scalar address arithmetic instead of exec-masked vector code)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            col = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, T = a.T, Tk = a.Tk;
  const int ns = RP ? 1 : max(a.nsplit, 1), qblk = blockIdx.x / ns, sp = blockIdx.x - qblk * ns;
  const int i0 = qblk * Gm::QB, iw = i0 + 16 * w, iq = iw + col, ic = min(iq, T - 1);
  const int nb = (Tk + KB - 1) / KB;
  const int jb0 = sp * nb / ns, jb1 = (sp + 1) * nb / ns;  // this workgroup's key blocks
  const float c2 = a.scale * 1.4426950408889634f;
  const int64_t zrow = ((int64_t)b * a.H + h) * T;

  issue_stage<DK, NW, RP, RM>(a, b, h, i0, jb0 * KB, ring, tid);
  if (jb0 + 1 < jb1) issue_stage<DK, NW, RP, RM>(a, b, h, i0, (jb0 + 1) * KB, ring + Gm::STAGE_BYTES, tid);
  if constexpr (!RM) {  // key padding bytes of this utterance (zeros without a mask; keys >= Tk are -inf anyway)
    const uint8_t* mr = a.mask ? a.mask + (int64_t)b * a.msb : nullptr;
    const int kpad = nb * KB;
    for (int j = tid; j < kpad; j += NT) kmask[j] = mr && j < Tk ? mr[j] : 0;
  }
  bf16x8 qu[KS], qv[KS], qv1[KS], dof[KS];
  load_q<DK>(a.qu, a.ldq, b * T + ic, h, lane, qu);
  load_q<DK>(a.dctx, a.ldc, b * T + ic, h, lane, dof);
  if constexpr (RP) {
    load_q<DK>(a.qv, a.ldq, b * T + ic, h, lane, qv);
    load_q<DK>(a.qv, a.ldq, b * T + min(iq + 1, T - 1), h, lane, qv1);
  }
  // the forward's statistics in log2 units (a fully masked row keeps the masked value)
  const float mx = a.stats[2 * (zrow + ic)], il = a.stats[2 * (zrow + ic) + 1];
  const float m2 = mx <= -1e38f ? -1e38f : mx * 1.4426950408889634f;
  // every row of the wave has an unmasked key (none fully masked): fully masked blocks may be skipped
  [[maybe_unused]] const bool rows_live = __builtin_amdgcn_ballot_w64(m2 <= -1e38f) == 0;
  // D_i = sum_c dO[i,c] O[i,c] on the MFMA that forms dP (the diagonal of O . dO^T over the
  // wave's 16 queries): the same products summed in the same order as dP, so dP - D cancels
  // exactly where it should (one key: P = 1, O = V)
  float D;
  {
    bf16x8 oq[KS];
    load_q<DK>(a.ctx_in, a.ldc, b * T + ic, h, lane, oq);
    f32x4 dt = zero4();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) dt = mfma(oq[ks], dof[ks], dt);
    // lane (g, col) holds rows 4g .. 4g+3 of column col: the diagonal sits in lane group col / 4
    const int e = col & 3;
    const float x = e == 0 ? dt[0] : e == 1 ? dt[1] : e == 2 ? dt[2] : dt[3];
    D = __shfl(x, ((col >> 2) << 4) | col, 64);
    if (g == 0 && iq < T && sp == 0) a.Dbuf[zrow + iq] = D;
  }
  bf16_t* dbd = RP ? a.dbd + (a.dbd_hb ? ((int64_t)h * a.B + b) * T : zrow) * a.ldS : nullptr;
  const GAddr ga = gaddr(ldsa(gsh + w * GWAVE), lane);
  f32x4 dq[DK / 16];
#pragma unroll
  for (int t = 0; t < DK / 16; ++t) dq[t] = zero4();

  const FragOffs<DK, NW, RP, RM> fo = frag_offs<DK, NW, RP, RM>(w, lane);
  const uint32_t ring0 = ldsa(ring), kmaddr = ldsa(kmask);
  KWFrags<DK, RP> f;
  wait_vmcnt<0>();  // both stages' pieces and the row loads
  lds_barrier();    // ... of every wave, and the key-padding bytes
  // the block barrier sits after the block's last reads of its stage (the K^T fragments,
  // consumed by the dQ products), where the stage is refilled with block jb+2 while the dBD
  // stores go out; the next block's score-side fragments are read at its start (prefetched
  // beside this block's live values they would spill at d_k 64)
  for (int jb = jb0; jb < jb1; ++jb) {
    const int j0 = jb * KB;
    const int stg = (jb - jb0) & 1;
    const uint32_t sb = ring0 + (uint32_t)(stg * Gm::STAGE_BYTES);
    issue_kw<DK, NW, RP, RM>(sb, fo, kmaddr + (uint32_t)j0, w, lane, f);
    f32x4 s[4];
    bool skip = false;
    if constexpr (RM) {
      bool zero_byte = false;
      lgkm0();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        keep(f.mw[c]);
        zero_byte |= ((f.mw[c] - 0x01010101u) & ~f.mw[c] & 0x80808080u) != 0u;
      }
      skip = rows_live && __builtin_amdgcn_ballot_w64(zero_byte) == 0;
    }
    v2i lo[2][DK / 16], hi[2][DK / 16];
    if (skip) {  // dS = 0 over the block: only its (zero) dBD entries are written
#pragma unroll
      for (int c = 0; c < 4; ++c) s[c] = zero4();
    } else {
      const bool msk = scores_kw<DK, NW, RP, RM>(a, f, ga, qu, qv, qv1, j0 - iw + T - 16, j0, c2, lane, s);
      // V fragments for dP^T = V . dO^T (V rows = keys as the A operand), then the K^T
      // fragments for dQu^T += K^T dS^T, in flight during dP and dS
      v4i rv[4][KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint32_t va = sb + fo.k[ks];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(rv[c][ks]) : "v"(va), "i"(Gm::V0 * 16 + c * 16 * DK * 2));
      }
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) {
        const uint32_t ka = sb + fo.v[t];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo[ks][t]) : "v"(ka), "i"(32 * ks * DK * 2));
          asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[ks][t]) : "v"(ka), "i"((32 * ks + 16) * DK * 2));
        }
      }
      lgkm<(4 * DK / 16 > 15 ? 15 : 4 * DK / 16)>();  // the V fragments (older than the K^T reads)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) keep(rv[c][ks]);
      f32x4 dp[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 acc = mfma(as_frag(rv[c][0]), dof[0], zero4());
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) acc = mfma(as_frag(rv[c][ks]), dof[ks], acc);
        dp[c] = acc;
      }
      // dS = P (dP - D), zero where masked or past Tk (the forward's masked_fill backward), on
      // packed fp32 pairs (the same roundings per element); the select only in masked blocks
      const lasr_f2 m2v = {m2, m2}, ilv = {il, il}, Dv = {D, D};
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const lasr_f2 v = {s[c][e], s[c][e + 1]};
          lasr_f2 x = v - m2v;
          x[0] = __builtin_amdgcn_exp2f(x[0]);
          x[1] = __builtin_amdgcn_exp2f(x[1]);
          const lasr_f2 dd = {dp[c][e], dp[c][e + 1]};
          x = (x * ilv) * (dd - Dv);
          s[c][e] = x[0];
          s[c][e + 1] = x[1];
          if (msk) {
            s[c][e] = v[0] > -1e38f ? s[c][e] : 0.f;
            s[c][e + 1] = v[1] > -1e38f ? s[c][e + 1] : 0.f;
          }
        }
    }
    if (!skip) {
      lgkm0();  // the K^T fragments
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int t = 0; t < DK / 16; ++t) {
          keep(lo[ks][t]);
          keep(hi[ks][t]);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 db = pack8(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
        for (int t = 0; t < DK / 16; ++t) dq[t] = mfma(as_frag(lo[ks][t], hi[ks][t]), db, dq[t]);
      }
    }
    // this block's reads of its stage are done: retire it, refill it with block jb+2 and read
    // block jb+1's score-side fragments while the dBD stores go out (placed after the dQ
    // products, whose K^T fragments would otherwise be live beside the next block's)
    if (jb + 1 < jb1) {
      wait_vmcnt<0>();  // block jb+1's pieces (and the previous block's dBD stores)
      lds_barrier();
      if (jb + 2 < jb1) issue_stage<DK, NW, RP, RM>(a, b, h, i0, j0 + 2 * KB, ring + stg * Gm::STAGE_BYTES, tid);
    }
    if constexpr (RP && !(LASR_ATTN_EXP & 1)) {
      // inverse rel_shift: the bd entry each score read (none for j == i + 1).  A lane's 4 keys
      // of a tile land on 4 consecutive columns of one dBD row unless they straddle the
      // diagonal or T: 2 or 3 stores (by column parity; ldS is even) instead of 4.
      // A block entirely below the wave's diagonal band (or above it) and inside T -- every
      // block but the one or two around the diagonal -- takes one uniform path: 4 16-bit
      // stores per tile and lane, no per-lane parity or straddle branches.
      bf16_t* const rowL = dbd + (int64_t)iq * a.ldS + (T - 1 - iq);  // + j for j <= iq
      bf16_t* const rowU = dbd + (int64_t)(iq + 1) * a.ldS - (iq + 2);  // + j for j >= iq + 2
      const bool below = j0 + KB - 1 <= iw, above = j0 >= iw + 17;
      if (j0 + KB <= T && (below || above)) {
        if (iq < T) {
          bf16_t* const row = above ? rowU : rowL;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t w01 = pk_bf16(s[c][0], s[c][1]), w23 = pk_bf16(s[c][2], s[c][3]);
            bf16_t* d = row + (j0 + 16 * c + 4 * g);
            d[0] = (bf16_t)w01;
            d[1] = (bf16_t)(w01 >> 16);
            d[2] = (bf16_t)w23;
            d[3] = (bf16_t)(w23 >> 16);
          }
        }
      } else if (iq < T) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int ja = j0 + 16 * c + 4 * g;  // first of the 4 keys
          const uint32_t w01 = pk_bf16(s[c][0], s[c][1]), w23 = pk_bf16(s[c][2], s[c][3]);
          const bool lowr = ja + 3 <= iq, highr = ja >= iq + 2;
          if ((lowr || highr) && ja + 3 < T) {
            const int64_t off = lowr ? (int64_t)iq * a.ldS + (T - 1 - iq + ja) : (int64_t)(iq + 1) * a.ldS + (ja - iq - 2);
            bf16_t* d = dbd + off;
            if ((off & 1) == 0) {
              *(uint32_t*)d = w01;
              *(uint32_t*)(d + 2) = w23;
            } else {
              *(uint16_t*)d = (uint16_t)w01;
              *(uint32_t*)(d + 1) = (w01 >> 16) | (w23 << 16);
              *(uint16_t*)(d + 3) = (uint16_t)(w23 >> 16);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int j = ja + e;
              if (j < T && j != iq + 1) {
                const int64_t off = j <= iq ? (int64_t)iq * a.ldS + (T - 1 - iq + j) : (int64_t)(iq + 1) * a.ldS + (j - iq - 2);
                dbd[off] = f2bf(s[c][e]);
              }
            }
          }
        }
      }
    }
  }
  if (ns > 1) {  // a key split: the unscaled partial dQ, summed by flash_dq_combine_kernel
    if (iq < T) {
      float* dp = a.opart + ((int64_t)sp * a.B * a.H * T + zrow + iq) * DK + 4 * g;
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) *(f32x4*)(dp + 16 * t) = dq[t];
    }
    return;
  }
  if (iq < T) {
    bf16_t* dst = a.dqu + ((int64_t)b * T + iq) * a.ldq + h * DK + 4 * g;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
      const uint2 pk = make_uint2(pk_bf16(dq[t][0] * a.scale, dq[t][1] * a.scale),
                                  pk_bf16(dq[t][2] * a.scale, dq[t][3] * a.scale));
      *(uint2*)(dst + 16 * t) = pk;
    }
  }
  // bd row 0, columns 0..T-2 are read by no score (rel_shift pads them): zero gradient
  if (RP && blockIdx.x == 0)
    for (int c = tid; c < T - 1; c += NT) dbd[c] = f2bf(0.f);
}

template <int DK, int NW, bool RP, bool RM>
void launch_bwd_q_t(const FlashP& a, hipStream_t st) {
  const dim3 grid((unsigned)(cdiv(a.T, 16 * NW) * (RP || a.nsplit < 1 ? 1 : a.nsplit)), (unsigned)a.H, (unsigned)a.B);
  flash_bwd_q_kernel<DK, NW, RP, RM><<<grid, NW * 64, 0, st>>>(a);
}

void launch_flash_bwd_q(const FlashP& a, int dk, bool rp, bool rm, hipStream_t st) {
  if (rp) {
    if (dk == 64) rm ? launch_bwd_q_t<64, 8, true, true>(a, st) : launch_bwd_q_t<64, 8, true, false>(a, st);
    else rm ? launch_bwd_q_t<32, 4, true, true>(a, st) : launch_bwd_q_t<32, 4, true, false>(a, st);
    return;
  }
  if (dk == 64) rm ? launch_bwd_q_t<64, 4, false, true>(a, st) : launch_bwd_q_t<64, 4, false, false>(a, st);
  else rm ? launch_bwd_q_t<32, 4, false, true>(a, st) : launch_bwd_q_t<32, 4, false, false>(a, st);
}

// ---- backward, key side --------------------------------------------------------------------
// Per (b, h, 16*NW keys): wave w owns 16 keys (its lanes' columns: the lane's K and V rows live in
// registers) and loops over query blocks of 64 staged by LDS-DMA (Qu, dO, Qv + one row, the
// position window, the mask tile), with the forward statistics and D of the block in a small
// double-buffered LDS slot.  Scores in the forward's orientation, S[query][key] = Qu . K^T, so
// the products with the queries as k are register-fed again: dV^T += dO^T P and dK^T += Qu^T dS,
// with P / dS of two 16-query tiles as the B operand and dO / Qu read transposed in that order.
// The positional term: a wave's 16 keys x 16 queries span 31 window rows: two MFMA tiles of
// G[query][m], parked [m][query] in the wave's scratch and read along the diagonal.
constexpr int QBK = 64;   // queries per block of the key-side kernel
// Its G scratch: [16 queries][32 m] fp32 per wave, query row q at float kro(q), parked by
// ds_write_b32 and read along the diagonal by ds_read_b32.  kro(4 + e) - kro(e) = 20 (mod 32)
// makes every diagonal read conflict free (the round-4 [32 m][16 queries] image, parked by
// b128 writes, was 4-way conflicted on those reads: 16-B aligned rows put all 32 lanes of a
// read on the 8 banks of one residue mod 4); the parking writes are at most 2-way, which costs
// a b32 store nothing.
constexpr int KWAVE = 564;  // floats per wave (kro(15) + 32)
LASR_DEV int kro(int q) { return 32 * q + 20 * ((q >> 2) & 1) + 32 * (q >> 3); }

template <int DK, int NW, bool RP, bool RM>
struct GeoKV {
  static constexpr int NT = NW * 64, KBW = 16 * NW, CPR = DK / 8;
  static constexpr int Q_CH = QBK * CPR, O_CH = QBK * CPR;
  static constexpr int QV_CH = RP ? ((QBK + 1) * CPR + 63) / 64 * 64 : 0;
  static constexpr int QV_ROWS = QV_CH / CPR;
  static constexpr int M_CH = RM ? QBK * KBW / 16 : 0;
  static constexpr int BASE = Q_CH + O_CH + QV_CH + M_CH;
  static constexpr int W_CH0 = RP ? (QBK + KBW) * CPR : 0;
  static constexpr int TOT = ((BASE + W_CH0 + NT - 1) / NT) * NT;
  static constexpr int W_CH = TOT - BASE, W_ROWS = W_CH / CPR;
  static constexpr int GL = TOT / NT, STAGE_BYTES = TOT * 16;
  static constexpr int O0 = Q_CH, QV0 = Q_CH + O_CH, M0 = QV0 + QV_CH, W0 = M0 + M_CH;
  static_assert(Q_CH % 64 == 0 && QV_CH % 64 == 0 && M_CH % 64 == 0 && W_CH % 64 == 0, "wave-aligned regions");
  static_assert(!RP || W_ROWS >= QBK + KBW - 1, "window rows");
  static_assert(RP || W_CH == 0, "no window without the positional term");
  static constexpr int LDS = 2 * STAGE_BYTES + (RP ? NW * KWAVE * 4 : 0) + 2 * 3 * QBK * 4;
};

template <int DK, int NW, bool RP, bool RM>
LASR_DEV void issue_stage_kv(const FlashP& a, int b, int h, int i0, int j0, char* st, int tid) {
  using Gm = GeoKV<DK, NW, RP, RM>;
  const int T = a.T;
  const int64_t qb = (int64_t)b * T;
  // one region at a time (uniform region bounds); a query block whose rows all exist, and a
  // window on one side of m = T, take a uniform base plus the thread's loop-invariant offset
  auto rows3 = [&](int nrows, auto&& emit) {
    if (i0 + nrows <= T) {
      emit([&](const bf16_t* base, int64_t ld, int r, int c) {
        return (const void*)(base + (qb + i0) * ld + (uint32_t)(r * ld + c));
      });
    } else {
      emit([&](const bf16_t* base, int64_t ld, int r, int c) {
        return (const void*)(base + (qb + min(i0 + r, T - 1)) * ld + c);
      });
    }
  };
  rows3(QBK, [&](auto addr) {
    dma_region<Gm::Q_CH, Gm::NT>(st, 0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return addr(a.qu + h * DK, a.ldq, r, c);
    });
    dma_region<Gm::O_CH, Gm::NT>(st, Gm::O0, tid, [&](int p) {
      int r, c;
      chunk_rc<DK>(p, r, c);
      return addr(a.dctx + h * DK, a.ldc, r, c);
    });
  });
  if constexpr (RP)
    rows3(Gm::QV_ROWS, [&](auto addr) {
      dma_region<Gm::QV_CH, Gm::NT>(st, Gm::QV0, tid, [&](int p) {
        int r, c;
        chunk_rc<DK>(p, r, c);
        return addr(a.qv + h * DK, a.ldq, r, c);
      });
    });
  if constexpr (RM)
    dma_region<Gm::M_CH, Gm::NT>(st, Gm::M0, tid, [&](int q) {
      const int rr = q / (Gm::KBW / 16), c16 = (q % (Gm::KBW / 16)) * 16;
      const int64_t col = min<int64_t>(j0 + c16, a.msq - 16);
      return (const void*)(a.mask + (int64_t)b * a.msb + (int64_t)min(i0 + rr, T - 1) * a.msq + col);
    });
  if constexpr (RP) {
    const int mb = j0 - (i0 + QBK - 1) + T - 1;  // m of window row 0
    const bool lo_side = mb >= 0 && mb + Gm::W_ROWS <= T;
    const bool hi_side = mb >= T + 1 && mb + Gm::W_ROWS <= 2 * T + 1;
    if (lo_side || hi_side) {
      const bf16_t* wb = a.pos + (int64_t)(lo_side ? mb : mb - T - 1) * a.ldp + h * DK;
      dma_region<Gm::W_CH, Gm::NT>(st, Gm::W0, tid, [&](int p) {
        int r, c;
        chunk_rc<DK>(p, r, c);
        return (const void*)(wb + (uint32_t)(r * a.ldp + c));
      });
    } else {
      dma_region<Gm::W_CH, Gm::NT>(st, Gm::W0, tid, [&](int p) {
        int r, c;
        chunk_rc<DK>(p, r, c);
        return wrow(a, h, DK, mb + r, c);
      });
    }
  }
}

template <int DK, int NW, bool RP, bool RM>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_bwd_kv_kernel(FlashP a, bf16_t* dk_out, bf16_t* dv_out,
                                                                  int64_t lddkv) {
  using Gm = GeoKV<DK, NW, RP, RM>;
  constexpr int KS = DK / 32;
  __shared__ __attribute__((aligned(16))) char smem[Gm::LDS];
  char* ring = smem;
  float* gsh = (float*)(smem + 2 * Gm::STAGE_BYTES);
  float* sst = gsh + (RP ? NW * KWAVE : 0);  // [2][3][QBK]: m (log2 units), 1/sum, D
  // the wave index through readfirstlane: wave-uniform values derived from it stay in SGPRs
  // (uniform branches and scalar address arithmetic instead of exec-masked vector code)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            col = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, T = a.T, Tk = a.Tk;
  const int j0 = blockIdx.x * Gm::KBW, jw = j0 + 16 * w, jq = jw + col;
  const int nq = (T + QBK - 1) / QBK;
  const float c2 = a.scale * 1.4426950408889634f;
  const int64_t zrow = ((int64_t)b * a.H + h) * T;

  issue_stage_kv<DK, NW, RP, RM>(a, b, h, 0, j0, ring, tid);
  // the lane's key: K and V rows (B operands), its padding byte
  bf16x8 kf[KS], vf[KS];
  load_q<DK>(a.k, a.ldkv, b * Tk + min(jq, Tk - 1), h, lane, kf);
  load_q<DK>(a.v, a.ldkv, b * Tk + min(jq, Tk - 1), h, lane, vf);
  bool kmasked = false;
  if (!RM && a.mask) kmasked = a.mask[(int64_t)b * a.msb + min(jq, Tk - 1)] != 0;
  // (key padding) any masked key among the wave's 16: the per-element selects are needed
  const bool kany = __builtin_amdgcn_ballot_w64(kmasked) != 0;
  // the block's statistics, loaded by wave 0 one block ahead
  float st_m = 0.f, st_l = 0.f, st_d = 0.f;
  auto load_stats = [&](int i0) {
    const int i = i0 + lane, ic = min(i, T - 1);
    st_m = a.stats[2 * (zrow + ic)];
    // (raw loads: the queries-past-T select happens where the value is written to LDS, after
    // the block's wait -- a select here made hipcc wait vmcnt(0) right behind the next
    // stage's LDS-DMA)
    st_l = a.stats[2 * (zrow + ic) + 1];
    st_d = a.Dbuf[zrow + ic];
  };
  if (w == 0) load_stats(0);
  // per-lane LDS offsets, hoisted: row fragments (Q / dO / Qv images, rows lane%16 (+16r), and
  // Qv shifted one query), the wave's window rows (16w + lane%16, + (48 - 16r + 16uu) as an
  // immediate), transposed fragments (rows 4g + (lane/4)%4, + 32rs / +16), the G scratch
  // parking and diagonal addresses, the RM mask byte of (row 4g, the lane's key)
  struct {
    uint32_t rq[KS], rq1[KS], w[KS], tr[DK / 16], gw[4], gr[4], mk;
  } ko;
  {
    const uint32_t gka = ldsa(gsh + w * KWAVE);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ko.rq[ks] = 2u * (uint32_t)toff<DK>(lane & 15, 32 * ks + 8 * g);
      ko.rq1[ks] = Gm::QV0 * 16u + 2u * (uint32_t)toff<DK>(1 + (lane & 15), 32 * ks + 8 * g);
      ko.w[ks] = Gm::W0 * 16u + 2u * (uint32_t)toff<DK>(16 * w + (lane & 15), 32 * ks + 8 * g);
    }
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) ko.tr[t] = 2u * (uint32_t)toff<DK>(4 * g + ((lane >> 2) & 3), 16 * t + (lane & 3) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ko.gw[e] = gka + 4u * (uint32_t)(kro(4 * g + e) + col);
      ko.gr[e] = gka + 4u * (uint32_t)(kro(4 * g + e) + col - 4 * g - e + 15);
    }
    ko.mk = (uint32_t)(4 * g * Gm::KBW + 16 * w + col);
  }
  const uint32_t ring0 = ldsa(ring);
  // the lane's K / V rows have landed (with the first stage): passed through asm, so hipcc no
  // longer tracks their loads -- it waited vmcnt(0) before their first MFMA in every tile loop,
  // which also drained the next stage's LDS-DMA
  wait_vmcnt<0>();
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) { keep(kf[ks]); keep(vf[ks]); }
  f32x4 dkt[DK / 16], dvt[DK / 16];
#pragma unroll
  for (int t = 0; t < DK / 16; ++t) { dkt[t] = zero4(); dvt[t] = zero4(); }

  for (int qb = 0; qb < nq; ++qb) {
    const int i0 = qb * QBK;
    char* st = ring + (qb & 1) * Gm::STAGE_BYTES;
    float* ss = sst + (qb & 1) * 3 * QBK;
    wait_vmcnt<0>();
    if (w == 0) {  // this block's statistics into its slot (the other slot may still be read)
      const float m2 = st_m <= -1e38f ? -1e38f : st_m * 1.4426950408889634f;
      const uint32_t sa = ldsa(ss + lane);
      const float lv = i0 + lane < T ? st_l : 0.f;  // queries past T: P = 0
      asm volatile("ds_write_b32 %0, %1" ::"v"(sa), "v"(m2) : "memory");
      asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(sa), "v"(lv), "i"(4 * QBK) : "memory");
      asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(sa), "v"(st_d), "i"(8 * QBK) : "memory");
    }
    lds_barrier();
    if (qb + 1 < nq) {
      issue_stage_kv<DK, NW, RP, RM>(a, b, h, i0 + QBK, j0, ring + ((qb + 1) & 1) * Gm::STAGE_BYTES, tid);
      if (w == 0) load_stats(i0 + QBK);
    }
    const uint32_t sb = ring0 + (uint32_t)((qb & 1) * Gm::STAGE_BYTES);
    const uint32_t ssa = ldsa(ss) + 16u * (uint32_t)g;  // the lane's 4 query rows' statistics (+16r floats)
    uint32_t bq[KS], bq1[KS], bw[RP ? KS : 1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bq[ks] = sb + ko.rq[ks];
      if constexpr (RP) {
        bq1[ks] = sb + ko.rq1[ks];
        bw[ks] = sb + ko.w[ks];
      }
    }
    const uint32_t mrow = sb + Gm::M0 * 16u + ko.mk;
    uint32_t tb[DK / 16];  // the transposed fragments' per-lane bases in this stage
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) tb[t] = sb + ko.tr[t];
#pragma unroll
    for (int rs = 0; rs < 2; ++rs) {  // query tile pairs (2rs, 2rs + 1)
      f32x4 p2[2], ds2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = 2 * rs + u;  // queries i0 + 16r ..; lane rows 4g + e
        // every LDS read of the tile up front: S = Qu . K^T and dP = dO . V^T (query rows as the A
        // operand), the rows' statistics and mask bytes, then the window products' fragments;
        // addresses are the hoisted per-lane bases plus immediates (rows +16 keep the swizzle)
        const uint32_t rofs = (uint32_t)(r * 16 * DK * 2);  // (immediates after unrolling: no address adds)
        v4i aq[KS], ao[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(aq[ks]) : "v"(bq[ks]), "i"(rofs));
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ao[ks]) : "v"(bq[ks]), "i"(Gm::O0 * 16 + rofs));
        }
        v4i smv, slv, sdv;  // m, 1/sum, D of the lane's 4 query rows
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(smv) : "v"(ssa), "i"(64 * r));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(slv) : "v"(ssa), "i"(64 * r + 4 * QBK));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(sdv) : "v"(ssa), "i"(64 * r + 8 * QBK));
        uint32_t mb[4] = {0u, 0u, 0u, 0u};
        if constexpr (RM) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(mb[e]) : "v"(mrow), "i"(16 * r * Gm::KBW + e * Gm::KBW));
        }
        // window rows of this (query tile, key tile): m0 = jw - (i0 + 16r + 15) + T - 1 at image
        // row 16w - 16r + 48; G1 uses qv rows i, G2 rows i + 1
        v4i av[RP ? KS : 1], av1[RP ? KS : 1], bwf[RP ? 2 : 1][RP ? KS : 1];
        if constexpr (RP) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            // (window rows 16w - 16r + 48 (+16): r <= 3 keeps the immediates non-negative)
            static_assert(QBK - 16 - 16 * 3 >= 0, "window immediates");
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(av[ks]) : "v"(bq[ks]), "i"(Gm::QV0 * 16 + rofs));
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(av1[ks]) : "v"(bq1[ks]), "i"(rofs));
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bwf[0][ks]) : "v"(bw[ks]), "i"((QBK - 16 - 16 * r) * DK * 2));
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bwf[1][ks]) : "v"(bw[ks]), "i"((QBK - 16 * r) * DK * 2));
          }
          lgkm<4 * KS>();  // all but the window fragments
        } else {
          lgkm0();
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) { keep(aq[ks]); keep(ao[ks]); }
        keep(smv); keep(slv); keep(sdv);
#pragma unroll
        for (int e = 0; e < 4; ++e) keep(mb[e]);
        const f32x4 sm = __builtin_bit_cast(f32x4, smv), sl = __builtin_bit_cast(f32x4, slv),
                    sd = __builtin_bit_cast(f32x4, sdv);
        bool anym = kany;
        if constexpr (RM) {
          // the tile's 16 queries x the wave's 16 keys all masked, for rows that each have an
          // unmasked key elsewhere: P = dS = 0 exactly (the streaming chunk mask's future chunks)
          const bool any_zero = mb[0] == 0u || mb[1] == 0u || mb[2] == 0u || mb[3] == 0u;
          const bool dead_row = sm[0] <= -1e38f || sm[1] <= -1e38f || sm[2] <= -1e38f || sm[3] <= -1e38f;
          if (__builtin_amdgcn_ballot_w64(any_zero || dead_row) == 0) {
            lgkm0();  // the window reads issued above land before their registers are reused
            if constexpr (RP)
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) { keep(av[ks]); keep(av1[ks]); keep(bwf[0][ks]); keep(bwf[1][ks]); }
            p2[u] = zero4();
            ds2[u] = zero4();
            continue;
          }
          anym = __builtin_amdgcn_ballot_w64((mb[0] | mb[1] | mb[2] | mb[3]) != 0u) != 0;
        }
        f32x4 sc = mfma(as_frag(aq[0]), kf[0], zero4()), dp = mfma(as_frag(ao[0]), vf[0], zero4());
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) {
          sc = mfma(as_frag(aq[ks]), kf[ks], sc);
          dp = mfma(as_frag(ao[ks]), vf[ks], dp);
        }
        float bd[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (RP && !(LASR_ATTN_EXP & 2)) {
          const int mlo = jw - (i0 + 16 * r + 15) + T - 1;
          lgkm0();
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) { keep(av[ks]); keep(av1[ks]); keep(bwf[0][ks]); keep(bwf[1][ks]); }
#pragma unroll
          for (int uu = 0; uu < 2; ++uu) {
            const int lo = mlo + 16 * uu;
            // lane (g, col) holds G[query 4g + e][m = lo + col]: rows m <= T from qv_i (G1), m >= T
            // from qv_{i+1} (G2; the window's row m = T is zero), the tile across m = T both, selected
            // per column; parked as [query][m] (row 4g + e at kro(4g + e))
            f32x4 gs;
            if (lo + 15 <= T) {
              gs = mfma(as_frag(av[0]), as_frag(bwf[uu][0]), zero4());
#pragma unroll
              for (int ks = 1; ks < KS; ++ks) gs = mfma(as_frag(av[ks]), as_frag(bwf[uu][ks]), gs);
            } else if (lo >= T) {
              gs = mfma(as_frag(av1[0]), as_frag(bwf[uu][0]), zero4());
#pragma unroll
              for (int ks = 1; ks < KS; ++ks) gs = mfma(as_frag(av1[ks]), as_frag(bwf[uu][ks]), gs);
            } else {
              f32x4 g1 = mfma(as_frag(av[0]), as_frag(bwf[uu][0]), zero4());
              f32x4 g2 = mfma(as_frag(av1[0]), as_frag(bwf[uu][0]), zero4());
#pragma unroll
              for (int ks = 1; ks < KS; ++ks) {
                g1 = mfma(as_frag(av[ks]), as_frag(bwf[uu][ks]), g1);
                g2 = mfma(as_frag(av1[ks]), as_frag(bwf[uu][ks]), g2);
              }
              gs = lo + col <= T - 1 ? g1 : g2;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
              asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(ko.gw[e]), "v"(gs[e]), "i"(64 * uu) : "memory");
          }
          // bd(query 4g + e, key col) = G[4g + e][m - mlo = col - 4g - e + 15] (the wave's writes
          // above retire first)
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) asm volatile("ds_read_b32 %0, %1" : "=v"(v[e]) : "v"(ko.gr[e]));
          lgkm0();
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            keep(v[e]);
            bd[e] = v[e];
          }
        }
        // packed fp32 pairs (the same roundings per element); masking only where the wave's
        // tile has a masked score (uniform)
        const lasr_f2 c2v = {c2, c2};
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          lasr_f2 x = {sc[e], sc[e + 1]};
          x = (x + (lasr_f2){bd[e], bd[e + 1]}) * c2v;
          if (anym) {
            if (RM ? mb[e] != 0u : kmasked) x[0] = -1e38f;
            if (RM ? mb[e + 1] != 0u : kmasked) x[1] = -1e38f;
          }
          lasr_f2 pv = x - (lasr_f2){sm[e], sm[e + 1]};
          pv[0] = __builtin_amdgcn_exp2f(pv[0]);
          pv[1] = __builtin_amdgcn_exp2f(pv[1]);
          pv *= (lasr_f2){sl[e], sl[e + 1]};
          const lasr_f2 dsv = pv * ((lasr_f2){dp[e], dp[e + 1]} - (lasr_f2){sd[e], sd[e + 1]});
          p2[u][e] = pv[0];
          p2[u][e + 1] = pv[1];
          ds2[u][e] = dsv[0];
          ds2[u][e + 1] = dsv[1];
          if (anym) {
            if (!(x[0] > -1e38f)) ds2[u][e] = 0.f;
            if (!(x[1] > -1e38f)) ds2[u][e + 1] = 0.f;
          }
        }
      }
      // dV^T += dO^T P, dK^T += Qu^T dS (queries of the pair as k: 32rs + 4g + e, then + 16)
      const bf16x8 pb = pack8(p2[0], p2[1]), sbf = pack8(ds2[0], ds2[1]);
      v2i olo[DK / 16], ohi[DK / 16], qlo[DK / 16], qhi[DK / 16];
      const uint32_t pofs = (uint32_t)(32 * rs * DK * 2);
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(olo[t]) : "v"(tb[t]), "i"(Gm::O0 * 16 + pofs));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(ohi[t]) : "v"(tb[t]), "i"(Gm::O0 * 16 + pofs + 16 * DK * 2));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(qlo[t]) : "v"(tb[t]), "i"(pofs));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(qhi[t]) : "v"(tb[t]), "i"(pofs + 16 * DK * 2));
      }
      lgkm0();
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) { keep(olo[t]); keep(ohi[t]); keep(qlo[t]); keep(qhi[t]); }
#pragma unroll
      for (int t = 0; t < DK / 16; ++t) {
        dvt[t] = mfma(as_frag(olo[t], ohi[t]), pb, dvt[t]);
        dkt[t] = mfma(as_frag(qlo[t], qhi[t]), sbf, dkt[t]);
      }
    }
  }
  if (jq < Tk) {
    bf16_t* pk = dk_out + ((int64_t)b * Tk + jq) * lddkv + h * DK + 4 * g;
    bf16_t* pv = dv_out + ((int64_t)b * Tk + jq) * lddkv + h * DK + 4 * g;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
      *(uint2*)(pk + 16 * t) = make_uint2(pk_bf16(dkt[t][0] * a.scale, dkt[t][1] * a.scale),
                                          pk_bf16(dkt[t][2] * a.scale, dkt[t][3] * a.scale));
      *(uint2*)(pv + 16 * t) = make_uint2(pk_bf16(dvt[t][0], dvt[t][1]), pk_bf16(dvt[t][2], dvt[t][3]));
    }
  }
}

template <int DK, int NW, bool RP, bool RM>
void launch_bwd_kv_t(const FlashP& a, bf16_t* dk, bf16_t* dv, int64_t lddkv, hipStream_t st) {
  const dim3 grid((unsigned)cdiv(a.Tk, 16 * NW), (unsigned)a.H, (unsigned)a.B);
  flash_bwd_kv_kernel<DK, NW, RP, RM><<<grid, NW * 64, 0, st>>>(a, dk, dv, lddkv);
}

void launch_flash_bwd_kv(const FlashP& a, int dk, bool rp, bool rm, bf16_t* dko, bf16_t* dvo, int64_t ld,
                         hipStream_t st) {
  if (rp) {
    if (dk == 64) rm ? launch_bwd_kv_t<64, 8, true, true>(a, dko, dvo, ld, st) : launch_bwd_kv_t<64, 8, true, false>(a, dko, dvo, ld, st);
    else rm ? launch_bwd_kv_t<32, 4, true, true>(a, dko, dvo, ld, st) : launch_bwd_kv_t<32, 4, true, false>(a, dko, dvo, ld, st);
    return;
  }
  if (dk == 64) rm ? launch_bwd_kv_t<64, 4, false, true>(a, dko, dvo, ld, st) : launch_bwd_kv_t<64, 4, false, false>(a, dko, dvo, ld, st);
  else rm ? launch_bwd_kv_t<32, 4, false, true>(a, dko, dvo, ld, st) : launch_bwd_kv_t<32, 4, false, false>(a, dko, dvo, ld, st);
}

template <int DK, int NW, bool RP, bool RM>
void launch_fwd_t(const FlashP& a, hipStream_t st) {
  const dim3 grid((unsigned)(cdiv(a.T, 16 * NW) * (RP || a.nsplit < 1 ? 1 : a.nsplit)), (unsigned)a.H, (unsigned)a.B);
  flash_fwd_kernel<DK, NW, RP, RM><<<grid, NW * 64, 0, st>>>(a);
}

// The key-split combines (plain attention, nsplit > 1), one thread per (row, 4 columns), the
// splits in order.  Forward: M = max_s m_s, L = sum_s l_s 2^(m_s - M), O = sum_s 2^(m_s - M) O_s,
// ctx = O / L and the statistics the backward reads (as the one-pass epilogue writes them).
template <int DK>
__global__ __launch_bounds__(256) void flash_fwd_combine_kernel(FlashP a) {
  const int64_t BHT = (int64_t)a.B * a.H * a.T;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= BHT * (DK / 4)) return;
  const int64_t row = e / (DK / 4);
  const int cg = (int)(e - row * (DK / 4));
  const int iq = (int)(row % a.T), h = (int)((row / a.T) % a.H), b = (int)(row / ((int64_t)a.T * a.H));
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.mpart[2 * (s * BHT + row)]);
  float L = 0.f;
  f32x4 O = zero4();
  for (int s = 0; s < a.nsplit; ++s) {
    const float2 ml = *(const float2*)(a.mpart + 2 * (s * BHT + row));
    const float wgt = __builtin_amdgcn_exp2f(ml.x - M);
    L += ml.y * wgt;
    O += *(const f32x4*)(a.opart + (s * BHT + row) * DK + 4 * cg) * wgt;
  }
  const float il = 1.f / L;
  bf16_t* dst = a.ctx + ((int64_t)b * a.T + iq) * a.ldc + h * DK + 4 * cg;
  *(uint2*)dst = make_uint2(pk_bf16(O[0] * il, O[1] * il), pk_bf16(O[2] * il, O[3] * il));
  if (cg == 0) *(float2*)(a.stats + 2 * row) = make_float2(M <= -1e38f ? -1e38f : M * 0.6931471805599453f, il);
}
// Backward: dQ = scale * sum_s dQ_s.
template <int DK>
__global__ __launch_bounds__(256) void flash_dq_combine_kernel(FlashP a) {
  const int64_t BHT = (int64_t)a.B * a.H * a.T;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= BHT * (DK / 4)) return;
  const int64_t row = e / (DK / 4);
  const int cg = (int)(e - row * (DK / 4));
  const int iq = (int)(row % a.T), h = (int)((row / a.T) % a.H), b = (int)(row / ((int64_t)a.T * a.H));
  f32x4 q = zero4();
  for (int s = 0; s < a.nsplit; ++s) q += *(const f32x4*)(a.opart + (s * BHT + row) * DK + 4 * cg);
  bf16_t* dst = a.dqu + ((int64_t)b * a.T + iq) * a.ldq + h * DK + 4 * cg;
  *(uint2*)dst = make_uint2(pk_bf16(q[0] * a.scale, q[1] * a.scale), pk_bf16(q[2] * a.scale, q[3] * a.scale));
}

unsigned combine_blocks(const FlashP& a, int dk) { return (unsigned)cdiv((int64_t)a.B * a.H * a.T * (dk / 4), 256); }

// RP: the encoder's relative-position attention (8 waves, 128 queries per workgroup; 4 waves at d_k 32); plain:
// the decoder's (4 waves, 64 queries: Tq = L + 1 is short)
void launch_flash_fwd(const FlashP& a, int dk, bool rp, bool rm, hipStream_t st) {
  if (rp) {
    // d_k 32: 4-wave workgroups (62 KB of LDS: two per CU, whose block loops and prologues
    // interleave; 47 -> 43.6 us at config 4's shape, profiles/r04/attn_nw.jsonl); d_k 64 keeps 8
    // waves (its 4-wave workgroup needs 95 KB: one per CU, 15 -> 25 us at config 2's)
    if (dk == 64) rm ? launch_fwd_t<64, 8, true, true>(a, st) : launch_fwd_t<64, 8, true, false>(a, st);
    else rm ? launch_fwd_t<32, 4, true, true>(a, st) : launch_fwd_t<32, 4, true, false>(a, st);
    return;
  }
  if (dk == 64) rm ? launch_fwd_t<64, 4, false, true>(a, st) : launch_fwd_t<64, 4, false, false>(a, st);
  else rm ? launch_fwd_t<32, 4, false, true>(a, st) : launch_fwd_t<32, 4, false, false>(a, st);
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// query-dependent masks are staged by LDS-DMA: 16-B aligned rows
int check_mask(const uint8_t* mask, int64_t msb, int64_t msq, int Tk, const char* who) {
  if (mask && msq != 0)
    LASR_CHECK_ARG(al16(mask) && msq % 16 == 0 && msb % 16 == 0 && msq >= Tk,
                   "%s: a query-dependent mask needs 16-B aligned rows (row stride %% 16 == 0, >= Tk)", who);
  else
    LASR_CHECK_ARG(Tk <= KMASK_BYTES, "%s: Tk=%d above %d keys", who, Tk, KMASK_BYTES);
  return LASR_OK;
}

}  // namespace

extern "C" int lasr_relattn_fwd(const void* qu, const void* qv, int64_t ldq, const void* k,
                                const void* v, int64_t ldkv, const void* pos, int64_t ldp, int B,
                                int H, int T, int dk, const uint8_t* mask, int64_t mask_sb,
                                int64_t mask_sq, float scale, float* stats, void* ctx, int64_t ldc,
                                void* stream) {
  LASR_CHECK_ARG(dk == 64 || dk == 32, "lasr_relattn_fwd: d_k=%d (32 or 64)", dk);
  LASR_CHECK_ARG(B >= 0 && H > 0 && T >= 0 && B <= 65535 && H <= 65535, "lasr_relattn_fwd: bad B/H/T");
  LASR_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldp % 8 == 0 && ldc % 8 == 0 && ldc >= H * dk,
                 "lasr_relattn_fwd: row strides must be multiples of 8");
  LASR_CHECK_ARG(al16(qu) && al16(qv) && al16(k) && al16(v) && al16(pos) && al16(ctx), "lasr_relattn_fwd: 16-B alignment");
  if (B == 0 || T == 0) return LASR_OK;
  if (int rc = check_mask(mask, mask_sb, mask_sq, T, "lasr_relattn_fwd")) return rc;
  FlashP a = {};
  a.qu = (const bf16_t*)qu; a.qv = (const bf16_t*)qv; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.pos = (const bf16_t*)pos;
  a.ldq = ldq; a.ldkv = ldkv; a.ldp = ldp;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = T; a.Tk = T; a.scale = scale;
  a.stats = stats; a.ctx = (bf16_t*)ctx; a.ldc = ldc;
  launch_flash_fwd(a, dk, true, mask && mask_sq != 0, (hipStream_t)stream);
  return lasr_check_launch("relattn_fwd");
}

// lasr_relattn_fwd with lasr_qbias_fwd folded in: q [B*T, ldqin] (the q slot of the fused
// projection) and pos_bias_u / v [H*d_k] fp32 in; qu = q + u and qv = q + v are formed in the
// kernel (the same fp32 sum and bf16 rounding as lasr_qbias_fwd) and written to qu / qv [B*T,
// ldq] for the backward -- one launch and one re-read of q fewer per layer.
extern "C" int lasr_relattn_fwd_qb(const void* q, int64_t ldqin, const float* bu, const float* bv, void* qu,
                                   void* qv, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                                   const void* pos, int64_t ldp, int B, int H, int T, int dk, const uint8_t* mask,
                                   int64_t mask_sb, int64_t mask_sq, float scale, float* stats, void* ctx,
                                   int64_t ldc, void* stream) {
  LASR_CHECK_ARG(dk == 64 || dk == 32, "lasr_relattn_fwd_qb: d_k=%d (32 or 64)", dk);
  LASR_CHECK_ARG(B >= 0 && H > 0 && T >= 0 && B <= 65535 && H <= 65535, "lasr_relattn_fwd_qb: bad B/H/T");
  LASR_CHECK_ARG(ldqin % 8 == 0 && ldq % 8 == 0 && ldkv % 8 == 0 && ldp % 8 == 0 && ldc % 8 == 0 && ldc >= H * dk &&
                     ldq >= H * dk && ldqin >= H * dk,
                 "lasr_relattn_fwd_qb: row strides must be multiples of 8");
  LASR_CHECK_ARG(al16(q) && al16(qu) && al16(qv) && al16(k) && al16(v) && al16(pos) && al16(ctx) && al16(bu) &&
                     al16(bv),
                 "lasr_relattn_fwd_qb: 16-B alignment");
  if (B == 0 || T == 0) return LASR_OK;
  if (int rc = check_mask(mask, mask_sb, mask_sq, T, "lasr_relattn_fwd_qb")) return rc;
  FlashP a = {};
  a.qu = (const bf16_t*)qu; a.qv = (const bf16_t*)qv; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.pos = (const bf16_t*)pos;
  a.ldq = ldq; a.ldkv = ldkv; a.ldp = ldp;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = T; a.Tk = T; a.scale = scale;
  a.stats = stats; a.ctx = (bf16_t*)ctx; a.ldc = ldc;
  a.qin = (const bf16_t*)q; a.ldqin = ldqin; a.bu = bu; a.bv = bv;
  launch_flash_fwd(a, dk, true, mask && mask_sq != 0, (hipStream_t)stream);
  return lasr_check_launch("relattn_fwd_qb");
}

// Plain scaled dot-product attention (no positional term) with Tk keys per utterance: the
// decoder's self attention (Tk = Tq, causal + padding mask) and source attention over the
// encoder output (Tk = T', key padding).  nsplit > 1 splits the key blocks over that many
// workgroups per query block (work: lasr_attn_split_work floats), combined in a second launch.
static int attn_fwd_impl(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                         int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                         float* stats, void* ctx, int64_t ldc, int nsplit, float* work, int64_t work_floats,
                         void* stream) {
  LASR_CHECK_ARG(dk == 64 || dk == 32, "lasr_attn_fwd: d_k=%d (32 or 64)", dk);
  LASR_CHECK_ARG(B >= 0 && H > 0 && Tq >= 0 && Tk > 0 && B <= 65535 && H <= 65535, "lasr_attn_fwd: bad B/H/T");
  LASR_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldc % 8 == 0 && ldc >= H * dk,
                 "lasr_attn_fwd: row strides must be multiples of 8");
  LASR_CHECK_ARG(al16(q) && al16(k) && al16(v) && al16(ctx), "lasr_attn_fwd: 16-B alignment");
  if (B == 0 || Tq == 0) return LASR_OK;
  if (int rc = check_mask(mask, mask_sb, mask_sq, Tk, "lasr_attn_fwd")) return rc;
  const int nb = (Tk + KB - 1) / KB;
  LASR_CHECK_ARG(nsplit >= 1 && nsplit <= nb, "lasr_attn_fwd: nsplit=%d outside [1, %d key blocks]", nsplit, nb);
  if (nsplit > 1)
    LASR_CHECK_ARG(work && al16(work) && work_floats >= lasr_attn_split_work(B, H, Tq, dk, nsplit) &&
                   ((uintptr_t)stats & 7) == 0, "lasr_attn_fwd: split workspace");
  FlashP a = {};
  a.qu = a.qv = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.ldq = ldq; a.ldkv = ldkv;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = Tq; a.Tk = Tk; a.scale = scale;
  a.stats = stats; a.ctx = (bf16_t*)ctx; a.ldc = ldc;
  a.nsplit = nsplit;
  if (nsplit > 1) {
    a.opart = work;
    a.mpart = work + (int64_t)nsplit * B * H * Tq * dk;
  }
  launch_flash_fwd(a, dk, false, mask && mask_sq != 0, (hipStream_t)stream);
  if (int rc = lasr_check_launch("attn_fwd")) return rc;
  if (nsplit > 1) {
    if (dk == 64) flash_fwd_combine_kernel<64><<<combine_blocks(a, dk), 256, 0, (hipStream_t)stream>>>(a);
    else flash_fwd_combine_kernel<32><<<combine_blocks(a, dk), 256, 0, (hipStream_t)stream>>>(a);
    return lasr_check_launch("attn_fwd_combine");
  }
  return LASR_OK;
}

extern "C" int64_t lasr_attn_split_work(int B, int H, int Tq, int dk, int nsplit) {
  return nsplit > 1 ? (int64_t)nsplit * B * H * Tq * (dk + 2) : 0;
}

// Key blocks per workgroup >= 4 and about 512 workgroups: only long key runs over few query
// blocks split (the decoder's source attention at T' 999: 96 query blocks x 16 key blocks -> 4)
extern "C" int lasr_attn_split_count(int B, int H, int Tq, int Tk) {
  if (B <= 0 || H <= 0 || Tq <= 0 || Tk <= 0) return 1;
  const int64_t qblocks = cdiv(Tq, 64) * (int64_t)B * H;
  const int nb = (Tk + KB - 1) / KB;
  int ns = 1;
  while (ns * 2 <= nb / 4 && qblocks * ns * 2 <= 512) ns *= 2;
  return ns;
}

extern "C" int lasr_attn_fwd(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B,
                             int H, int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb,
                             int64_t mask_sq, float scale, float* stats, void* ctx, int64_t ldc, void* stream) {
  return attn_fwd_impl(q, ldq, k, v, ldkv, B, H, Tq, Tk, dk, mask, mask_sb, mask_sq, scale, stats, ctx, ldc, 1,
                       nullptr, 0, stream);
}

extern "C" int lasr_attn_fwd_split(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B,
                                   int H, int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb,
                                   int64_t mask_sq, float scale, float* stats, void* ctx, int64_t ldc, int nsplit,
                                   float* work, int64_t work_floats, void* stream) {
  return attn_fwd_impl(q, ldq, k, v, ldkv, B, H, Tq, Tk, dk, mask, mask_sb, mask_sq, scale, stats, ctx, ldc,
                       nsplit, work, work_floats, stream);
}

extern "C" int lasr_relattn_bwd(const void* qu, const void* qv, int64_t ldq, const void* k,
                                const void* v, int64_t ldkv, const void* pos, int64_t ldp, int B,
                                int H, int T, int dk, const uint8_t* mask, int64_t mask_sb,
                                int64_t mask_sq, float scale, const float* stats, const void* ctx,
                                const void* dctx, int64_t ldc, float* Dbuf, void* dqu, void* dbd,
                                int ldS, int dbd_head_major, void* dk_out, void* dv_out, int64_t lddkv,
                                void* stream) {
  LASR_CHECK_ARG(dk == 64 || dk == 32, "lasr_relattn_bwd: d_k=%d (32 or 64)", dk);
  LASR_CHECK_ARG(B >= 0 && H > 0 && T >= 0 && B <= 65535 && H <= 65535, "lasr_relattn_bwd: bad B/H/T");
  LASR_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldp % 8 == 0 && ldc % 8 == 0 && ldc >= H * dk,
                 "lasr_relattn_bwd: row strides must be multiples of 8");
  LASR_CHECK_ARG(ldS >= T && ldS % 2 == 0 && ((uintptr_t)dbd & 3) == 0,
                 "lasr_relattn_bwd: dBD rows need ldS >= T, ldS even and a 4-B aligned base");
  LASR_CHECK_ARG(al16(qu) && al16(qv) && al16(k) && al16(v) && al16(pos) && al16(dctx) && al16(ctx) && al16(dqu),
                 "lasr_relattn_bwd: 16-B alignment");
  if (B == 0 || T == 0) return LASR_OK;
  if (int rc = check_mask(mask, mask_sb, mask_sq, T, "lasr_relattn_bwd")) return rc;
  FlashP a = {};
  a.qu = (const bf16_t*)qu; a.qv = (const bf16_t*)qv; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.pos = (const bf16_t*)pos;
  a.ldq = ldq; a.ldkv = ldkv; a.ldp = ldp;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = T; a.Tk = T; a.scale = scale;
  a.stats = (float*)stats; a.ldc = ldc;
  a.dctx = (const bf16_t*)dctx; a.ctx_in = (const bf16_t*)ctx; a.Dbuf = Dbuf;
  a.dqu = (bf16_t*)dqu; a.dbd = (bf16_t*)dbd; a.ldS = ldS; a.dbd_hb = dbd_head_major;
  LASR_CHECK_ARG(lddkv % 8 == 0 && al16(dk_out) && al16(dv_out), "lasr_relattn_bwd: dk/dv rows 16-B aligned");
  const bool rm = mask && mask_sq != 0;
  launch_flash_bwd_q(a, dk, true, rm, (hipStream_t)stream);
  if (int rc = lasr_check_launch("relattn_bwd_q")) return rc;
  launch_flash_bwd_kv(a, dk, true, rm, (bf16_t*)dk_out, (bf16_t*)dv_out, lddkv, (hipStream_t)stream);
  return lasr_check_launch("relattn_bwd_kv");
}

static int attn_bwd_impl(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B, int H,
                         int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb, int64_t mask_sq, float scale,
                         const float* stats, const void* ctx, const void* dctx, int64_t ldc, float* Dbuf, void* dq,
                         void* dk_out, void* dv_out, int64_t lddkv, int nsplit, float* work, int64_t work_floats,
                         void* stream) {
  LASR_CHECK_ARG(dk == 64 || dk == 32, "lasr_attn_bwd: d_k=%d (32 or 64)", dk);
  LASR_CHECK_ARG(B >= 0 && H > 0 && Tq >= 0 && Tk > 0 && B <= 65535 && H <= 65535, "lasr_attn_bwd: bad B/H/T");
  LASR_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldc % 8 == 0 && ldc >= H * dk && lddkv % 8 == 0,
                 "lasr_attn_bwd: row strides must be multiples of 8");
  LASR_CHECK_ARG(al16(q) && al16(k) && al16(v) && al16(dctx) && al16(ctx) && al16(dq), "lasr_attn_bwd: 16-B alignment");
  if (B == 0 || Tq == 0) return LASR_OK;
  if (int rc = check_mask(mask, mask_sb, mask_sq, Tk, "lasr_attn_bwd")) return rc;
  const int nb = (Tk + KB - 1) / KB;
  LASR_CHECK_ARG(nsplit >= 1 && nsplit <= nb, "lasr_attn_bwd: nsplit=%d outside [1, %d key blocks]", nsplit, nb);
  if (nsplit > 1)
    LASR_CHECK_ARG(work && al16(work) && work_floats >= lasr_attn_split_work(B, H, Tq, dk, nsplit),
                   "lasr_attn_bwd: split workspace");
  FlashP a = {};
  a.qu = a.qv = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v;
  a.ldq = ldq; a.ldkv = ldkv;
  a.mask = mask; a.msb = mask_sb; a.msq = mask_sq;
  a.B = B; a.H = H; a.T = Tq; a.Tk = Tk; a.scale = scale;
  a.stats = (float*)stats; a.ldc = ldc;
  a.dctx = (const bf16_t*)dctx; a.ctx_in = (const bf16_t*)ctx; a.Dbuf = Dbuf;
  a.dqu = (bf16_t*)dq;
  a.nsplit = nsplit;
  a.opart = nsplit > 1 ? work : nullptr;
  LASR_CHECK_ARG(al16(dk_out) && al16(dv_out), "lasr_attn_bwd: dk/dv 16-B alignment");
  const bool rm = mask && mask_sq != 0;
  launch_flash_bwd_q(a, dk, false, rm, (hipStream_t)stream);
  if (int rc = lasr_check_launch("attn_bwd_q")) return rc;
  if (nsplit > 1) {
    if (dk == 64) flash_dq_combine_kernel<64><<<combine_blocks(a, dk), 256, 0, (hipStream_t)stream>>>(a);
    else flash_dq_combine_kernel<32><<<combine_blocks(a, dk), 256, 0, (hipStream_t)stream>>>(a);
    if (int rc = lasr_check_launch("attn_dq_combine")) return rc;
  }
  launch_flash_bwd_kv(a, dk, false, rm, (bf16_t*)dk_out, (bf16_t*)dv_out, lddkv, (hipStream_t)stream);
  return lasr_check_launch("attn_bwd_kv");
}

extern "C" int lasr_attn_bwd(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B,
                             int H, int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb,
                             int64_t mask_sq, float scale, const float* stats, const void* ctx, const void* dctx,
                             int64_t ldc, float* Dbuf, void* dq, void* dk_out, void* dv_out, int64_t lddkv,
                             void* stream) {
  return attn_bwd_impl(q, ldq, k, v, ldkv, B, H, Tq, Tk, dk, mask, mask_sb, mask_sq, scale, stats, ctx, dctx, ldc,
                       Dbuf, dq, dk_out, dv_out, lddkv, 1, nullptr, 0, stream);
}

extern "C" int lasr_attn_bwd_split(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, int B,
                                   int H, int Tq, int Tk, int dk, const uint8_t* mask, int64_t mask_sb,
                                   int64_t mask_sq, float scale, const float* stats, const void* ctx,
                                   const void* dctx, int64_t ldc, float* Dbuf, void* dq, void* dk_out, void* dv_out,
                                   int64_t lddkv, int nsplit, float* work, int64_t work_floats, void* stream) {
  return attn_bwd_impl(q, ldq, k, v, ldkv, B, H, Tq, Tk, dk, mask, mask_sb, mask_sq, scale, stats, ctx, dctx, ldc,
                       Dbuf, dq, dk_out, dv_out, lddkv, nsplit, work, work_floats, stream);
}
