// Shared CDNA4 (gfx950) MFMA tile machinery: LDS images of bf16 operand tiles, their
// fragment reads for v_mfma_f32_16x16x32_bf16, the LDS-DMA (global_load_lds) tile issue
// and the counted-vmcnt ring waits.  Used by gemm.hip (the generic GEMM) and ffn.hip
// (the fused feed-forward chains).
#pragma once
#include "common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

LASR_DEV int swz(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }
LASR_DEV int lds_off(int row, int chunk) { return row * 32 + ((chunk ^ swz(row)) << 3); }

// 8 consecutive elements along the contiguous axis; zero outside [0,lim).
LASR_DEV uint4 load8(const bf16_t* src, int start, int lim, bool vec) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (vec && start + 8 <= lim) {
    v = *(const uint4*)src;
  } else {
    uint32_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = (start + j < lim) ? (uint32_t)src[j] : 0u;
    v.x = e[0] | (e[1] << 16);
    v.y = e[2] | (e[3] << 16);
    v.z = e[4] | (e[5] << 16);
    v.w = e[6] | (e[7] << 16);
  }
  return v;
}

// Tile loader for one operand: R_TILE rows (M or N) x 32 k, 16-B global loads.
//  KC (operand K-contiguous in HBM): image [R_TILE][32 k], 64-B rows, chunk swizzle above;
//     fragments read with ds_read_b128.
//  !KC (operand M/N-contiguous, e.g. dW = dY^T X, dX = dY W): image [32 k][R_TILE] stored as
//     it arrives (no transposing writes); 32-B column slots XOR-swizzled per k row by
//     htr(k) so the 8 k-rows a 32-lane half touches in one ds_read_b64_tr_b16 land on 8
//     distinct 32-B bank groups (conflict-free); fragments read with 2 transposed reads.
template <int R_TILE>
LASR_DEV int htr(int k) {
  return R_TILE >= 128 ? ((k & 3) | ((k >> 1) & 4)) : (((k >> 1) & 1) | ((k >> 2) & 2));
}
template <int R_TILE>
LASR_DEV int tr_off(int k, int col) {  // element offset of (k, col), col % 4 == 0
  return k * R_TILE + ((((col >> 4) ^ htr<R_TILE>(k))) << 4) + (col & 15);
}

template <int R_TILE, bool KC, int NT = 256>
struct TileLoader {
  static constexpr int UNITS = R_TILE * 4;  // 16-B units per 32-deep k tile
  static constexpr int PER = (UNITS + NT - 1) / NT;
  uint4 r0[PER];

  LASR_DEV void load(const bf16_t* base, int64_t ld_r, int64_t ld_k, int row0, int R, int k0,
                     int kend, bool vec, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = tid + i * NT;
      if (u < UNITS) {
        if (KC) {
          const int r = u >> 2, c = u & 3;
          const int gr = row0 + r, gk = k0 + c * 8;
          if (gr < R) r0[i] = load8(base + (int64_t)gr * ld_r + gk, gk, kend, vec);
          else r0[i] = make_uint4(0, 0, 0, 0);
        } else {
          const int c = u % (R_TILE / 8), k = u / (R_TILE / 8);
          const int gr = row0 + c * 8, gk = k0 + k;
          if (gk < kend) r0[i] = load8(base + (int64_t)gk * ld_k + gr, gr, R, vec);
          else r0[i] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  }
  LASR_DEV void store(bf16_t* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = tid + i * NT;
      if (u < UNITS) {
        if (KC) {
          const int r = u >> 2, c = u & 3;
          *(uint4*)(lds + lds_off(r, c)) = r0[i];
        } else {
          const int c = u % (R_TILE / 8), k = u / (R_TILE / 8);
          *(uint4*)(lds + tr_off<R_TILE>(k, c * 8)) = r0[i];
        }
      }
    }
  }
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// MFMA 16x16x32 operand fragment of rows rbase..rbase+15: lane l gets row rbase + (l&15),
// k = 8(l>>4) .. 8(l>>4)+7.  EXEC must be full for the transposed reads (no divergence).
template <int R_TILE, bool KC>
LASR_DEV bf16x8 frag(const bf16_t* tile, int rbase, int lane) {
  if (KC) return *(const bf16x8*)(tile + lds_off(rbase + (lane & 15), lane >> 4));
  const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + tr_off<R_TILE>(8 * g + q, rbase + pc)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + tr_off<R_TILE>(8 * g + 4 + q, rbase + pc)));
  const short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int N>
LASR_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt out of range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Retire ring tile kt when `after` (<= S-2) later tiles of GL glds each are still in flight.
template <int S, int GL>
LASR_DEV void wait_ring(int after) {
  if constexpr (S >= 6) if (after >= 4) { wait_vmcnt<4 * GL>(); return; }
  if constexpr (S >= 5) if (after >= 3) { wait_vmcnt<3 * GL>(); return; }
  if constexpr (S >= 4) if (after >= 2) { wait_vmcnt<2 * GL>(); return; }
  if (after >= 1) wait_vmcnt<GL>();
  else wait_vmcnt<0>();
}
LASR_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef int v2i __attribute__((ext_vector_type(2)));

// Transposed LDS read in inline asm: hipcc would otherwise treat the builtin as possibly
// aliasing the in-flight LDS-DMA and drain the ring (vmcnt(0)) before every k step.  asm
// loads are invisible to hipcc's waitcnt bookkeeping, so the caller waits explicitly
// (tie_lgkm) before the results are used.
LASR_DEV v2i ds_tr_asm(const bf16_t* p) {
  v2i r;
  const uint32_t a = (uint32_t)(uintptr_t)(lptr_t)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// s_waitcnt lgkmcnt(0) that the consumers of r[0..N) depend on (in/out operands).
template <int N>
LASR_DEV void tie_lgkm(v2i* r) {
  if constexpr (N == 4)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]));
  else if constexpr (N == 8)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]),
                 "+v"(r[5]), "+v"(r[6]), "+v"(r[7]));
  else if constexpr (N == 16)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]),
                 "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]),
                 "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]));
  else
    static_assert(N < 0, "tie_lgkm: unsupported count");
}
// Byte offsets (in the tile image) of the two halves frag_tr_raw reads for fragment rbase:
// loop invariant per thread, so a k step adds only the uniform tile base (frag_tr_raw_at).
template <int R_TILE>
LASR_DEV void frag_tr_offsets(int rbase, int lane, uint32_t* o) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
  o[0] = 2u * (uint32_t)tr_off<R_TILE>(8 * g + q, rbase + pc);
  o[1] = 2u * (uint32_t)tr_off<R_TILE>(8 * g + 4 + q, rbase + pc);
}
// uniform by construction (the ring slot of a k step): readfirstlane keeps it in an SGPR
LASR_DEV uint32_t lds_addr(const bf16_t* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lptr_t)p);
}
LASR_DEV void frag_tr_raw_at(uint32_t tile_base, const uint32_t* o, v2i* r) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[0]) : "v"(tile_base + o[0]));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[1]) : "v"(tile_base + o[1]));
}
// Raw halves of a transposed fragment (see frag<>): k = 8g+q and 8g+4+q rows.
template <int R_TILE>
LASR_DEV void frag_tr_raw(const bf16_t* tile, int rbase, int lane, v2i* r) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
  r[0] = ds_tr_asm(tile + tr_off<R_TILE>(8 * g + q, rbase + pc));
  r[1] = ds_tr_asm(tile + tr_off<R_TILE>(8 * g + 4 + q, rbase + pc));
}
typedef int v4i __attribute__((ext_vector_type(4)));
LASR_DEV v4i ds_b128_asm(const bf16_t* p) {
  v4i r;
  const uint32_t a = (uint32_t)(uintptr_t)(lptr_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// Row sums of an M-contiguous A tile image ([32 k][BM], tr_off layout): thread owns the 8
// rows 8*(tid % (BM/8)).. and k rows tid / (BM/8) + j * (NT / (BM/8)).
template <int BM, int NT = 256>
LASR_DEV void rowsum_tile(const bf16_t* tile, int tid, float* rs) {
  constexpr int CH = BM / 8, KG = NT / CH, KR = 32 / KG;
  static_assert(KR >= 1 && KR <= 4 && KR * KG == 32, "rowsum_tile geometry");
  const int c = tid % CH, k0 = tid / CH;
  v4i r[KR];
#pragma unroll
  for (int j = 0; j < KR; ++j) r[j] = ds_b128_asm(tile + tr_off<BM>(k0 + j * KG, 8 * c));
  if constexpr (KR == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]));
  else if constexpr (KR == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]));
  else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]));
#pragma unroll
  for (int j = 0; j < KR; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t u = (uint32_t)r[j][q];
      rs[2 * q] += __uint_as_float(u << 16);
      rs[2 * q + 1] += __uint_as_float(u & 0xffff0000u);
    }
}

// 8-B LDS write / read in inline asm: a plain LDS access after an in-flight LDS-DMA makes
// hipcc assume they may alias and drain the ring (vmcnt(0)); these are invisible to that
// bookkeeping, so the caller orders them (lgkmcnt waits / lds_barrier)
LASR_DEV void ds_w64_asm(bf16_t* p, v2i v) {
  const uint32_t a = (uint32_t)(uintptr_t)(lptr_t)p;
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
LASR_DEV v2i ds_r64_asm(const bf16_t* p) {
  v2i r;
  const uint32_t a = (uint32_t)(uintptr_t)(lptr_t)p;
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
LASR_DEV v2i pack4_bf16(const float* v) {
  v2i r;
  r[0] = (int)pk_bf16(v[0], v[1]);
  r[1] = (int)pk_bf16(v[2], v[3]);
  return r;
}

LASR_DEV bf16x8 frag_from_raw(const v2i* r) {
  const int __attribute__((ext_vector_type(4))) v = {r[0][0], r[0][1], r[1][0], r[1][1]};
  return __builtin_bit_cast(bf16x8, v);
}

// Issue the glds of one operand tile (R_TILE rows x 32 k) into `dst` (NT threads).
template <int R_TILE, bool KC, int NT = 256>
LASR_DEV void glds_tile(const bf16_t* base, int64_t ld, int row0, int R, int k0, bf16_t* dst,
                        int tid) {
  constexpr int PER = R_TILE * 4 / NT;  // 16-B positions per thread
  static_assert(PER >= 1 && PER * NT == R_TILE * 4, "glds_tile: tile / thread count");
  const int wid = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int P = i * NT + tid;  // linear 16-B position in the image
    const bf16_t* src;
    if (KC) {
      const int r = P >> 2, c = (P & 3) ^ swz(r);
      const int gr = min(row0 + r, R - 1);
      src = base + (int64_t)gr * ld + k0 + c * 8;
    } else {
      constexpr int CPR = R_TILE / 8;
      const int k = P / CPR, ps = P % CPR;
      const int ls = ((((ps >> 1) ^ htr<R_TILE>(k))) << 1) | (ps & 1);
      const int gc = min(row0 + ls * 8, ((R + 7) & ~7) - 8);  // host: row stride >= roundup8(R)
      // the k0 row offset is uniform (scalar multiply) and the thread's own part is loop
      // invariant (hoisted): (k0 + k) * ld as one vector product cost three quarter-rate
      // multiplies per load and k tile
      src = (base + (int64_t)k0 * ld) + ((int64_t)k * ld + gc);
    }
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (i * NT + wid * 64) * 8), 16, 0, 0);
    (void)lane;
  }
}
