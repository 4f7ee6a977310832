// Fused position-wise feed-forward chains (lasr_ffn_fwd / lasr_ffn_bwd_dx).
//
// Reference: PositionwiseFeedForward (liteasr/nets/feed_forward.py:18-19) inside the
// Conformer layer's half-step residual branches (liteasr/nets/conformer_layer.py:37-47,
// 58-66): out = res + res_scale * drop2(W2 drop1(act(W1 ln + b1)) + b2).
//
// One workgroup owns FB_M = 32 rows and walks the inner dimension F in chunks of 128: the
// [32 x 128] slice of the 2048-wide intermediate lives in registers / LDS only, and the
// second product accumulates straight into a [32 x D] register tile, so the intermediate
// never makes the HBM round trip between two GEMM launches.
//   forward:  z_c = ln W1_c^T + b1_c -> (store g_c = act'(z_c) * keep1, h_c =
//             drop1(act(z_c)) -> store h_c, LDS) -> acc += h_c W2_c^T ;
//             out = res + res_scale * drop2(acc + b2)
//   backward (input gradient): dh_c = gb W2_c -> dz_c = dh_c * g_c * scale1 -> store dz_c
//             (for dW1), LDS -> acc += dz_c W1_c ; dx = acc
// g / h / dz are written because the backward (g) and the weight gradients (split-K GEMMs
// over all rows: h, dz) need them; everything else stays on chip.  g is the GEMM
// epilogue's zout_mode-1 gate, so the backward needs no activation derivative and no
// dropout draw.  Dropout masks are the same pure function of
// (seed, step counter, element index) as the GEMM epilogues', and both products
// accumulate in the same k order as the two-launch path.
//
// Pipeline: the resident A tile (ln or gb, [32 x D] bf16, all of K) is copied once by
// LDS-DMA; the weights stream through an S-stage ring of equal-size slots (per chunk:
// 4 slots of the first product's B operand, 4 of the second's), S-1 slots in flight, one
// raw barrier per slot behind a counted vmcnt (tile.h).  The backward also streams the z
// chunk (its activation-gradient input) into a double buffer 7 slots ahead of its use.
// The issue pattern is periodic (past the end the ring re-issues its last tile into a free
// slot), so every wait count is a compile-time constant.  Weights stay in each XCD's L2
// (2 MB at D 256); the kernel is bound by that L2 -> CU stream (~2 MB per workgroup).
#include "common.h"
#include "tile.h"

namespace {

constexpr int FB_M = 32;   // rows per workgroup
constexpr int FB_CH = 128;  // inner-dimension chunk

struct FfnP {
  int M, F;
  const bf16_t* x;    // fwd: ln [M, D]; bwd: gb [M, D]
  const bf16_t* W1;   // [F, D]
  const float* b1;    // [F]
  const bf16_t* W2;   // [D, F]
  const float* b2;    // [D]
  DropCfg d1, d2;
  const float* res;
  float res_scale;
  bf16_t* z;          // fwd: out; bwd: in
  bf16_t* h;          // fwd: out
  float* out;         // fwd: [M, D]
  bf16_t* dz;         // bwd: out [M, F]
  bf16_t* dx;         // bwd: out [M, D]
};

// number of d in [1, S-1] with (J - d) = R (mod 8): how many of the iterations that issued
// after ring tile t (t = J mod 8) carry the extra vector-memory ops issued at position R
template <int S, int J, int R>
constexpr int nwin() {
  int n = 0;
  for (int d = 1; d <= S - 1; ++d)
    if ((((J - d) % 8) + 8) % 8 == R) ++n;
  return n;
}
constexpr int FB_MAXF = 2048;  // b1 staged in LDS

template <int D, int ACT, bool BWD, int S>
struct Chain {
  static constexpr int BM = FB_M, CH = FB_CH;
  static constexpr int KT = D / 32;             // k-tiles of the resident A tile
  static constexpr int SLOT = D * 32;           // bf16 elements per ring slot
  static constexpr int NI = D / 128;            // first-product images per slot (32 k each)
  static constexpr int KW = D / 4;              // k extent of a first-product slot
  static constexpr int GL = D / 64;             // glds per thread per slot
  static constexpr int NA = BM * CH / 8 / 256;  // glds per thread per aux chunk (2)
  static constexpr int FN2 = D / 64;            // second-product column frags per wave
  static constexpr int NS = BWD ? 4 : 8;        // epilogue-1 stores per thread (dz | z, h)
  static constexpr int A_EL = BM * D, H_EL = BM * CH, AUX_EL = BM * CH;
  static constexpr int LDS_BYTES = 2 * (A_EL + H_EL + (BWD ? 2 * AUX_EL : 0) + S * SLOT) + (BWD ? 0 : 4 * FB_MAXF);
  // vector-memory ops younger than ring tile t at the top of iteration t (J = t mod 8): the
  // S-2 ring tiles issued since, the aux chunk issued at position 4 (backward) and the
  // epilogue-1 stores issued at position 3 inside that window
  template <int J>
  static constexpr int younger() {
    return (S - 2) * GL + (BWD ? NA * nwin<S, J, 4>() : 0) + NS * nwin<S, J, 3>();
  }

  const FfnP& p;
  bf16_t *As, *Hs, *Aux, *Ring;
  float* B1s;
  int tid, lane, wid, m0, nch, total, c0;
  uint32_t key1, key2;
  f32x4 acc1[2][2];
  f32x4 acc2[2][FN2];

  LASR_DEV Chain(const FfnP& pp, bf16_t* smem) : p(pp) {
    As = smem;
    Hs = As + A_EL;
    Aux = Hs + H_EL;
    Ring = Aux + (BWD ? 2 * AUX_EL : 0);
    B1s = reinterpret_cast<float*>(Ring + S * SLOT);
    tid = threadIdx.x;
    lane = tid & 63;
    wid = tid >> 6;
    m0 = blockIdx.x * BM;
    nch = p.F / CH;
    total = nch * 8;
    // chunk rotation: the 32 workgroups an XCD hosts (blockIdx = xcd + 8 k) start at
    // different chunks, so they do not all pull the same weight tile from the same L2
    // channels at once; only the order of the second product's chunk sum changes
    c0 = (int)((blockIdx.x >> 3) % (unsigned)nch);
    key1 = p.d1.p > 0.f ? drop_key(p.d1) : 0u;
    key2 = (!BWD && p.d2.p > 0.f) ? drop_key(p.d2) : 0u;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j) acc2[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  LASR_DEV int chunk(int c) const { return c + c0 < nch ? c + c0 : c + c0 - nch; }

  LASR_DEV void glds(const bf16_t* src, bf16_t* wave_dst) {
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)wave_dst, 16, 0, 0);
  }

  // resident A tile: KT images [BM][32], 16-B chunk swizzle applied to the source
  LASR_DEV void issue_A() {
    constexpr int PER = A_EL / 8 / 256;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int P = i * 256 + tid;
      const int kt = P / (BM * 4), q = P % (BM * 4);
      const int r = q >> 2, cs = (q & 3) ^ swz(r);
      const int gr = min(m0 + r, p.M - 1);
      glds(p.x + (int64_t)gr * D + kt * 32 + cs * 8, As + (i * 256 + wid * 64) * 8);
    }
  }

  // z chunk c ([BM][CH], 16-B chunks XOR (row & 15)) into aux buffer c & 1
  LASR_DEV void issue_aux(int c) {
    bf16_t* dst = Aux + (c & 1) * AUX_EL;  // past the end: reload the last chunk, free buffer
    c = chunk(min(c, nch - 1));
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int P = i * 256 + tid;
      const int r = P / (CH / 8), cs = (P % (CH / 8)) ^ (r & 15);
      const int gr = min(m0 + r, p.M - 1);
      glds(p.z + (int64_t)gr * p.F + c * CH + cs * 8, dst + (i * 256 + wid * 64) * 8);
    }
  }

  LASR_DEV void issue_ring(int t) {
    bf16_t* dst = Ring + (t % S) * SLOT;
    t = min(t, total - 1);  // past the end: re-issue the last tile into the (free) slot
    const int c = chunk(t >> 3), j = t & 7;
    if (j < 4) {
#pragma unroll
      for (int ii = 0; ii < NI; ++ii) {
        const int k0 = j * KW + 32 * ii;
        if (!BWD) glds_tile<CH, true>(p.W1, D, c * CH, p.F, k0, dst + ii * CH * 32, tid);
        else glds_tile<CH, false>(p.W2, p.F, c * CH, p.F, k0, dst + ii * CH * 32, tid);
      }
    } else {
      const int k0 = c * CH + (j - 4) * 32;
      if (!BWD) glds_tile<D, true>(p.W2, p.F, 0, D, k0, dst, tid);
      else glds_tile<D, false>(p.W1, D, 0, D, k0, dst, tid);
    }
  }

  // first product, one ring slot (NI k-tiles of 32)
  LASR_DEV void gemm1(const bf16_t* slot, int j) {
#pragma unroll
    for (int ii = 0; ii < NI; ++ii) {
      const bf16_t* a_img = As + (j * NI + ii) * BM * 32;
      const bf16_t* b_img = slot + ii * CH * 32;
      bf16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag<BM, true>(a_img, i * 16, lane);
      if constexpr (!BWD) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) bf[jj] = frag<CH, true>(b_img, wid * 32 + jj * 16, lane);
      } else {
        v2i rb[4];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) frag_tr_raw<CH>(b_img, wid * 32 + jj * 16, lane, rb + 2 * jj);
        tie_lgkm<4>(rb);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) bf[jj] = frag_from_raw(rb + 2 * jj);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc1[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[jj], af[i], acc1[i][jj], 0, 0, 0);
    }
  }

  // second product, one ring slot (32 k of the chunk)
  LASR_DEV void gemm2(const bf16_t* slot, int jj) {
    const bf16_t* a_img = Hs + jj * BM * 32;
    bf16x8 af[2], bf[FN2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag<BM, true>(a_img, i * 16, lane);
    if constexpr (!BWD) {
#pragma unroll
      for (int j = 0; j < FN2; ++j) bf[j] = frag<D, true>(slot, wid * (D / 4) + j * 16, lane);
    } else {
      v2i rb[2 * FN2];
#pragma unroll
      for (int j = 0; j < FN2; ++j) frag_tr_raw<D>(slot, wid * (D / 4) + j * 16, lane, rb + 2 * j);
      tie_lgkm<2 * FN2>(rb);
#pragma unroll
      for (int j = 0; j < FN2; ++j) bf[j] = frag_from_raw(rb + 2 * j);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j)
        acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc2[i][j], 0, 0, 0);
  }

  // first product's epilogue: lane owns row 16i + (lane & 15), chunk columns
  // 32 wid + 16 jj + 4 (lane >> 4) .. +3 (= H image wid)
  LASR_DEV void epilogue1(int c) {
    const bf16_t* aux = Aux + (c & 1) * AUX_EL;
    bf16_t* himg = Hs + wid * BM * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = i * 16 + (lane & 15);
      // rows past M hold row M-1's operands (clamped loads) and compute its values exactly
      // (dropout indexed by the clamped row too), so every lane stores -- a duplicate write
      // of identical values -- and the store count per wave stays fixed for the vmcnt waits
      const int mc = min(m0 + r, p.M - 1);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int kc = wid * 32 + jj * 16 + 4 * (lane >> 4);  // column within the chunk
        const int f = chunk(c) * CH + kc;
        float v[4];
        if constexpr (!BWD) {
          // b1 from LDS through an asm read: a plain LDS load here makes hipcc assume it may
          // alias the in-flight LDS-DMA and drain the ring with vmcnt(0)
          v4i bb = ds_b128_asm(reinterpret_cast<const bf16_t*>(B1s + f));
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bb));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc1[i][jj][e] + __int_as_float(bb[e]);
          float keep[4] = {1.f, 1.f, 1.f, 1.f}, gate[4];
          if (p.d1.p > 0.f) drop_keep_n<4>(p.d1, key1, (uint64_t)mc * p.F + f, keep);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gate[e] = (ACT == LASR_ACT_RELU ? (v[e] > 0.f ? 1.f : 0.f) : swish_grad(v[e])) * keep[e];
            v[e] = (ACT == LASR_ACT_RELU ? fmaxf(v[e], 0.f) : swishf(v[e])) * keep[e] * (p.d1.p > 0.f ? p.d1.scale : 1.f);
          }
          stv<4>(p.z + (int64_t)mc * p.F + f, gate);  // act'(z) * keep, the backward's aux
        } else {
          // the gate act'(z) * keep streamed from the forward (swizzled [BM][CH] image)
          const int q = kc >> 3, half = (kc >> 2) & 1;
          v2i zr = ds_r64_asm(aux + r * CH + ((q ^ (r & 15)) << 3) + 4 * half);
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(zr));
          const float gt[4] = {__uint_as_float((uint32_t)zr[0] << 16), __uint_as_float((uint32_t)zr[0] & 0xffff0000u),
                               __uint_as_float((uint32_t)zr[1] << 16), __uint_as_float((uint32_t)zr[1] & 0xffff0000u)};
          const float sc = p.d1.p > 0.f ? p.d1.scale : 1.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc1[i][jj][e] * sc * gt[e];
        }
        stv<4>((BWD ? p.dz : p.h) + (int64_t)mc * p.F + f, v);
        const int kk = jj * 16 + 4 * (lane >> 4);
        ds_w64_asm(himg + lds_off(r, kk >> 3) + (kk & 7), pack4_bf16(v));  // ordered by the next lds_barrier
#pragma unroll
        for (int e = 0; e < 4; ++e) acc1[i][jj][e] = 0.f;
      }
    }
  }

  LASR_DEV void final_epilogue() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + i * 16 + (lane & 15);
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < FN2; ++j) {
        const int n = wid * (D / 4) + j * 16 + 4 * (lane >> 4);
        float v[4] = {acc2[i][j][0], acc2[i][j][1], acc2[i][j][2], acc2[i][j][3]};
        if constexpr (!BWD) {
          float t[4];
          ldv<4>(p.b2 + n, t);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += t[e];
          if (p.d2.p > 0.f) {
            float dm[4];
            drop_mul_n<4>(p.d2, key2, (uint64_t)m * D + n, dm);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= dm[e];
          }
          if (p.res) {
            ldv<4>(p.res + (int64_t)m * D + n, t);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = t[e] + p.res_scale * v[e];
          }
          stv<4>(p.out + (int64_t)m * D + n, v);
        } else {
          stv<4>(p.dx + (int64_t)m * D + n, v);
        }
      }
    }
  }

  template <int J>
  LASR_DEV void step(int c) {
    const int t = c * 8 + J;
    wait_vmcnt<younger<J>()>();
    lds_barrier();
    issue_ring(t + S - 1);
    if constexpr (BWD && J == 4) issue_aux(c + 1);
    const bf16_t* slot = Ring + (t % S) * SLOT;
    if constexpr (J < 4) {
      gemm1(slot, J);
      if constexpr (J == 3) epilogue1(c);
    } else {
      gemm2(slot, J - 4);
    }
  }

  LASR_DEV void run() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc1[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (!BWD)  // b1 staged in LDS before the ring starts (no global loads in the loop)
      for (int f = tid * 4; f < p.F; f += 1024) {
        float bb[4];
        ldv<4>(p.b1 + f, bb);
        stv<4>(B1s + f, bb);
      }
    issue_A();
    if constexpr (BWD && S <= 4) issue_aux(0);
#pragma unroll
    for (int u = -(S - 1); u < 0; ++u) {
      issue_ring(u + S - 1);
      if constexpr (BWD && S > 4)
        if (u == -4) issue_aux(0);
    }
    for (int c = 0; c < nch; ++c) {
      step<0>(c);
      step<1>(c);
      step<2>(c);
      step<3>(c);
      step<4>(c);
      step<5>(c);
      step<6>(c);
      step<7>(c);
    }
    wait_vmcnt<0>();  // the padded tail issues: nothing may still be landing in LDS
    final_epilogue();
  }
};

template <int D, int ACT, bool BWD, int S>
__global__ __launch_bounds__(256, 1) void ffn_chain_kernel(FfnP p) {
  using Ch = Chain<D, ACT, BWD, S>;
  __shared__ __attribute__((aligned(16))) char smem[Ch::LDS_BYTES];
  Ch ch(p, reinterpret_cast<bf16_t*>(smem));
  ch.run();
}

template <int D, bool BWD, int S>
int launch_chain(const FfnP& p, int act, hipStream_t st) {
  const unsigned g = (unsigned)cdiv(p.M, FB_M);
  if (act == LASR_ACT_RELU) ffn_chain_kernel<D, LASR_ACT_RELU, BWD, S><<<g, 256, 0, st>>>(p);
  else ffn_chain_kernel<D, LASR_ACT_SWISH, BWD, S><<<g, 256, 0, st>>>(p);
  return lasr_check_launch(BWD ? "ffn_bwd_dx" : "ffn_fwd");
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

int check_args(const lasr_ffn_args* a, bool bwd) {
  LASR_CHECK_ARG(a != nullptr, "lasr_ffn: null args");
  LASR_CHECK_ARG(a->D == 256 || a->D == 512, "lasr_ffn: D must be 256 or 512 (got %d)", a->D);
  LASR_CHECK_ARG(a->F > 0 && a->F % FB_CH == 0, "lasr_ffn: F must be a positive multiple of 128");
  LASR_CHECK_ARG(a->M >= 0, "lasr_ffn: negative M");
  LASR_CHECK_ARG(a->act == LASR_ACT_RELU || a->act == LASR_ACT_SWISH, "lasr_ffn: act must be relu or swish");
  LASR_CHECK_ARG(a->x && a->W1 && a->W2 && al16(a->x) && al16(a->W1) && al16(a->W2),
                 "lasr_ffn: x/W1/W2 must be non-null and 16-B aligned");
  if (!bwd) {
    LASR_CHECK_ARG(a->b1 && a->b2 && a->out && al16(a->b1) && al16(a->b2) && al16(a->out),
                   "lasr_ffn_fwd: b1/b2/out must be non-null and 16-B aligned");
    LASR_CHECK_ARG(a->z && a->h && al16(a->z) && al16(a->h) && (!a->res || al16(a->res)),
                   "lasr_ffn_fwd: z/h must be non-null, z/h/res 16-B aligned");
    LASR_CHECK_ARG(a->F <= FB_MAXF, "lasr_ffn_fwd: F > %d", FB_MAXF);
  } else {
    LASR_CHECK_ARG(a->z && a->dz && a->dx && al16(a->z) && al16(a->dz) && al16(a->dx),
                   "lasr_ffn_bwd_dx: z/dz/dx must be non-null and 16-B aligned");
  }
  return LASR_OK;
}

FfnP make_params(const lasr_ffn_args* a) {
  FfnP p;
  p.M = a->M;
  p.F = a->F;
  p.x = (const bf16_t*)a->x;
  p.W1 = (const bf16_t*)a->W1;
  p.b1 = a->b1;
  p.W2 = (const bf16_t*)a->W2;
  p.b2 = a->b2;
  p.d1 = mkdrop(a->p1, a->seed1);
  p.d2 = mkdrop(a->p2, a->seed2);
  p.res = a->res;
  p.res_scale = a->res_scale;
  p.z = (bf16_t*)a->z;
  p.h = (bf16_t*)a->h;
  p.out = a->out;
  p.dz = (bf16_t*)a->dz;
  p.dx = (bf16_t*)a->dx;
  return p;
}

}  // namespace

extern "C" int lasr_ffn_fwd(const lasr_ffn_args* a, void* stream) {
  int rc = check_args(a, false);
  if (rc) return rc;
  if (a->M == 0) return LASR_OK;
  const FfnP p = make_params(a);
  hipStream_t st = (hipStream_t)stream;
  return a->D == 256 ? launch_chain<256, false, 7>(p, a->act, st) : launch_chain<512, false, 3>(p, a->act, st);
}

extern "C" int lasr_ffn_bwd_dx(const lasr_ffn_args* a, void* stream) {
  int rc = check_args(a, true);
  if (rc) return rc;
  if (a->M == 0) return LASR_OK;
  const FfnP p = make_params(a);
  hipStream_t st = (hipStream_t)stream;
  return a->D == 256 ? launch_chain<256, true, 7>(p, a->act, st) : launch_chain<512, true, 3>(p, a->act, st);
}
