// Kernel templates of the generic GEMM (gemm.hip) and its implicit-GEMM conv instances
// (gemm_conv.hip): operand tiles, epilogues, the register-staged / LDS-DMA / fp32 kernels and
// the split-K reduction.  Split from gemm.hip so the two translation units compile in parallel.
#pragma once
#include "common.h"
#include "tile.h"

#include <cstring>
#include <type_traits>

// Ablation hooks for GEMM experiments (tools/gemm_exp.sh); 0 in every product build.
// bit 1: skip the MFMAs, bit 2: skip the epilogue stores, bit 4: skip the glds loads,
// bit 8: no dropout draws in the Swish-gate epilogue (keep all), bit 16: no activation math there.
#ifndef LASR_EXP
#define LASR_EXP 0
#endif


// Geometry of the subsampling conv2 (3x3, stride 2, C -> C, channels-last y1 [B,T1,F1,C]) for
// the implicit-GEMM kernel instances (G_FWD / G_DW / G_DX below).
struct ConvG {
  int B, T1, F1, T2, F2, C;
  int M2;               // B * T2 * F2 (rows of y2 / dy2)
  int cls;              // G_DX: output parity class (t1 & 1) * 2 + (f1 & 1)
  int q32, r32;         // G_DW: 32 = q32 * F2 + r32 (row-walk increments)
  const bf16_t* zero;   // G_DX: >= 32 zero bf16 (taps that fall outside dy2)
  // G_DX with EPI_AUX_RELU_W1 (the conv1 weight gradient in the epilogue): conv1's input
  // x [B, T0, F0] fp32, the per-tile partials [rows][10][C] and this class's first row
  const float* x;
  int T0, F0;
  float* w1part;
  int w1rb;
};
typedef ConvG ConvGeom;
enum { G_LIN = 0, G_FWD = 1, G_DW = 2, G_DX = 3 };

struct GemmP {
  int M, N, K, batch, batch_div;
  const void* A;
  int64_t lda_m, lda_k, sa1, sa2;
  const void* B;
  int64_t ldb_n, ldb_k, sb1, sb2;
  void* C;
  int64_t ldc, sc1, sc2;
  float alpha;
  const float* alpha_dev;
  float beta;
  const float* bias;
  int act;
  void* zout;
  const void* aux;
  int aux_dtype;
  int64_t ldaux;
  int aux_act;
  DropCfg drop;
  const void* res;
  int res_dtype;
  int64_t ldres;
  float res_scale;
  int split_k;
  int kchunk;
  float* ws;
  int a_vec, b_vec;
  int c_vec, aux_vec, res_vec, ws_vec;  // 8-wide epilogue access allowed
  // Epilogue mode of the bf16 kernel: 0 = no per-element loads, 1 = exactly one of
  // aux/res, 16-B aligned and prefetched before the staging barrier, 2 = generic.
  int epi_mode;
  int bias_vec;
  // rowsum[m] += sum_k A[m,k] (bias gradient of a dW = dY^T X GEMM): computed by the
  // n-tile-0 blocks of the LDS-DMA kernel (A M-contiguous); split-K slices write
  // partials to rs_ws[s*M + m], summed in fixed order by splitk_reduce_kernel.
  float* rowsum;
  float* rs_ws;
  int v4;  // direct epilogue: 4-wide C/zout/aux/res/bias/ws access allowed (host-checked)
  int zout_mode;  // 0: zout = pre-activation; 1: zout = act'(pre-activation) * keep (gate)
  ConvGeom cv;    // implicit-GEMM instances of the subsampling conv2 only (G != 0)
};

// A row post-op that may take over a split-K GEMM's reduction launch (gemm_ln.hip: the
// reduction fused with the next LayerNorm, forward or backward).  launch returns 1 when it
// launched the fused reduction (done), 0 when lasr_gemm must run the plain one, < 0 on error.
struct GemmRowPost {
  int (*launch)(const GemmP& p, const void* ctx, hipStream_t st);
  const void* ctx;
  int done;
};
struct lasr_gemm_args;
int gemm_run(const lasr_gemm_args* a, void* stream, GemmRowPost* post);

LASR_DEV float load_any(const void* p, int dt, int64_t i) {
  return dt == LASR_F32 ? ((const float*)p)[i] : bf2f(((const bf16_t*)p)[i]);
}

// Epilogue core on N consecutive columns after bias: zout (pre-activation or gate),
// activation, aux factor, dropout (one draw per column pair), residual.  zst(vals) stores
// the zout values; auxv / resv are the loaded aux / res values (nullable).  Every mode
// switch is a wave-uniform branch around its own loop (a per-element select would make
// the compiler evaluate every activation and its derivative for every element).
// dkey = epi_key(p), computed ONCE per thread before the output loops: drop_key reads the
// device step counter, and a load inside the loop is re-issued and waited for on every
// iteration (the stores in between may alias it).
// Compile-time epilogue modes of the hot FFN GEMMs (host-selected by epi_code, gemm_launch.h):
// the same per-element arithmetic as the runtime path, without its mode branches (which, with
// the uniform values they keep live, cost SGPR spills and ~2x the VALU of the arithmetic).
enum {
  EPI_RT = 0, EPI_SWISH_GATE_DROP = 1, EPI_AUX_GATE = 2, EPI_PLAIN = 3, EPI_RES_DROP = 4, EPI_RELU_GATE_DROP = 5,
  EPI_RELU = 6, EPI_AUX_RELU = 7,
  // G_DX only: EPI_AUX_RELU's values are not stored but reduced into the conv1 weight-gradient
  // partials of the tile (dx_w1_epilogue)
  EPI_AUX_RELU_W1 = 8
};

template <int N, int EPI = EPI_RT, typename ZST>
LASR_DEV void epi_core(const GemmP& p, uint32_t dkey, uint64_t dbase, float (&v)[N], const float (&auxv)[N],
                       bool has_aux, const float (&resv)[N], bool has_res, ZST zst) {
  if constexpr (EPI == EPI_SWISH_GATE_DROP) {
    // zout_mode 1, Swish, dropout on; no aux, residual or beta (FFN fc1 forward)
    const uint32_t km = (LASR_EXP & 8) ? 0xffffffffu : drop_keep_mask_even<N>(p.drop, dkey, dbase);
    float g[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
      if constexpr ((LASR_EXP & 16) != 0) {
        g[q] = v[q];
      } else {
        const float s = sigmoidf_(v[q]);
        g[q] = s * (1.f + v[q] * (1.f - s));
        v[q] *= s;
      }
    }
#pragma unroll
    for (int q = 0; q < N; ++q) g[q] *= (km >> q) & 1u ? 1.f : 0.f;
    zst(g);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= (km >> q) & 1u ? p.drop.scale : 0.f;
    return;
  } else if constexpr (EPI == EPI_AUX_GATE) {
    // v * aux (the stored gate); no activation, zout, dropout or residual (FFN fc1 dz)
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= auxv[q];
    return;
  } else if constexpr (EPI == EPI_RELU_GATE_DROP) {
    // zout_mode 1, ReLU, dropout on; no aux, residual or beta (the decoder's FFN fc1 forward)
    const uint32_t km = drop_keep_mask_even<N>(p.drop, dkey, dbase);
    float g[N];
#pragma unroll
    for (int q = 0; q < N; ++q) g[q] = v[q] > 0.f ? 1.f : 0.f;
#pragma unroll
    for (int q = 0; q < N; ++q) g[q] *= (km >> q) & 1u ? 1.f : 0.f;
    zst(g);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = fmaxf(v[q], 0.f);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= (km >> q) & 1u ? p.drop.scale : 0.f;
    return;
  } else if constexpr (EPI == EPI_RELU) {  // bias + ReLU (subsampling conv2 forward)
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = fmaxf(v[q], 0.f);
    return;
  } else if constexpr (EPI == EPI_AUX_RELU || EPI == EPI_AUX_RELU_W1) {  // * relu'(aux) (conv2 data gradient)
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= auxv[q] > 0.f ? 1.f : 0.f;
    return;
  } else if constexpr (EPI == EPI_PLAIN) {
    return;  // alpha * acc + bias only (input-gradient GEMMs)
  } else if constexpr (EPI == EPI_RES_DROP) {
    // res + res_scale * dropout(v), dropout on; no activation, zout or aux (residual projections)
    const uint32_t km = drop_keep_mask_even<N>(p.drop, dkey, dbase);
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= (km >> q) & 1u ? p.drop.scale : 0.f;
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = resv[q] + p.res_scale * v[q];
    return;
  }
  const bool drop = p.drop.p > 0.f;
  const uint32_t km = drop ? drop_keep_mask<N>(p.drop, dkey, dbase) : 0u;
  bool acted = false;  // activation already applied (the gate shares the sigmoid)
  if (p.zout) {
    if (p.zout_mode == 1) {
      float g[N];
      if (p.act == LASR_ACT_SWISH) {
#pragma unroll
        for (int q = 0; q < N; ++q) {
          const float s = sigmoidf_(v[q]);  // = swish_grad / swishf's sigmoid, evaluated once
          g[q] = s * (1.f + v[q] * (1.f - s));
          v[q] *= s;
        }
        acted = true;
      } else if (p.act == LASR_ACT_RELU) {
#pragma unroll
        for (int q = 0; q < N; ++q) g[q] = v[q] > 0.f ? 1.f : 0.f;
      } else if (p.act == LASR_ACT_TANH) {
#pragma unroll
        for (int q = 0; q < N; ++q) {
          v[q] = tanhf(v[q]);
          g[q] = 1.f - v[q] * v[q];
        }
        acted = true;
      } else {
#pragma unroll
        for (int q = 0; q < N; ++q) g[q] = 1.f;
      }
      if (drop) {
#pragma unroll
        for (int q = 0; q < N; ++q) g[q] *= (km >> q) & 1u ? 1.f : 0.f;
      }
      zst(g);
    } else {
      zst(v);
    }
  }
  if (acted) {
  } else if (p.act == LASR_ACT_SWISH) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = swishf(v[q]);
  } else if (p.act == LASR_ACT_RELU) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = fmaxf(v[q], 0.f);
  } else if (p.act == LASR_ACT_TANH) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = tanhf(v[q]);
  }
  if (has_aux) {
    if (p.aux_act == LASR_ACT_GATE) {
#pragma unroll
      for (int q = 0; q < N; ++q) v[q] *= auxv[q];
    } else if (p.aux_act == LASR_ACT_RELU) {
#pragma unroll
      for (int q = 0; q < N; ++q) v[q] *= auxv[q] > 0.f ? 1.f : 0.f;
    } else if (p.aux_act == LASR_ACT_TANH) {  // aux = the stored tanh output y: tanh' = 1 - y^2
#pragma unroll
      for (int q = 0; q < N; ++q) v[q] *= 1.f - auxv[q] * auxv[q];
    } else {
#pragma unroll
      for (int q = 0; q < N; ++q) v[q] *= swish_grad(auxv[q]);
    }
  }
  if (drop) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] *= (km >> q) & 1u ? p.drop.scale : 0.f;  // x * 0 keeps NaN, as torch
  }
  if (has_res) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = resv[q] + p.res_scale * v[q];
  }
}

// Dropout key of a GEMM epilogue (0 without dropout).
LASR_DEV uint32_t epi_key(const GemmP& p) { return p.drop.p > 0.f ? drop_key(p.drop) : 0u; }

// Full epilogue for one output element.
template <typename TC>
LASR_DEV void epi_store(const GemmP& p, uint32_t dkey, int z1, int z2, int z, int m, int n, float acc,
                        float alpha_eff) {
  if (m >= p.M || n >= p.N) return;
  float v[1] = {acc * alpha_eff};
  if (p.bias) v[0] += p.bias[n];
  const int64_t cidx = (int64_t)z1 * p.sc1 + (int64_t)z2 * p.sc2 + (int64_t)m * p.ldc + n;
  float a[1], r[1];
  if (p.aux) a[0] = load_any(p.aux, p.aux_dtype, (int64_t)m * p.ldaux + n);
  if (p.res) r[0] = load_any(p.res, p.res_dtype, (int64_t)m * p.ldres + n);
  epi_core<1>(p, dkey, ((uint64_t)z * p.M + m) * (uint64_t)p.N + n, v, a, p.aux != nullptr, r, p.res != nullptr,
              [&](const float (&zv)[1]) { ((TC*)p.zout)[cidx] = from_f<TC>(zv[0]); });
  TC* C = (TC*)p.C;
  if (p.beta != 0.f) v[0] += p.beta * to_f(C[cidx]);
  C[cidx] = from_f<TC>(v[0]);
}

// 8 values of a (f32|bf16) matrix row starting at element idx; cnt < 8 -> tail.
LASR_DEV void ld_any8(const void* base, int dt, int64_t idx, bool vec, int cnt, float* o) {
  if (vec && cnt == 8) {
    if (dt == LASR_F32) ld8((const float*)base + idx, o);
    else ld8((const bf16_t*)base + idx, o);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = q < cnt ? load_any(base, dt, idx + q) : 0.f;
  }
}
template <typename T>
LASR_DEV void st_8(T* dst, const float* v, bool vec, int cnt) {
  if ((LASR_EXP & 2) && v[0] != 1234.5f) return;
  if (vec && cnt == 8) st8(dst, v);
  else {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < cnt) dst[q] = from_f<T>(v[q]);
  }
}

// Epilogue for 8 consecutive columns n..n+7 of row m (same order as epi_store).
template <typename TC>
LASR_DEV void epi_store8(const GemmP& p, uint32_t dkey, int z1, int z2, int z, int m, int n, const float* acc,
                         float alpha_eff) {
  const int cnt = min(8, p.N - n);
  float v[8], t[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = acc[q] * alpha_eff;
  if (p.bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += q < cnt ? p.bias[n + q] : 0.f;
  }
  const int64_t cidx = (int64_t)z1 * p.sc1 + (int64_t)z2 * p.sc2 + (int64_t)m * p.ldc + n;
  float r[8];
  if (p.aux) ld_any8(p.aux, p.aux_dtype, (int64_t)m * p.ldaux + n, p.aux_vec, cnt, t);
  if (p.res) ld_any8(p.res, p.res_dtype, (int64_t)m * p.ldres + n, p.res_vec, cnt, r);
  epi_core<8>(p, dkey, ((uint64_t)z * p.M + m) * (uint64_t)p.N + n, v, t, p.aux != nullptr, r, p.res != nullptr,
              [&](const float (&zv)[8]) { st_8((TC*)p.zout + cidx, zv, p.c_vec, cnt); });
  TC* C = (TC*)p.C + cidx;
  if (p.beta != 0.f) {
    ld_any8(C, sizeof(TC) == 4 ? LASR_F32 : LASR_BF16, 0, p.c_vec, cnt, t);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += p.beta * t[q];
  }
  st_8(C, v, p.c_vec, cnt);
}

// Epilogue modes 0/1: bias already in registers (bv), the one aux/res source prefetched
// (sv, mode 1 only; N % 8 == 0 there), beta == 0; cnt < 8 only on a ragged last vector.
template <typename TC, int EPI = EPI_RT>
LASR_DEV void epi_fast8(const GemmP& p, uint32_t dkey, int64_t cidx, int z, int m, int n, int cnt,
                        const float* acc, float alpha_eff, const float* bv, const float (&sv)[8]) {
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = acc[q] * alpha_eff + bv[q];
  epi_core<8, EPI>(p, dkey, ((uint64_t)z * p.M + m) * (uint64_t)p.N + n, v, sv, p.aux != nullptr, sv, p.res != nullptr,
              [&](const float (&zv)[8]) { st_8((TC*)p.zout + cidx, zv, true, cnt); });
  st_8((TC*)p.C + cidx, v, true, cnt);
}

LASR_DEV float alpha_of(const GemmP& p) {
  return p.alpha_dev ? p.alpha * p.alpha_dev[0] : p.alpha;
}

// ============================ bf16 MFMA kernel ===================================
// ============================ bf16 MFMA kernel ===================================
// (tile images, fragment reads, LDS-DMA issue and ring waits: tile.h)

// Epilogue shared by the bf16 kernels: stage each half of the C tile (WM rows x BN cols,
// fp32) through LDS, then every thread finishes 8 contiguous columns of a row with 16-B
// loads/stores (or writes its split-K partial).  The caller has passed a barrier after its
// last LDS read of the main loop.
// Element offset of output row m of a G_DX launch: class row (b, i, j) -> dy1 position
// (b, 2i + pt, 2j + pf), channels-last.
LASR_DEV int64_t dx_row(const ConvG& g, int m) {
  const int pt = g.cls >> 1, pf = g.cls & 1;
  const int nI = (g.T1 - pt + 1) >> 1, nJ = (g.F1 - pf + 1) >> 1;
  const int j = m % nJ, t = m / nJ, i = t % nI, b = t / nI;
  return ((int64_t)(b * g.T1 + 2 * i + pt) * g.F1 + 2 * j + pf) * g.C;
}

// dxrow (G_DX only): the tile's BM row offsets dx_row(m0 + r), computed once per tile (two
// integer divisions and two remainders each; per output vector they cost more VALU than the
// epilogue arithmetic).
template <int BM, int BN, typename TC, bool TRANS = false, int G = G_LIN, int NW = 4, int EPI = EPI_RT>
LASR_DEV void gemm_epilogue(const GemmP& p, f32x4 (&acc)[BM / 32][BN / (8 * NW)], char* smem_epi, int m0,
                            int n0, int s, int z, int z1, int z2, const int64_t* dxrow = nullptr) {
  // output-row offsets: linear (ldc, ld of the aux/res source), or the transposed-conv scatter
  // of a G_DX launch (aux = y1 shares dy1's layout)
  auto crow = [&](int m) -> int64_t {
    if constexpr (G == G_DX) return dxrow[m - m0];
    else return (int64_t)z1 * p.sc1 + (int64_t)z2 * p.sc2 + (int64_t)m * p.ldc;
  };
  // NW waves as 2 (rows) x NW/2 (columns); NT threads finish the staged rows
  constexpr int NT = NW * 64, WCOLS = NW / 2;
  constexpr int WM = BM / 2, WN = BN / WCOLS, FM = WM / 16, FN = WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WCOLS, wc = wid % WCOLS;
  constexpr int LDC = BN + 4;  // +4 floats: the 4 row-groups of a write land on distinct banks
  float* cs = reinterpret_cast<float*>(smem_epi);
  const int rq = (lane >> 4) * 4, cl = lane & 15;
  const float al = alpha_of(p);
  const uint32_t dkey = epi_key(p);
  const bool split = p.split_k > 1;
  float* wsp = split ? p.ws + ((int64_t)s * p.batch + z) * (int64_t)p.M * p.N : nullptr;
  // A thread's 8-column slot is the same in every epilogue iteration (NT % (BN/8) == 0):
  // its bias is loaded once; the aux/res rows of a half are prefetched before the barrier.
  constexpr int CPR = BN / 8, RPI = NT / CPR, ITERS = WM / RPI;
  static_assert(WM % RPI == 0, "epilogue tiling");
  const int ec8 = (tid % CPR) * 8, er0 = tid / CPR;
  const int en = n0 + ec8;
  // conv instances are host-checked onto the fast path (no split here, epi_mode < 2)
  const bool fast = G != G_LIN || (!split && p.epi_mode < 2);
  float bv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bv[q] = 0.f;
  if (fast && p.bias && en < p.N) {
    if (p.bias_vec && en + 8 <= p.N) ld8(p.bias + en, bv);
    else
#pragma unroll
      for (int q = 0; q < 8; ++q) bv[q] = en + q < p.N ? p.bias[en + q] : 0.f;
  }
  const void* src = p.aux ? p.aux : p.res;
  const int src_dt = p.aux ? p.aux_dtype : p.res_dtype;
  const int64_t src_ld = p.aux ? p.ldaux : p.ldres;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // prefetch PF row-iterations of the aux/res source at a time (register budget)
    constexpr int PF = ITERS < 2 ? ITERS : 2;
    float sv[PF][8];
    auto prefetch = [&](int b) {
      if (!(fast && p.epi_mode == 1)) return;
      const int mlast = p.M - 1, nc = min(en, p.N - 8);
      if (src_dt == LASR_F32) {
#pragma unroll
        for (int it = 0; it < PF; ++it) {
          const int m = min(m0 + h * WM + er0 + (b + it) * RPI, mlast);
          const int64_t ro = G == G_DX ? dxrow[m - m0] : (int64_t)m * src_ld;
          ld8((const float*)src + ro + nc, sv[it]);
        }
      } else {
#pragma unroll
        for (int it = 0; it < PF; ++it) {
          const int m = min(m0 + h * WM + er0 + (b + it) * RPI, mlast);
          const int64_t ro = G == G_DX ? dxrow[m - m0] : (int64_t)m * src_ld;
          ld8((const bf16_t*)src + ro + nc, sv[it]);
        }
      }
    };
    prefetch(0);
    if (wr == h) {
      if constexpr (TRANS) {
        // C^T fragments: lane owns row cl, columns rq..rq+3 -> one 16-B LDS write each
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            *(f32x4*)(cs + (i * 16 + cl) * LDC + wc * WN + j * 16 + rq) = acc[i][j];
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) cs[(i * 16 + rq + e) * LDC + wc * WN + j * 16 + cl] = acc[i][j][e];
      }
    }
    __syncthreads();
    if (fast) {
#pragma unroll
      for (int b = 0; b < ITERS; b += PF) {
        if (b > 0) prefetch(b);
#pragma unroll
        for (int it = 0; it < PF; ++it) {
          const int r = er0 + (b + it) * RPI;
          const int m = m0 + h * WM + r;
          if (m < p.M && en < p.N) {
            float a8[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) a8[q] = cs[r * LDC + ec8 + q];
            epi_fast8<TC, EPI>(p, dkey, crow(m) + en, z, m, en, min(8, p.N - en), a8, al, bv, sv[it]);
          }
        }
      }
      __syncthreads();
      continue;
    }
    constexpr int NV = WM * BN / 8;
    for (int v = tid; v < NV; v += NT) {
      const int r = v / (BN / 8), c8 = (v % (BN / 8)) * 8;
      const int m = m0 + h * WM + r, n = n0 + c8;
      if (m < p.M && n < p.N) {
        float a8[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) a8[q] = cs[r * LDC + c8 + q];
        if (split) {
          float* dst = wsp + (int64_t)m * p.N + n;
          if (p.ws_vec && n + 8 <= p.N) st8(dst, a8);
          else
            for (int q = 0; q < 8 && n + q < p.N; ++q) dst[q] = a8[q];
        } else {
          epi_store8<TC>(p, dkey, z1, z2, z, m, n, a8, al);
        }
      }
    }
    __syncthreads();
  }
}

template <int BM, int BN, bool AKC, bool BKC, typename TC>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmP p) {
  constexpr int BK = 32;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int MAIN_BYTES = 2 * (BM + BN) * BK * 2;
  constexpr int EPI_BYTES = WM * (BN + 4) * 4;
  __shared__ __attribute__((aligned(16))) char smem_epi[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_epi);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  const int zz = blockIdx.z;
  const int s = zz % p.split_k, z = zz / p.split_k;
  const int z1 = z / p.batch_div, z2 = z % p.batch_div;
  const bf16_t* A = (const bf16_t*)p.A + z1 * p.sa1 + z2 * p.sa2;
  const bf16_t* B = (const bf16_t*)p.B + z1 * p.sb1 + z2 * p.sb2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = s * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  TileLoader<BM, AKC> la;
  TileLoader<BN, BKC> lb;
  const int64_t a_ldr = AKC ? p.lda_m : 0, a_ldk = AKC ? 0 : p.lda_k;
  const int64_t b_ldr = BKC ? p.ldb_n : 0, b_ldk = BKC ? 0 : p.ldb_k;

  if (nk > 0) {
    la.load(A, a_ldr, a_ldk, m0, p.M, kbeg, kend, p.a_vec, tid);
    lb.load(B, b_ldr, b_ldk, n0, p.N, kbeg, kend, p.b_vec, tid);
    la.store(smem, tid);
    lb.store(smem + BM * BK, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    bf16_t* cur = smem + (kt & 1) * (BM + BN) * BK;
    bf16_t* nxt = smem + ((kt + 1) & 1) * (BM + BN) * BK;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      la.load(A, a_ldr, a_ldk, m0, p.M, k0, kend, p.a_vec, tid);
      lb.load(B, b_ldr, b_ldk, n0, p.N, k0, kend, p.b_vec, tid);
    }
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = frag<BM, AKC>(cur, wr * WM + i * 16, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = frag<BN, BKC>(cur + BM * BK, wc * WN + j * 16, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) {
      la.store(nxt, tid);
      lb.store(nxt + BM * BK, tid);
    }
    __syncthreads();
  }

  gemm_epilogue<BM, BN, TC>(p, acc, smem_epi, m0, n0, s, z, z1, z2);
}

// Epilogue of 4 consecutive columns n..n+3 of row m (same order as epi_store8); cnt < 4 or
// !vec -> element-wise tail.
// The value a TC store keeps, back in fp32 (the bf16 rounding of stv / pk_bf16).
template <typename TC>
LASR_DEV float stored_value(float x) {
  if constexpr (sizeof(TC) == 4) return x;
  else return __uint_as_float(pk_bf16(x, 0.f) << 16);
}

// vout (optional): the 4 values as stored in C (the row-LayerNorm post-ops of gemm_ln.hip
// continue from them in registers)
template <typename TC, bool VEC>
LASR_DEV void epi_store4(const GemmP& p, uint32_t dkey, int z1, int z2, int z, int m, int n, int cnt,
                         const float* acc, float al, float* vout = nullptr) {
  float v[4], t[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = acc[q] * al;
  if (p.bias) {
    if (VEC) {
      ldv<4>(p.bias + n, t);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = q < cnt ? p.bias[n + q] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += t[q];
  }
  const int64_t cidx = (int64_t)z1 * p.sc1 + (int64_t)z2 * p.sc2 + (int64_t)m * p.ldc + n;
  auto st4 = [&](TC* dst, const float* x) {
    if (VEC) stv<4>(dst, x);
    else
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < cnt) dst[q] = from_f<TC>(x[q]);
  };
  auto ld4 = [&](const void* base, int dtp, int64_t idx, float* o) {
    if (VEC) {
      if (dtp == LASR_F32) ldv<4>((const float*)base + idx, o);
      else ldv<4>((const bf16_t*)base + idx, o);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = q < cnt ? load_any(base, dtp, idx + q) : 0.f;
    }
  };
  float r[4];
  if (p.aux) ld4(p.aux, p.aux_dtype, (int64_t)m * p.ldaux + n, t);
  if (p.res) ld4(p.res, p.res_dtype, (int64_t)m * p.ldres + n, r);
  epi_core<4>(p, dkey, ((uint64_t)z * p.M + m) * (uint64_t)p.N + n, v, t, p.aux != nullptr, r, p.res != nullptr,
              [&](const float (&zv)[4]) { st4((TC*)p.zout + cidx, zv); });
  TC* C = (TC*)p.C + cidx;
  if (p.beta != 0.f) {
    ld4(C, sizeof(TC) == 4 ? LASR_F32 : LASR_BF16, 0, t);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += p.beta * t[q];
  }
  if ((LASR_EXP & 2) && v[0] != 1234.5f) return;
  st4(C, v);
  if (vout) {
#pragma unroll
    for (int q = 0; q < 4; ++q) vout[q] = stored_value<TC>(v[q]);
  }
}

// Epilogue straight from the accumulators, no LDS and no barrier.  The main loop issues
// the MFMAs with the operands swapped (D = B-frag x A-frag), so acc[i][j] is a fragment of
// C^T: lane l owns row m = mb + (l & 15) and the 4 consecutive columns nb + 4 (l >> 4) + e
// -> one 8-B (bf16) / 16-B (fp32) access per 4 outputs (a wave instruction covers 16 rows
// x 32 / 64 contiguous bytes; the L2 merges the row segments before write-back).
template <int BM, int BN, typename TC, int NW = 4>
LASR_DEV void gemm_epilogue_direct(const GemmP& p, f32x4 (&acc)[BM / 32][BN / (8 * NW)], int m0, int n0, int s,
                                   int z, int z1, int z2) {
  constexpr int WCOLS = NW / 2;
  constexpr int WM = BM / 2, WN = BN / WCOLS, FM = WM / 16, FN = WN / 16;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid / WCOLS, wc = wid % WCOLS;
  const float al = alpha_of(p);
  const uint32_t dkey = epi_key(p);
  const int mr = m0 + wr * WM + (lane & 15), nc = n0 + wc * WN + 4 * (lane >> 4);
  if (p.split_k > 1) {
    float* wsp = p.ws + ((int64_t)s * p.batch + z) * (int64_t)p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mr + i * 16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nc + j * 16;
        if (n >= p.N) continue;
        float* dst = wsp + (int64_t)m * p.N + n;
        const float a[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (p.v4 && n + 4 <= p.N) stv<4>(dst, a);
        else
          for (int q = 0; q < 4 && n + q < p.N; ++q) dst[q] = a[q];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = mr + i * 16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nc + j * 16;
      if (n >= p.N) continue;
      const float a[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (p.v4 && n + 4 <= p.N) epi_store4<TC, true>(p, dkey, z1, z2, z, m, n, 4, a, al);
      else epi_store4<TC, false>(p, dkey, z1, z2, z, m, n, min(4, p.N - n), a, al);
    }
  }
}

// Epilogue of the conv2 data gradient fused with conv1's weight gradient (EPI_AUX_RELU_W1,
// BM x 256 tiles, 4 waves): dy1 = bf16(acc) * relu'(y1) -- exactly the values the plain G_DX
// epilogue stores -- is never written; the tile's partial of dW1 [C][9] / db1 [C] is formed
// instead.  (1) every wave parks its accumulators as bf16 in LDS (the whole tile at once:
// 128 x 264 bf16 + the rows' conv1 patches xr -> [BM][12] fp32, 73.7 KB, inside the ring's
// space); (2) wave w takes rows w, w + NW, ..., lane l columns 4l..4l+3: per row one 8-B LDS
// read of v, the row's y1 (8 B per lane, coalesced 512-B rows, all loads issued before the
// staging), three broadcast 16-B reads of its patch, 20 packed FMAs into 40 accumulators;
// (3) the NW waves' sums combined in fixed order through LDS into one [10][C] partial row.
// The per-element work is ~20 VALU per 4 outputs; LDS traffic stays below it (the first,
// LDS-bound form -- fp32 staging and a column-per-thread sum with 9 patch reads per 4 rows --
// cost 53 us over the 343 us launch).
template <int BM, int BN, int NW>
LASR_DEV void dx_w1_epilogue(const GemmP& p, f32x4 (&acc)[BM / 32][BN / (8 * NW)], char* smem, int m0, int n0,
                             const int64_t* dxrow, const float (&xr)[(9 * BM + NW * 64 - 1) / (NW * 64)]) {
  static_assert(BN == 256 && NW == 4, "conv1 weight gradient: 4 columns per lane over a 256-column tile");
  constexpr int NT = NW * 64, WCOLS = NW / 2;
  constexpr int WM = BM / 2, WN = BN / WCOLS, FM = WM / 16, FN = WN / 16;
  constexpr int LDB = BN + 8;        // bf16 row stride of the parked tile (528 B: rows 4 banks apart)
  constexpr int RPW = BM / NW;       // rows per wave
  constexpr int XN = (9 * BM + NT - 1) / NT;
  static_assert(BM * LDB * 2 + BM * 12 * 4 <= 73728 && NW * 10 * BN * 4 <= BM * LDB * 2, "LDS budget");
  bf16_t* tb = reinterpret_cast<bf16_t*>(smem);
  float* xs = reinterpret_cast<float*>(smem + BM * LDB * 2);  // [BM][12]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WCOLS, wc = wid % WCOLS;
  // this wave's rows of y1 (the relu' factor), in flight during the staging
  const bf16_t* y1 = (const bf16_t*)p.aux;
  uint2 ya[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int r = wid + NW * i;
    ya[i] = m0 + r < p.M ? *(const uint2*)(y1 + dxrow[r] + n0 + 4 * lane) : make_uint2(0u, 0u);
  }
  // (the tile has passed a barrier after its last ring read; the epilogue's barriers are
  // LDS-only, so the y1 loads stay in flight across them)
  {
    const int rq = (lane >> 4) * 4, cl = lane & 15;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wr * WM + i * 16 + cl, c = wc * WN + j * 16 + rq;
        *(uint2*)(tb + r * LDB + c) = make_uint2(pk_bf16(acc[i][j][0], acc[i][j][1]), pk_bf16(acc[i][j][2], acc[i][j][3]));
      }
#pragma unroll
    for (int i = 0; i < XN; ++i) {
      const int e = i * NT + tid;
      if (e < 9 * BM) xs[(e / 9) * 12 + e % 9] = xr[i];
    }
  }
  lds_barrier();
  lasr_f2 w[10][2];
#pragma unroll
  for (int k = 0; k < 10; ++k) w[k][0] = w[k][1] = (lasr_f2){0.f, 0.f};
#pragma unroll  // (fully: ya[] stays in registers)
  for (int i = 0; i < RPW; ++i) {
    const int r = wid + NW * i;
    const uint2 vb = *(const uint2*)(tb + r * LDB + 4 * lane);
    const uint2 ab = ya[i];
    // bf16 -> fp32 is exact; times relu'(y1) in {0, 1} as the store path (which rounds after
    // the product: the same value)
    const lasr_f2 g0 = {__uint_as_float(ab.x << 16) > 0.f ? 1.f : 0.f, __uint_as_float(ab.x & 0xffff0000u) > 0.f ? 1.f : 0.f};
    const lasr_f2 g1 = {__uint_as_float(ab.y << 16) > 0.f ? 1.f : 0.f, __uint_as_float(ab.y & 0xffff0000u) > 0.f ? 1.f : 0.f};
    const lasr_f2 v0 = (lasr_f2){__uint_as_float(vb.x << 16), __uint_as_float(vb.x & 0xffff0000u)} * g0;
    const lasr_f2 v1 = (lasr_f2){__uint_as_float(vb.y << 16), __uint_as_float(vb.y & 0xffff0000u)} * g1;
    const f32x4 xa = *(const f32x4*)(xs + r * 12), xb = *(const f32x4*)(xs + r * 12 + 4),
                xc = *(const f32x4*)(xs + r * 12 + 8);
    const float xv[9] = {xa[0], xa[1], xa[2], xa[3], xb[0], xb[1], xb[2], xb[3], xc[0]};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const lasr_f2 xx = {xv[k], xv[k]};
      w[k][0] += v0 * xx;
      w[k][1] += v1 * xx;
    }
    w[9][0] += v0;
    w[9][1] += v1;
  }
  lds_barrier();  // the parked tile is no longer read: its space takes the wave sums
  float* red = reinterpret_cast<float*>(smem);  // [NW][10][BN]
#pragma unroll
  for (int k = 0; k < 10; ++k)
    *(f32x4*)(red + (wid * 10 + k) * BN + 4 * lane) = (f32x4){w[k][0][0], w[k][0][1], w[k][1][0], w[k][1][1]};
  lds_barrier();
  float* dst = p.cv.w1part + (int64_t)(p.cv.w1rb + m0 / BM) * 10 * p.N + n0 + tid;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += red[(q * 10 + k) * BN + tid];
    dst[(int64_t)k * p.N] = t;
  }
}

// ---------------- bf16 kernel, LDS-DMA pipeline (16-B aligned operands) ----------------
// Same tiles, LDS images, fragment reads and epilogue as gemm_bf16_kernel, but every full
// 32-deep k tile is copied HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging) into an
// S-stage ring, S-1 tiles in flight.  The image is lane-linear per wave instruction, so the
// swizzles of lds_off / tr_off are applied to the SOURCE address (the XOR maps are
// involutions).  One raw barrier per k tile, preceded by a counted vmcnt that retires only
// the tile about to be read.  A ragged last k tile goes through the register loader
// (zero fill).  Rows past M/N read clamped (valid) addresses; they only feed discarded
// outputs.  Blocks are remapped so consecutive tiles share an XCD (and its L2).

// Implicit-GEMM operand walkers of the subsampling conv2 instances (G != G_LIN).  Each
// keeps per-thread element offsets of the 16-B LDS-DMA positions it issues (the positions
// of glds_tile), so an issue is one add per position.
//  G_FWD, A = im2col(y1) [M2, 9C], K-contiguous: row m = (b, t2, f2) starts at y1 position
//    (b, 2 t2, 2 f2); column k = (kh*3 + kw)*C + cin adds ((kh F1 + kw) C + cin): separable.
//  G_DX, A = dy2 rows of the taps that reach output class (pt, pf), K-contiguous: row m =
//    (b, i, j), output (b, 2i+pt, 2j+pf); tap (dt, df) reads dy2 row (b, i-dt, j-df), or the
//    zero row when that falls outside [0,T2) x [0,F2).
//  G_DW, B = im2col(y1) [M2, 9C] with k = m2 rows (M/N-contiguous operand): every k row is a
//    contiguous run of one tap; the row walk advances (b, t2, f2) by 32 rows per tile.
template <int R_TILE, int NT = 256>
struct ConvRowsKC {  // G_FWD / G_DX A operand
  static constexpr int PER = R_TILE * 4 / NT;
  int off[PER];
  int vm[PER];  // G_DX: bit dt*2+df set when tap (dt, df) is inside dy2
  LASR_DEV void init_fwd(const ConvG& g, int row0, int R, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int P = i * NT + tid, r = P >> 2, c = (P & 3) ^ swz(r);
      const int m = min(row0 + r, R - 1);
      const int f2 = m % g.F2, t = m / g.F2, t2 = t % g.T2, b = t / g.T2;
      off[i] = ((b * g.T1 + 2 * t2) * g.F1 + 2 * f2) * g.C + c * 8;
      vm[i] = 0;
    }
  }
  LASR_DEV void init_dx(const ConvG& g, int row0, int R, int tid) {
    const int pt = g.cls >> 1, pf = g.cls & 1;
    const int nI = (g.T1 - pt + 1) >> 1, nJ = (g.F1 - pf + 1) >> 1;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int P = i * NT + tid, r = P >> 2, c = (P & 3) ^ swz(r);
      const int m = min(row0 + r, R - 1);
      const int j = m % nJ, t = m / nJ, ii = t % nI, b = t / nI;
      off[i] = ((b * g.T2 + ii) * g.F2 + j) * g.C + c * 8;
      const int vt = (ii < g.T2 ? 1 : 0) | (ii >= 1 && ii - 1 < g.T2 ? 2 : 0);
      const int vf = (j < g.F2 ? 1 : 0) | (j >= 1 && j - 1 < g.F2 ? 2 : 0);
      vm[i] = ((vt & 1) && (vf & 1) ? 1 : 0) | ((vt & 1) && (vf & 2) ? 2 : 0) |
              ((vt & 2) && (vf & 1) ? 4 : 0) | ((vt & 2) && (vf & 2) ? 8 : 0);
    }
  }
  LASR_DEV void issue(const bf16_t* base, int64_t koff, bf16_t* dst, int tid) const {
    const int wid = tid >> 6;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(base + off[i] + koff), (lptr_t)(dst + (i * NT + wid * 64) * 8),
                                       16, 0, 0);
  }
  LASR_DEV void issue_dx(const bf16_t* base, int64_t shift, int bit, const bf16_t* zero, bf16_t* dst,
                         int tid) const {
    const int wid = tid >> 6;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c8 = ((i * NT + tid) & 3) * 8;
      const bf16_t* src = (vm[i] >> bit) & 1 ? base + off[i] + shift : zero + c8;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + (i * NT + wid * 64) * 8), 16, 0, 0);
    }
  }
};

template <int R_TILE, int NT = 256>
struct ConvRowsDW {  // G_DW B operand: tile [32 k][R_TILE n] of im2col(y1), k = m2
  static constexpr int PER = R_TILE * 4 / NT, CPR = R_TILE / 8;
  int noff[PER], f2[PER], t2[PER], b[PER];
  LASR_DEV void init(const ConvG& g, int n0, int N, int kbeg, int tid) {
    const int tap = n0 / g.C, kh = tap / 3, kw = tap - 3 * kh;
    const int tbase = (kh * g.F1 + kw) * g.C - tap * g.C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int P = i * NT + tid, k = P / CPR, ps = P % CPR;
      const int ls = ((((ps >> 1) ^ htr<R_TILE>(k))) << 1) | (ps & 1);
      const int gc = min(n0 + ls * 8, ((N + 7) & ~7) - 8);
      noff[i] = tbase + gc;
      const int m = kbeg + k;
      f2[i] = m % g.F2;
      const int t = m / g.F2;
      t2[i] = t % g.T2;
      b[i] = t / g.T2;
    }
  }
  // issue the tile whose k rows are the current walk positions, then advance 32 rows
  LASR_DEV void issue(const ConvG& g, const bf16_t* base, bf16_t* dst, int tid) {
    const int wid = tid >> 6;
    const int last = ((g.B * g.T1 - g.T1 + 2 * (g.T2 - 1)) * g.F1 + 2 * (g.F2 - 1)) * g.C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int rb = b[i] < g.B ? ((b[i] * g.T1 + 2 * t2[i]) * g.F1 + 2 * f2[i]) * g.C : last;
      __builtin_amdgcn_global_load_lds((gptr_t)(base + rb + noff[i]), (lptr_t)(dst + (i * NT + wid * 64) * 8),
                                       16, 0, 0);
      f2[i] += g.r32;
      t2[i] += g.q32;
      if (f2[i] >= g.F2) { f2[i] -= g.F2; t2[i] += 1; }
      while (t2[i] >= g.T2) { t2[i] -= g.T2; b[i] += 1; }
    }
  }
};

// KS: 32-deep k sub-tiles per ring stage (G_LIN only).  KS = 2 makes the stage 64 deep: one
// counted wait + barrier per 64 k and twice the DMA bytes per issue (the guide's "fix BK first").
// XCD-aware (bijective) remap of tile `orig` among `nwg` tiles: tiles that share an XCD (the
// hardware deals blocks round-robin over the 8 XCDs) get consecutive tile indices.
LASR_DEV int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// One output tile (tx, ty) of K slice / batch index zz: the body shared by the launch-grid
// kernel (gemm_bf16_glds_kernel) and the grouped weight-gradient kernel (gemm_dw_group_kernel).
template <int BM, int BN, bool AKC, bool BKC, typename TC, int S, int G, int KS, int NW = 4, int EPI = EPI_RT>
LASR_DEV void gemm_glds_tile(const GemmP& p, const int tx, const int ty, const int zz) {
  static_assert(G == G_LIN || (G == G_DW ? (!AKC && !BKC) : (AKC && (G == G_FWD) == BKC)),
                "gather instance operand orientation");
  static_assert(KS == 1 || KS == 2, "k sub-tiles per ring stage");
  static_assert(NW == 4 || NW == 8, "4 waves (2 x 2) or 8 waves (2 x 4)");
  constexpr int BK = 32;
  constexpr int NT = NW * 64, WCOLS = NW / 2;
  constexpr int WM = BM / 2, WN = BN / WCOLS, FM = WM / 16, FN = WN / 16;
  constexpr int TILE = (BM + BN) * BK;  // elements per 32-deep sub-tile
  constexpr int STAGE = KS * TILE;      // elements per ring stage
  constexpr int MAIN_BYTES = S * STAGE * 2;  // >= the rowsum combine slab (NT/(BM/8) x BM floats)
  constexpr int EPI_BYTES = WM * (BN + 4) * 4;
  constexpr int GL = (BM + BN) * 4 / NT;  // glds per thread per k tile
  __shared__ __attribute__((aligned(16))) char smem_epi[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_epi);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WCOLS, wc = wid % WCOLS;

  const int s = zz % p.split_k, z = zz / p.split_k;
  const int z1 = z / p.batch_div, z2 = z % p.batch_div;
  const bf16_t* A = (const bf16_t*)p.A + z1 * p.sa1 + z2 * p.sa2;
  const bf16_t* B = (const bf16_t*)p.B + z1 * p.sb1 + z2 * p.sb2;
  const int m0 = ty * BM, n0 = tx * BN;
  const int kbeg = s * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int64_t lda = AKC ? p.lda_m : p.lda_k, ldb = BKC ? p.ldb_n : p.ldb_k;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // full 32-deep tiles go through the glds ring; a ragged last tile is handled after the
  // loop (ordinary loads inside the loop would make hipcc drain the ring with vmcnt(0))
  const int nfull = (kend - kbeg) > 0 ? (kend - kbeg) / BK : 0;
  [[maybe_unused]] ConvRowsKC<BM, NT> ga;
  [[maybe_unused]] ConvRowsDW<BN, NT> gb;
  if constexpr (G == G_FWD) ga.init_fwd(p.cv, m0, p.M, tid);
  if constexpr (G == G_DX) ga.init_dx(p.cv, m0, p.M, tid);
  // the epilogue's scatter rows (read after the main loop's barriers); rows past M clamped
  [[maybe_unused]] __shared__ int64_t dxrow[G == G_DX ? BM : 1];
  if constexpr (G == G_DX)
    for (int r = tid; r < BM; r += NT) dxrow[r] = dx_row(p.cv, min(m0 + r, p.M - 1));
  // EPI_AUX_RELU_W1: the conv1 patch x[b, 2 t1 + kh, 2 f1 + kw] of every tile row (dy1 position
  // (b, t1, f1)), loaded into registers here (in flight under the main loop) and staged for
  // dx_w1_epilogue
  constexpr bool W1 = G == G_DX && EPI == EPI_AUX_RELU_W1;
  constexpr int XN = W1 ? (9 * BM + NT - 1) / NT : 1;
  [[maybe_unused]] float xr[XN];
  if constexpr (W1) {
    const ConvG& g = p.cv;
    const int pt = g.cls >> 1, pf = g.cls & 1;
    const int nI = (g.T1 - pt + 1) >> 1, nJ = (g.F1 - pf + 1) >> 1;
#pragma unroll
    for (int i = 0; i < XN; ++i) {
      const int e = i * NT + tid, r = e / 9, k = e - 9 * r;
      xr[i] = 0.f;
      if (e < 9 * BM) {
        const int m = min(m0 + r, p.M - 1);
        const int j = m % nJ, t = m / nJ, ii = t % nI, b = t / nI;
        const int kh = k / 3, kw = k - 3 * kh;
        xr[i] = g.x[((int64_t)b * g.T0 + 2 * (2 * ii + pt) + kh) * g.F0 + 2 * (2 * j + pf) + kw];
      }
    }
  }
  if constexpr (G == G_DW) gb.init(p.cv, n0, p.N, kbeg, tid);
  // one 32-deep sub-tile at k0 into dst (the conv walkers keep per-position state: sub-tiles
  // are issued in k order)
  auto issue_sub = [&](const int k0, bf16_t* dst) {
    if (LASR_EXP & 4) return;
    if constexpr (G == G_LIN) {
      glds_tile<BM, AKC, NT>(A, lda, m0, p.M, k0, dst, tid);
      glds_tile<BN, BKC, NT>(B, ldb, n0, p.N, k0, dst + BM * BK, tid);
    } else if constexpr (G == G_FWD) {
      const int C = p.cv.C, tap = k0 / C, kh = tap / 3, kw = tap - 3 * kh;
      ga.issue(A, (int64_t)(kh * p.cv.F1 + kw) * C + (k0 - tap * C), dst, tid);
      glds_tile<BN, true, NT>(B, ldb, n0, p.N, k0, dst + BM * BK, tid);
    } else if constexpr (G == G_DW) {
      glds_tile<BM, false, NT>(A, lda, m0, p.M, k0, dst, tid);
      gb.issue(p.cv, B, dst + BM * BK, tid);
    } else {
      // class tap ti = k0 / C: (kh, kw) = (pt ? 1 : 2a, pf ? 1 : 2c), reading dy2 row (i-dt, j-df)
      const int C = p.cv.C, ti = k0 / C, cin = k0 - ti * C;
      const int pt = p.cv.cls >> 1, pf = p.cv.cls & 1, nkw = pf ? 1 : 2;
      const int a = ti / nkw, c = ti - a * nkw;
      const int dt = pt ? 0 : a, df = pf ? 0 : c;
      const int kh = pt ? 1 : 2 * a, kw = pf ? 1 : 2 * c;
      ga.issue_dx(A, cin - (int64_t)(dt * p.cv.F2 + df) * C, dt * 2 + df, p.cv.zero, dst, tid);
      glds_tile<BN, false, NT>(B + (kh * 3 + kw) * C, ldb, n0, p.N, cin, dst + BM * BK, tid);
    }
  };
  auto issue = [&](int t) {
    bf16_t* dst = smem + (t % S) * STAGE;
    const int k0 = kbeg + t * (KS * BK);
#pragma unroll
    for (int u = 0; u < KS; ++u) issue_sub(k0 + u * BK, dst + u * TILE);
  };
  // the transposed fragments' per-thread image offsets, computed once (a k step then adds
  // only the tile's uniform LDS base: one VALU per read instead of the recomputed address)
  [[maybe_unused]] uint32_t aoff[AKC ? 1 : FM][2], boff[BKC ? 1 : FN][2];
  if constexpr (!AKC)
#pragma unroll
    for (int i = 0; i < FM; ++i) frag_tr_offsets<BM>(wr * WM + i * 16, lane, aoff[i]);
  if constexpr (!BKC)
#pragma unroll
    for (int j = 0; j < FN; ++j) frag_tr_offsets<BN>(wc * WN + j * 16, lane, boff[j]);
  auto compute = [&](const bf16_t* cur) {
    bf16x8 af[FM], bfr[FN];
    v2i ra[2 * FM], rb[2 * FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (AKC) af[i] = frag<BM, true>(cur, wr * WM + i * 16, lane);
      else frag_tr_raw_at(lds_addr(cur), aoff[i], ra + 2 * i);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BKC) bfr[j] = frag<BN, true>(cur + BM * BK, wc * WN + j * 16, lane);
      else frag_tr_raw_at(lds_addr(cur + BM * BK), boff[j], rb + 2 * j);
    }
    if constexpr (!AKC) {
      tie_lgkm<2 * FM>(ra);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_from_raw(ra + 2 * i);
    }
    if constexpr (!BKC) {
      tie_lgkm<2 * FN>(rb);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_from_raw(rb + 2 * j);
    }
    if (LASR_EXP & 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[i][0][0] += (float)af[i][0] + (float)bfr[0][i & 1];
      return;
    }
    // swapped operands: acc[i][j] accumulates the C^T fragment (gemm_epilogue_direct)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

  // fused bias gradient (rowsum of A) on the n-tile-0 blocks; uniform per block
  const bool do_rs = !AKC && p.rowsum != nullptr && tx == 0;
  float rs[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) rs[q] = 0.f;

  const int nst = nfull / KS;  // full ring stages; KS > 1 leaves nfull % KS sub-tiles
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nst) issue(t);

  for (int kt = 0; kt < nst; ++kt) {
    const int after = min(S - 2, nst - 1 - kt);  // stages issued after kt (still in flight)
    wait_ring<S, GL * KS>(after);
    lds_barrier();
    if (kt + S - 1 < nst) issue(kt + S - 1);
#pragma unroll
    for (int u = 0; u < KS; ++u) compute(smem + (kt % S) * STAGE + u * TILE);
    if constexpr (!AKC)
      if (do_rs)
#pragma unroll
        for (int u = 0; u < KS; ++u) rowsum_tile<BM, NT>(smem + (kt % S) * STAGE + u * TILE, tid, rs);
  }
  if constexpr (KS > 1) {
    // leftover full sub-tile(s): the loop's last wait was vmcnt(0), so no DMA is in flight
    for (int j = nst * KS; j < nfull; ++j) {
      __syncthreads();
      issue_sub(kbeg + j * BK, smem);
      wait_vmcnt<0>();
      lds_barrier();
      compute(smem);
      if constexpr (!AKC)
        if (do_rs) rowsum_tile<BM, NT>(smem, tid, rs);
    }
  }
  if (G == G_LIN && nfull < nk) {  // ragged tail: register loader with zero fill (conv: host-checked K % 32 == 0)
    __syncthreads();
    TileLoader<BM, AKC, NT> la;
    TileLoader<BN, BKC, NT> lb;
    const int k0 = kbeg + nfull * BK;
    la.load(A, AKC ? p.lda_m : 0, AKC ? 0 : p.lda_k, m0, p.M, k0, kend, true, tid);
    lb.load(B, BKC ? p.ldb_n : 0, BKC ? 0 : p.ldb_k, n0, p.N, k0, kend, true, tid);
    la.store(smem, tid);
    lb.store(smem + BM * BK, tid);
    __syncthreads();
    compute(smem);
    if constexpr (!AKC)
      if (do_rs) rowsum_tile<BM, NT>(smem, tid, rs);
  }
  __syncthreads();
  if constexpr (!AKC) {
    if (do_rs) {  // combine the k groups in fixed order, then one slot per row
      constexpr int CH = BM / 8, KG = NT / CH;
      float* red = reinterpret_cast<float*>(smem_epi);
      const int c = tid % CH, kg = tid / CH;
#pragma unroll
      for (int q = 0; q < 8; ++q) red[kg * BM + 8 * c + q] = rs[q];
      __syncthreads();
      if (tid < BM) {
        float t = 0.f;
        for (int g = 0; g < KG; ++g) t += red[g * BM + tid];
        const int m = m0 + tid;
        if (m < p.M) {
          if (p.split_k > 1) p.rs_ws[(int64_t)s * p.M + m] = t;
          else p.rowsum[m] += t;
        }
      }
      __syncthreads();
    }
  }
  if constexpr (W1) {
    dx_w1_epilogue<BM, BN, NW>(p, acc, smem_epi, m0, n0, dxrow, xr);
    return;
  }
  // split-K partials: fp32, 16-B per lane straight from the accumulators; final outputs:
  // staged through LDS (full 256-B rows per wave store)
  if (p.split_k > 1) gemm_epilogue_direct<BM, BN, TC, NW>(p, acc, m0, n0, s, z, z1, z2);
  else gemm_epilogue<BM, BN, TC, true, G, NW, EPI>(p, acc, smem_epi, m0, n0, s, z, z1, z2, dxrow);
}

// Tile order of a weight-gradient GEMM (both operands [K, M] / [K, N] with K = rows): the
// tiles that share the LARGER operand's column strip get consecutive indices, so after the
// XCD remap they sit on one XCD and that strip is fetched from HBM once (the smaller operand
// is the one re-fetched per XCD).  M >= N: N-tiles fastest; N > M: M-tiles fastest.
LASR_DEV void dw_tile_order(int wg, int nx, int ny, bool n_major, int& tx, int& ty) {
  if (n_major) { tx = wg / ny; ty = wg % ny; }
  else { tx = wg % nx; ty = wg / nx; }
}

// NW = 8: 512-thread workgroups, waves 2 (rows) x 4 (columns) over the tile (the 256 x 256
// tiles of the large GEMMs: half the LDS-DMA ingest per MFMA of 128 x 256 at 4 waves).
// MINB = workgroups per CU; the launch bound's second operand is waves per SIMD.
template <int BM, int BN, bool AKC, bool BKC, typename TC, int S, int MINB = 3, int G = G_LIN, int KS = 1,
          int NW = 4, int EPI = EPI_RT>
__global__ __launch_bounds__(NW * 64, MINB * NW / 4) void gemm_bf16_glds_kernel(GemmP p) {
  const int nx = gridDim.x, ny = gridDim.y;
  const int wg = xcd_remap(blockIdx.y * nx + blockIdx.x, nx * ny);
  int tx, ty;
  dw_tile_order(wg, nx, ny, !AKC && !BKC && G == G_LIN && p.N > p.M, tx, ty);
  gemm_glds_tile<BM, BN, AKC, BKC, TC, S, G, KS, NW, EPI>(p, tx, ty, blockIdx.z);
}

// Grouped split-K weight-gradient GEMMs (partials only): up to LASR_DW_GROUP_MAX independent
// problems dW_i = A_i^T B_i (A [K, M] and B [K, N] row-major, i.e. both M/N-contiguous), each
// with its own split, in ONE launch.  Problem i owns the blocks [start[i], start[i+1]) (starts
// multiples of 8, so the XCD remap inside a problem stays exact), K-slice-major like the
// launch grid of the single-problem kernel; the tile code and the partial layout
// ([split][M][N] + [split][M] rowsum partials) are those of gemm_bf16_glds_kernel, so the
// partials are bit-identical to separate launches.
#define LASR_DW_GROUP_MAX 8
struct DwGroupP {
  int n;
  int start[LASR_DW_GROUP_MAX + 1];
  int M[LASR_DW_GROUP_MAX], N[LASR_DW_GROUP_MAX], K[LASR_DW_GROUP_MAX];
  int split[LASR_DW_GROUP_MAX], kchunk[LASR_DW_GROUP_MAX], v4[LASR_DW_GROUP_MAX];
  const void* A[LASR_DW_GROUP_MAX];
  const void* B[LASR_DW_GROUP_MAX];
  int64_t lda[LASR_DW_GROUP_MAX], ldb[LASR_DW_GROUP_MAX];
  float* ws[LASR_DW_GROUP_MAX];
  float* rs_ws[LASR_DW_GROUP_MAX];  // null: no fused bias rowsum
  int slice_xcd;                    // K slices tied to XCDs (gemm_dw_group_kernel)
  // direct problems (split 1): full-K tiles that write the weight gradient itself (C = beta C +
  // dY^T X, fp32) and add their bias rowsum into rowsum -- no partial slab, no reduction
  int direct[LASR_DW_GROUP_MAX];
  float* C[LASR_DW_GROUP_MAX];
  int64_t ldc[LASR_DW_GROUP_MAX];
  float beta[LASR_DW_GROUP_MAX];
  float* rowsum[LASR_DW_GROUP_MAX];
};

template <int BM, int BN, int S, int MINB, int NW = 4>
__global__ __launch_bounds__(NW * 64, MINB * NW / 4) void gemm_dw_group_kernel(DwGroupP g) {
  const int blk = blockIdx.x;
  int i = 0;
  for (int j = 1; j < g.n; ++j)
    if (blk >= g.start[j]) i = j;
  const int ntx = (g.N[i] + BN - 1) / BN, nty = (g.M[i] + BM - 1) / BM, ntile = ntx * nty;
  const int local = blk - g.start[i];
  if (local >= ntile * g.split[i]) return;  // alignment padding
  GemmP p = {};
  p.M = g.M[i]; p.N = g.N[i]; p.K = g.K[i]; p.batch = 1; p.batch_div = 1;
  p.A = g.A[i]; p.lda_m = 1; p.lda_k = g.lda[i];
  p.B = g.B[i]; p.ldb_n = 1; p.ldb_k = g.ldb[i];
  p.split_k = g.split[i]; p.kchunk = g.kchunk[i]; p.ws = g.ws[i]; p.v4 = g.v4[i];
  p.rowsum = g.rs_ws[i];  // only tested for null when split_k > 1: the partials go to rs_ws
  p.rs_ws = g.rs_ws[i];
  p.alpha = 1.f;
  if (g.direct[i]) {  // the lone split-1 launch's epilogue: beta C + acc, rowsum += (n-tile 0)
    p.C = g.C[i]; p.ldc = g.ldc[i]; p.beta = g.beta[i];
    p.rowsum = g.rowsum[i]; p.rs_ws = nullptr; p.ws = nullptr;
    p.c_vec = ((uintptr_t)p.C & 15) == 0 && p.ldc % 8 == 0;
    p.epi_mode = p.c_vec && p.beta == 0.f ? 0 : 2;
  }
  // Block -> (tile, K slice).  The hardware deals blocks to the 8 XCDs round-robin (block % 8;
  // problem ranges start at multiples of 8).  When the split divides 8 and the tiles divide
  // evenly, K slice s lives on XCDs [s * 8/split, (s+1) * 8/split) only, each of them taking
  // a run of consecutive tiles (consecutive tiles share the larger operand's strip): both
  // operands of a slice are then fetched by its own XCDs only, instead of the small operand
  // by all 8 L2s (dg.slice_xcd; LASR_DW_SLICE_XCD=0 keeps the old map).  Same tile body, same
  // k range per (tile, slice): the partials are bit-identical either way.
  int tile, slice;
  const int sp = g.split[i], per = 8 / (sp > 0 ? sp : 1);
  if (g.slice_xcd && 8 % sp == 0 && ntile % per == 0 && (ntile * sp) % 8 == 0) {
    const int x = local & 7, q = local >> 3, run = ntile / per;  // q < run by construction
    slice = x / per;
    tile = (x % per) * run + q;
  } else {
    tile = xcd_remap(local % ntile, ntile);
    slice = local / ntile;
  }
  int tx, ty;
  dw_tile_order(tile, ntx, nty, p.N > p.M, tx, ty);
  gemm_glds_tile<BM, BN, false, false, float, S, G_LIN, 2, NW>(p, tx, ty, slice);
}

// ============================ fp32 MFMA kernel ===================================
template <bool AKC, bool BKC, typename TC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmP p) {
  constexpr int BM = 64, BN = 64, BK = 16, LD = BK + 1;
  __shared__ float As[BM * LD], Bs[BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int zz = blockIdx.z;
  const int s = zz % p.split_k, z = zz / p.split_k;
  const int z1 = z / p.batch_div, z2 = z % p.batch_div;
  const float* A = (const float*)p.A + z1 * p.sa1 + z2 * p.sa2;
  const float* B = (const float*)p.B + z1 * p.sb1 + z2 * p.sb2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = s * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int k0 = kbeg; k0 < kend; k0 += BK) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * 256;
      int r, k;
      if (AKC) { r = e >> 4; k = e & 15; } else { r = e & 63; k = e >> 6; }
      const int gm = m0 + r, gk = k0 + k;
      As[r * LD + k] = (gm < p.M && gk < kend) ? A[(int64_t)gm * p.lda_m + (int64_t)gk * p.lda_k] : 0.f;
      if (BKC) { r = e >> 4; k = e & 15; } else { r = e & 63; k = e >> 6; }
      const int gn = n0 + r, gk2 = k0 + k;
      Bs[r * LD + k] = (gn < p.N && gk2 < kend) ? B[(int64_t)gn * p.ldb_n + (int64_t)gk2 * p.ldb_k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float af[2], bfv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[(wr * 32 + i * 16 + (lane & 15)) * LD + kk + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfv[j] = Bs[(wc * 32 + j * 16 + (lane & 15)) * LD + kk + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  const int rq = (lane >> 4) * 4, cl = lane & 15;
  if (p.split_k > 1) {
    float* ws = p.ws + ((int64_t)s * p.batch + z) * (int64_t)p.M * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wr * 32 + i * 16 + rq + e, n = n0 + wc * 32 + j * 16 + cl;
          if (m < p.M && n < p.N) ws[(int64_t)m * p.N + n] = acc[i][j][e];
        }
    return;
  }
  const float al = alpha_of(p);
  const uint32_t dkey = epi_key(p);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wr * 32 + i * 16 + rq + e, n = n0 + wc * 32 + j * 16 + cl;
        epi_store<TC>(p, dkey, z1, z2, z, m, n, acc[i][j][e], al);
      }
}

// Split-K reduction: sums the split partials in fixed order, then the epilogue.  The body
// takes its block index and block count, so a fused launch can run it on a block range
// (gemm_ln.hip: beside the positional-bias reduction).
template <typename TC>
LASR_DEV void splitk_reduce_body(const GemmP& p, int bx, int nbx) {
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t total = MN * p.batch;
  const float al = alpha_of(p);
  const uint32_t dkey = epi_key(p);
  if (p.v4) {
    // 4 consecutive columns per thread (N % 4 == 0): 16-B partial loads, 4 slices in
    // flight, summed in slice order
    const int64_t sstride = (int64_t)p.batch * MN;
    for (int64_t i4 = (int64_t)bx * 256 + threadIdx.x; i4 < total / 4; i4 += (int64_t)nbx * 256) {
      const int64_t i = i4 * 4;
      const int z = (int)(i / MN);
      const int64_t r = i - (int64_t)z * MN;
      const float* src = p.ws + (int64_t)z * MN + r;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      int sl = 0;
      for (; sl + 4 <= p.split_k; sl += 4) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const f32x4*)(src + (int64_t)(sl + u) * sstride);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += v[u][e];
      }
      for (; sl < p.split_k; ++sl) {
        const f32x4 v = *(const f32x4*)(src + (int64_t)sl * sstride);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += v[e];
      }
      const int m = (int)(r / p.N), n = (int)(r - (int64_t)m * p.N);
      epi_store4<TC, true>(p, dkey, z / p.batch_div, z % p.batch_div, z, m, n, 4, acc, al);
    }
  } else {
    for (int64_t i = (int64_t)bx * 256 + threadIdx.x; i < total; i += (int64_t)nbx * 256) {
      const int z = (int)(i / MN);
      const int64_t r = i - (int64_t)z * MN;
      float acc = 0.f;
      for (int s = 0; s < p.split_k; ++s) acc += p.ws[((int64_t)s * p.batch + z) * MN + r];
      const int m = (int)(r / p.N), n = (int)(r - (int64_t)m * p.N);
      epi_store<TC>(p, dkey, z / p.batch_div, z % p.batch_div, z, m, n, acc, al);
    }
  }
  if (p.rs_ws) {  // bias-gradient partials (batch == 1)
    for (int64_t m = (int64_t)bx * 256 + threadIdx.x; m < p.M; m += (int64_t)nbx * 256) {
      float acc = 0.f;
      for (int s = 0; s < p.split_k; ++s) acc += p.rs_ws[(int64_t)s * p.M + m];
      p.rowsum[m] += acc;
    }
  }
}
template <typename TC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmP p) {
  splitk_reduce_body<TC>(p, blockIdx.x, gridDim.x);
}


// Compile-time epilogue of the hot FFN GEMMs (gemm_kernel.h EPI_*), or EPI_RT.  Host-checked
// against exactly the parameters the specialised path assumes; LASR_EPI_SPEC=0 disables it.
static inline int epi_code(const GemmP& p) {
  static const int on = [] { const char* e = getenv("LASR_EPI_SPEC"); return e && e[0] ? atoi(e) : 1; }();
  // (N % 8 == 0: every 8-column vector of the specialised epilogues starts on an even element,
  // so their dropout draws take the pair-aligned path only)
  if (!on || p.split_k > 1 || p.beta != 0.f || p.alpha_dev || p.N % 8 != 0) return EPI_RT;
  if (p.res) {
    return !p.zout && p.act == LASR_ACT_NONE && !p.aux && p.drop.p > 0.f && p.epi_mode == 1 ? EPI_RES_DROP : EPI_RT;
  }
  if (!p.zout && p.act == LASR_ACT_NONE && !p.aux && p.drop.p <= 0.f && p.epi_mode == 0) return EPI_PLAIN;
  if (!p.zout && p.act == LASR_ACT_RELU && !p.aux && p.drop.p <= 0.f && p.epi_mode == 0) return EPI_RELU;
  if (!p.zout && p.act == LASR_ACT_NONE && p.aux && p.aux_act == LASR_ACT_RELU && p.drop.p <= 0.f && p.epi_mode == 1)
    return EPI_AUX_RELU;
  if (p.zout && p.zout_mode == 1 && p.act == LASR_ACT_SWISH && p.drop.p > 0.f && !p.aux && p.epi_mode == 0)
    return EPI_SWISH_GATE_DROP;
  if (p.zout && p.zout_mode == 1 && p.act == LASR_ACT_RELU && p.drop.p > 0.f && !p.aux && p.epi_mode == 0)
    return EPI_RELU_GATE_DROP;
  if (!p.zout && p.act == LASR_ACT_NONE && p.aux && p.aux_act == LASR_ACT_GATE && p.drop.p <= 0.f && p.epi_mode == 1)
    return EPI_AUX_GATE;
  return EPI_RT;
}

static inline bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }
