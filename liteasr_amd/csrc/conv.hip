// Convolutions of the U2 encoder, channels-last.
//  * Conv2d subsampling (liteasr/nets/subsampling.py:31-47): conv1 (1->C, 3x3, s2)+ReLU
//    as a direct kernel; conv2 (C->C, 3x3, s2) as im2col + lasr_gemm (K = 9C), with the
//    col2im backward fusing relu'(conv1 out).
//  * Conformer convolution module (liteasr/nets/conformer_convolution.py:44-57):
//    GLU -> depthwise conv (K=15, "same" padding, no padding mask, exactly like the
//    reference) -> BatchNorm1d(train: batch stats over B*T incl. padding) -> Swish.
//    pw1/pw2 are lasr_gemm calls around these kernels.
#include "common.h"

// ----------------------------- conv1 -----------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ x, int T_, int F,
                                                        int C, int T1, int F1, const float* w,
                                                        const float* bias, T* y1) {
  extern __shared__ float sh[];
  float* xs = sh;           // 3 rows x F
  float* ws = sh + 3 * F;   // C x 10 (9 taps + bias)
  const int bt = blockIdx.x;
  const int b = bt / T1, t1 = bt - b * T1;
  for (int i = threadIdx.x; i < 3 * F; i += blockDim.x) {
    const int kh = i / F, f = i - kh * F;
    xs[i] = x[((int64_t)b * T_ + 2 * t1 + kh) * F + f];
  }
  for (int i = threadIdx.x; i < C * 9; i += blockDim.x) ws[(i / 9) * 10 + (i % 9)] = w[i];
  for (int c = threadIdx.x; c < C; c += blockDim.x) ws[c * 10 + 9] = bias[c];
  __syncthreads();
  T* out = y1 + (int64_t)bt * F1 * C;
  for (int e = threadIdx.x; e < F1 * C; e += blockDim.x) {
    const int f1 = e / C, c = e - f1 * C;
    const float* wc = ws + c * 10;
    float acc = wc[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) acc = fmaf(wc[kh * 3 + kw], xs[kh * F + 2 * f1 + kw], acc);
    out[e] = from_f<T>(fmaxf(acc, 0.f));
  }
}

constexpr int C1B_ROWS = 16;  // (b,t1) rows per conv1-bwd block
template <typename T>
__global__ __launch_bounds__(256) void conv1_bwd_kernel(const float* __restrict__ x, int T_, int F,
                                                        int C, int T1, int F1, int nrows,
                                                        const T* __restrict__ dy1, float* part) {
  extern __shared__ float xs[];  // C1B_ROWS x 3 x F input rows
  const int r0 = blockIdx.x * C1B_ROWS;
  const int nr = min(C1B_ROWS, nrows - r0);
  for (int i = threadIdx.x; i < nr * 3 * F; i += blockDim.x) {
    const int rr = i / (3 * F), q = i - rr * 3 * F;
    const int kh = q / F, f = q - kh * F;
    const int r = r0 + rr;
    const int b = r / T1, t1 = r - b * T1;
    xs[i] = x[((int64_t)b * T_ + 2 * t1 + kh) * F + f];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] = 0.f;
    for (int rr = 0; rr < nr; ++rr) {
      const float* xr = xs + rr * 3 * F;
      const T* d = dy1 + (int64_t)(r0 + rr) * F1 * C + c;
      for (int f1 = 0; f1 < F1; ++f1) {
        const float g = to_f(d[(int64_t)f1 * C]);
        acc[9] += g;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] += g * xr[kh * F + 2 * f1 + kw];
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) part[((int64_t)blockIdx.x * 10 + k) * C + c] = acc[k];
  }
}
__global__ void conv1_bwd_reduce_kernel(const float* part, int nparts, int C, float* dw,
                                        float* db) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // e = c*10 + k
  if (e >= C * 10) return;
  const int c = e / 10, k = e - c * 10;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[((int64_t)p * 10 + k) * C + c];
  if (k < 9) dw[c * 9 + k] += s;
  else db[c] += s;
}

// Vectorised conv1 (C % 8 == 0, 256 % (C/8) == 0): a thread owns 8 consecutive channels
// (their 8x10 weights in registers) and a strided set of output columns f1, so every
// y1 / dy1 access is one 16-B (bf16) vector and a wave covers whole 512-B channel rows.
// Same per-output arithmetic as the scalar kernels above: bias, then one fused multiply-add
// per tap in tap order (spelled fmaf: left to the compiler, the vectorised kernel got a packed
// multiply and a separate add per tap, 2.7x the VALU of packed FMAs in a VALU-bound kernel).
constexpr int C1V_ROWS = 32;  // largest (b,t1) row count per vectorised conv1-bwd block (A/B)
constexpr int C1F_ROWS = 8;   // (b,t1) rows per vectorised conv1-fwd block

typedef float c1_f2 __attribute__((ext_vector_type(2)));
template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_v8_kernel(const float* __restrict__ x, int T_, int F,
                                                           int C, int T1, int F1, int nrows, const float* w,
                                                           const float* bias, T* y1, int rpb) {
  // C1F_ROWS output rows (b, t1) per block: the 72 weights and 8 biases a thread keeps in
  // registers are loaded once per block, not once per row; the 3 input rows of each output
  // row are staged in LDS.  Each output: bias + sum over the 9 taps in order, then ReLU.
  extern __shared__ float xs[];  // rpb x 3F
  const int r0 = blockIdx.x * rpb;
  const int nr = min(rpb, nrows - r0);
  // the 3 input rows of output row (b, t1) are input rows 2 t1 .. 2 t1 + 2: 3F contiguous
  // floats.  With 16-B rows and 8 output rows per block, 32 threads copy a row's 3F/4
  // vectors, all of a thread's loads in flight before its LDS writes.
  if (rpb == 8 && (F & 3) == 0 && 3 * F <= 4 * 32 * 4 && (((uintptr_t)x) & 15) == 0) {
    const int rr = threadIdx.x >> 5, l = threadIdx.x & 31, n4 = 3 * F / 4;
    if (rr < nr) {
      const int r = r0 + rr, b = r / T1, t1 = r - b * T1;
      const float4* src = (const float4*)(x + ((int64_t)b * T_ + 2 * t1) * F);
      float4* dst = (float4*)(xs + rr * 3 * F);
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (l + 32 * k < n4) v[k] = src[l + 32 * k];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (l + 32 * k < n4) dst[l + 32 * k] = v[k];
    }
  } else {
    for (int i = threadIdx.x; i < nr * 3 * F; i += 256) {
      const int rr = i / (3 * F), q = i - rr * 3 * F;
      const int r = r0 + rr;
      const int b = r / T1, t1 = r - b * T1;
      xs[i] = x[((int64_t)b * T_ + 2 * t1) * F + q];
    }
  }
  const int CG = C >> 3, cg = threadIdx.x % CG, fg = threadIdx.x / CG, NFG = 256 / CG;
  const int c0 = cg * 8;
  float wr[8][9], bv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bv[q] = bias[c0 + q];
#pragma unroll
    for (int k = 0; k < 9; ++k) wr[q][k] = w[(c0 + q) * 9 + k];
  }
  __syncthreads();
  for (int rr = 0; rr < nr; ++rr) {
    const float* xr = xs + rr * 3 * F;
    T* out = y1 + (int64_t)(r0 + rr) * F1 * C + c0;
    for (int f1 = fg; f1 < F1; f1 += NFG) {
      float xv[9];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xr[kh * F + 2 * f1 + kw];
      // channel pairs as 2-wide vectors: one v_pk_fma_f32 per tap and pair (the same fused
      // multiply-add per channel as fmaf)
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        c1_f2 acc = {bv[q], bv[q + 1]};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const c1_f2 wk = {wr[q][k], wr[q + 1][k]}, xk = {xv[k], xv[k]};
          acc = __builtin_elementwise_fma(wk, xk, acc);
        }
        o[q] = fmaxf(acc[0], 0.f);
        o[q + 1] = fmaxf(acc[1], 0.f);
      }
      st8(out + (int64_t)f1 * C, o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void conv1_bwd_v8_kernel(const float* __restrict__ x, int T_, int F,
                                                           int C, int T1, int F1, int nrows,
                                                           const T* __restrict__ dy1, float* part, int rpb) {
  extern __shared__ float sh[];  // rpb x 3F input rows, then the 8*256 reduce slab
  float* xs = sh;
  float* red = sh + rpb * 3 * F;
  const int r0 = blockIdx.x * rpb;
  const int nr = min(rpb, nrows - r0);
  for (int i = threadIdx.x; i < nr * 3 * F; i += 256) {
    const int rr = i / (3 * F), q = i - rr * 3 * F;
    const int r = r0 + rr;
    const int b = r / T1, t1 = r - b * T1;
    xs[i] = x[((int64_t)b * T_ + 2 * t1) * F + q];
  }
  __syncthreads();
  const int CG = C >> 3, cg = threadIdx.x % CG, fg = threadIdx.x / CG, NFG = 256 / CG;
  const int c0 = cg * 8;
  float acc[8][10];
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[q][k] = 0.f;
  for (int rr = 0; rr < nr; ++rr) {
    const float* xr = xs + rr * 3 * F;
    const T* d = dy1 + (int64_t)(r0 + rr) * F1 * C + c0;
    for (int f1 = fg; f1 < F1; f1 += NFG) {
      float g[8], xv[9];
      ld8(d + (int64_t)f1 * C, g);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xr[kh * F + 2 * f1 + kw];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[q][9] += g[q];
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[q][k] += g[q] * xv[k];
      }
    }
  }
  // combine the NFG column groups in fixed order, one tap at a time (8 KB slab)
#pragma unroll
  for (int k = 0; k < 10; ++k) {
#pragma unroll
    for (int q = 0; q < 8; ++q) red[fg * C + c0 + q] = acc[q][k];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float t = 0.f;
      for (int g2 = 0; g2 < NFG; ++g2) t += red[g2 * C + c];
      part[((int64_t)blockIdx.x * 10 + k) * C + c] = t;
    }
    __syncthreads();
  }
}

// ----------------------------- im2col / col2im ----------------------------------------
template <typename T>
__global__ void im2col_kernel(const T* __restrict__ y1, int B, int T1, int F1, int C, int T2,
                              int F2, T* col) {
  const int64_t n8 = (int64_t)B * T2 * F2 * 9 * C / 8;  // C % 8 == 0
  // 32-bit index arithmetic (host-checked: B*T2*F2*9*C < 2^31): the 64-bit divisions
  // otherwise dominate this copy
  const uint32_t KC = 9u * (uint32_t)C, P2 = (uint32_t)(T2 * F2);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t el = (uint32_t)e * 8u;
    const uint32_t m = el / KC;
    const uint32_t k = el - m * KC;
    const uint32_t tap = k / (uint32_t)C, cin = k - tap * (uint32_t)C;
    const uint32_t kh = tap / 3u, kw = tap - kh * 3u;
    const uint32_t b = m / P2;
    const uint32_t rem = m - b * P2;
    const uint32_t t2 = rem / (uint32_t)F2, f2 = rem - t2 * (uint32_t)F2;
    const T* src = y1 + ((int64_t)((b * T1 + 2 * t2 + kh) * F1 + 2 * f2 + kw)) * C + cin;
    if (sizeof(T) == 2) *(uint4*)(col + el) = *(const uint4*)src;
    else {
      *(float4*)(col + el) = *(const float4*)src;
      *(float4*)(col + el + 4) = *(const float4*)(src + 4);
    }
  }
}
template <typename T>
__global__ void col2im_kernel(const T* __restrict__ dcol, int B, int T1, int F1, int C, int T2,
                              int F2, const T* __restrict__ y1, T* dy1) {
  // 8 channels per thread (C % 8 == 0): 16-B loads/stores along cin
  const int C8 = C / 8;
  const int64_t n = (int64_t)B * T1 * F1 * C8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    // 32-bit index arithmetic (host-checked: B*T1*F1*C/8 < 2^31)
    const uint32_t e32 = (uint32_t)e, pix32 = e32 / (uint32_t)C8;
    const int cin = (int)(e32 - pix32 * (uint32_t)C8) * 8;
    const int64_t pix = pix32;
    const uint32_t bt = pix32 / (uint32_t)F1;
    const int fi = (int)(pix32 - bt * (uint32_t)F1);
    const uint32_t b32 = bt / (uint32_t)T1;
    const int ti = (int)(bt - b32 * (uint32_t)T1);
    const int64_t b = b32;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, t[8], yv[8];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int tt = ti - kh;
      if (tt < 0 || (tt & 1)) continue;
      const int t2 = tt >> 1;
      if (t2 >= T2) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ff = fi - kw;
        if (ff < 0 || (ff & 1)) continue;
        const int f2 = ff >> 1;
        if (f2 >= F2) continue;
        const int64_t m = (b * T2 + t2) * F2 + f2;
        ld8(dcol + m * 9 * C + (kh * 3 + kw) * C + cin, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += t[j];
      }
    }
    ld8(y1 + pix * C + cin, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = yv[j] > 0.f ? s[j] : 0.f;
    st8(dy1 + pix * C + cin, s);
  }
}

// ----------------------------- permute_last2 --------------------------------------
template <typename TS, typename TD>
__global__ void permute_last2_kernel(const TS* src, int64_t N, int64_t A, int64_t Bd, TD* dst,
                                     int reverse, int acc) {
  const int64_t n = N * A * Bd;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    // e indexes the [N][A][Bd] ("reference") layout
    const int64_t i = e / (A * Bd);
    const int64_t r = e - i * A * Bd;
    const int64_t a = r / Bd, bb = r - a * Bd;
    const int64_t e2 = i * A * Bd + bb * A + a;  // [N][Bd][A]
    if (!reverse) dst[e2] = from_f<TD>(to_f(src[e]));
    else {
      float v = to_f(src[e2]);
      if (acc) v += to_f(dst[e]);
      dst[e] = from_f<TD>(v);
    }
  }
}

// ------------------------ GLU + depthwise conv (K = 15) ----------------------------
constexpr int DW_TT = 32;   // time rows per block
constexpr int DW_K = 15;
constexpr int DW_P = (DW_K - 1) / 2;
constexpr int DW_WIN = DW_TT + 2 * DW_P;

// Thread layout of the GLU/depthwise kernels: DW_NT = 256 threads = DW_G time groups of DW_R rows
// x 64 channel pairs (128 channels, 2 per thread with 4-B / 8-B loads); a block covers
// DW_TT = DW_G * DW_R rows, its per-channel partials are combined across the groups in LDS
// in a fixed order (one partial per block, as lasr_dwconv_nparts counts them).
constexpr int DW_G = 4, DW_R = DW_TT / DW_G, DW_CP = 64;
constexpr int DW_NT = DW_G * DW_CP;  // threads per block
constexpr int DW_RW = DW_R + 2 * DW_P;  // rows a thread reads (window + halo)


// A window of DW_WIN rows (from tb - DW_P) x the block's 128 channels into LDS as channel
// pairs: src rows of stride ld (elements), channels from col0; f(row pointer, channel, v[2])
// turns two source values into the stored pair.  vec (C % 8 == 0, 16-B aligned rows): 8
// channels per access and every load of the thread issued before the first LDS store -- the
// window load is the latency these kernels wait on (two blocks per CU).
template <typename T>
LASR_DEV float2 glu2(const T* zr, int C, int c) {  // a * sigmoid(gate) for channels c, c+1
  float a[2], gt[2];
  ldv<2>(zr + c, a);
  ldv<2>(zr + C + c, gt);
  return make_float2(a[0] * sigmoidf_(gt[0]), a[1] * sigmoidf_(gt[1]));
}

template <int CP, typename TS, typename F>
LASR_DEV void dw_window(const TS* src, int64_t ld, int col0, int b, int T_, int C, int tb, bool vec,
                        float2 (*win)[CP], F f) {
  if (vec) {
    constexpr int CH = CP / 4, NE = DW_WIN * CH, IT = (NE + DW_NT - 1) / DW_NT;
    float v[IT][8], u[IT][8];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      const int e = threadIdx.x + DW_NT * j;
      const int rr = e / CH, q = e % CH, t = tb - DW_P + rr, ce = blockIdx.y * 2 * CP + q * 8;
      if (e < NE && ce < C && t >= 0 && t < T_) {
        f.load8(src + ((int64_t)b * T_ + t) * ld + col0, ce, v[j], u[j]);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[j][k] = u[j][k] = 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      const int e = threadIdx.x + DW_NT * j;
      if (e >= NE) continue;
      const int rr = e / CH, q = e % CH;
#pragma unroll
      for (int k = 0; k < 4; ++k) win[rr][q * 4 + k] = f.pair(v[j] + 2 * k, u[j] + 2 * k);
    }
    return;
  }
  for (int e = threadIdx.x; e < DW_WIN * CP; e += DW_NT) {
    const int rr = e / CP, cq = e % CP, t = tb - DW_P + rr, ce = (blockIdx.y * CP + cq) * 2;
    float2 r = make_float2(0.f, 0.f);
    if (ce < C && t >= 0 && t < T_) {
      float v[2], u[2];
      f.load2(src + ((int64_t)b * T_ + t) * ld + col0, ce, v, u);
      r = f.pair(v, u);
    }
    win[rr][cq] = r;
  }
}

// GLU of z1 rows [a | gate] (2C wide): the pair a * sigmoid(gate), glu2's arithmetic
template <typename T>
struct GluWin {
  int C;
  LASR_DEV void load8(const T* row, int ce, float* a, float* g) const { ldv<8>(row + ce, a); ldv<8>(row + C + ce, g); }
  LASR_DEV void load2(const T* row, int ce, float* a, float* g) const { ldv<2>(row + ce, a); ldv<2>(row + C + ce, g); }
  LASR_DEV float2 pair(const float* a, const float* g) const {
    return make_float2(a[0] * sigmoidf_(g[0]), a[1] * sigmoidf_(g[1]));
  }
};

template <typename T, typename TY>
__global__ __launch_bounds__(DW_NT) void glu_dwconv_fwd_kernel(const T* __restrict__ z1, int T_,
                                                             int C, const float* w,
                                                             const float* bias, TY* y,
                                                             float* stats, int vec) {
  __shared__ float sst[DW_G][3][2 * DW_CP];
  const int cp = threadIdx.x % DW_CP, grp = threadIdx.x / DW_CP;
  const int c = (blockIdx.y * DW_CP + cp) * 2;
  const int nchunk = (T_ + DW_TT - 1) / DW_TT;
  const int b = blockIdx.x / nchunk, t0 = (blockIdx.x - b * nchunk) * DW_TT + grp * DW_R;
  const bool live = c < C;
  // the block's GLU window (DW_TT + halo rows x 128 channels), each row computed once
  __shared__ float2 win[DW_WIN][DW_CP];
  const int tb = t0 - grp * DW_R;
  dw_window<DW_CP>(z1, 2 * (int64_t)C, 0, b, T_, C, tb, vec != 0, win, GluWin<T>{C});
  __syncthreads();
  float2 g[DW_RW];
#pragma unroll
  for (int i = 0; i < DW_RW; ++i) g[i] = win[grp * DW_R + i][cp];
  float cnt = 0.f, mean[2] = {0.f, 0.f}, m2[2] = {0.f, 0.f};
  if (live) {
    float w0[DW_K], w1[DW_K];
#pragma unroll
    for (int k = 0; k < DW_K; ++k) { w0[k] = w[c * DW_K + k]; w1[k] = w[(c + 1) * DW_K + k]; }
    const float b0 = bias[c], b1 = bias[c + 1];
#pragma unroll
    for (int i = 0; i < DW_R; ++i) {
      const int t = t0 + i;
      if (t < T_) {
        float acc[2] = {b0, b1};
#pragma unroll
        for (int k = 0; k < DW_K; ++k) {
          acc[0] += w0[k] * g[i + k].x;
          acc[1] += w1[k] * g[i + k].y;
        }
        TY* yr = y + ((int64_t)b * T_ + t) * C + c;
        stv<2>(yr, acc);
        cnt += 1.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float yv = to_f(from_f<TY>(acc[q]));  // stats on the stored value
          const float dlt = yv - mean[q];
          mean[q] += dlt / cnt;
          m2[q] += dlt * (yv - mean[q]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    sst[grp][0][2 * cp + q] = cnt;
    sst[grp][1][2 * cp + q] = mean[q];
    sst[grp][2][2 * cp + q] = m2[q];
  }
  __syncthreads();
  if (threadIdx.x >= 2 * DW_CP) return;
  const int cl = threadIdx.x, cc = blockIdx.y * 2 * DW_CP + cl;
  if (cc >= C) return;
  // Chan et al. pairwise combine of the time groups, fixed order
  float n = sst[0][0][cl], mu = sst[0][1][cl], M2 = sst[0][2][cl];
#pragma unroll
  for (int k = 1; k < DW_G; ++k) {
    const float nb = sst[k][0][cl];
    if (nb == 0.f) continue;
    const float nt = n + nb, dl = sst[k][1][cl] - mu;
    mu += dl * (nb / nt);
    M2 += sst[k][2][cl] + dl * dl * (n * nb / nt);
    n = nt;
  }
  float* st = stats + (int64_t)blockIdx.x * 3 * C;
  st[cc] = n;
  st[C + cc] = mu;
  st[2 * C + cc] = M2;
}

// the dy window: 8 values per access, stored as channel pairs (dw_window's pairing)
template <typename TD>
struct DyWin {
  LASR_DEV void load8(const TD* row, int ce, float* v, float* u) const {
    ldv<8>(row + ce, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = 0.f;
  }
  LASR_DEV void load2(const TD* row, int ce, float* v, float* u) const {
    ldv<2>(row + ce, v);
    u[0] = u[1] = 0.f;
  }
  LASR_DEV float2 pair(const float* v, const float*) const { return make_float2(v[0], v[1]); }
  LASR_DEV void finish(int) const {}
};

// Backward of y = dwconv(GLU(z1)) over the block's DW_TT rows x 128 channels: dW / db partials
// (dy x the GLU window), dg = the transposed conv of dy, dz1 = GLU'(z1) dg.  The two windows
// (GLU recomputed, dy) come in with 8-channel loads (dw_window); dg is staged through LDS so
// the z1 re-read and the dz1 stores are 16-B row vectors (8 channels of a and of the gate).
// DYW: how the dy window is read -- DyWin (a stored dy) or BnDyWin (dy computed from the
// BatchNorm + activation backward's inputs as the window is loaded, no stored dy)
template <typename T, typename TD, typename DYW = DyWin<TD>>
__global__ __launch_bounds__(DW_NT) void glu_dwconv_bwd_kernel(const T* __restrict__ z1,
                                                             const TD* __restrict__ dy, int T_,
                                                             int C, const float* w, T* dz1,
                                                             float* part, int vec, DYW fdy = DYW{}) {
  fdy.finish(C);
  __shared__ float sp[DW_G][DW_K + 1][2 * DW_CP];
  const int cp = threadIdx.x % DW_CP, grp = threadIdx.x / DW_CP;
  const int c = (blockIdx.y * DW_CP + cp) * 2;
  const int nchunk = (T_ + DW_TT - 1) / DW_TT;
  const int b = blockIdx.x / nchunk, t0 = (blockIdx.x - b * nchunk) * DW_TT + grp * DW_R;
  const bool live = c < C;
  // the block's GLU and dy windows (DW_TT + halo rows x 128 channels), loaded once
  __shared__ float2 wg[DW_WIN][DW_CP], wd[DW_WIN][DW_CP];
  const int tb = t0 - grp * DW_R;
  dw_window<DW_CP>(z1, 2 * (int64_t)C, 0, b, T_, C, tb, vec != 0, wg, GluWin<T>{C});
  dw_window<DW_CP>(dy, (int64_t)C, 0, b, T_, C, tb, vec != 0, wd, fdy);
  __syncthreads();
  float2 g[DW_RW], d[DW_RW];
#pragma unroll
  for (int i = 0; i < DW_RW; ++i) {
    g[i] = wg[grp * DW_R + i][cp];
    d[i] = wd[grp * DW_R + i][cp];
  }
  __syncthreads();  // wd is reused below as the dg tile
  float* dgs = reinterpret_cast<float*>(&wd[0][0]);  // [DW_TT][2 * DW_CP] fp32
  float dw0[DW_K], dw1[DW_K], db0 = 0.f, db1 = 0.f;
#pragma unroll
  for (int k = 0; k < DW_K; ++k) { dw0[k] = 0.f; dw1[k] = 0.f; }
  if (live) {
    float w0[DW_K], w1[DW_K];
#pragma unroll
    for (int k = 0; k < DW_K; ++k) { w0[k] = w[c * DW_K + k]; w1[k] = w[(c + 1) * DW_K + k]; }
#pragma unroll
    for (int i = 0; i < DW_R; ++i) {
      const int t = t0 + i;
      if (t < T_) {
        const float2 dyt = d[i + DW_P];
        db0 += dyt.x;
        db1 += dyt.y;
        float dg0 = 0.f, dg1 = 0.f;
#pragma unroll
        for (int k = 0; k < DW_K; ++k) {
          dw0[k] += dyt.x * g[i + k].x;
          dw1[k] += dyt.y * g[i + k].y;
          // dg[t] = sum_k w[k] * dy[t - k + P]
          dg0 += w0[k] * d[i + 2 * DW_P - k].x;
          dg1 += w1[k] * d[i + 2 * DW_P - k].y;
        }
        *(float2*)(dgs + (grp * DW_R + i) * 2 * DW_CP + 2 * cp) = make_float2(dg0, dg1);
      }
    }
  }
  __syncthreads();
  // dz1 = [dg * s | dg * a * s * (1 - s)], 8 channels per item: DW_TT rows x 16 channel octets
  {
    constexpr int OCT = 2 * DW_CP / 8;
    for (int e = threadIdx.x; e < DW_TT * OCT; e += DW_NT) {
      const int rr = e / OCT, q = e % OCT, t = tb + rr, ce = blockIdx.y * 2 * DW_CP + q * 8;
      if (t >= T_ || ce >= C) continue;
      const int64_t r = (int64_t)b * T_ + t;
      const float* dgr = dgs + rr * 2 * DW_CP + q * 8;
      if (vec) {
        float a[8], gt[8], da[8], dgt[8];
        ldv<8>(z1 + r * 2 * C + ce, a);
        ldv<8>(z1 + r * 2 * C + C + ce, gt);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float s = sigmoidf_(gt[k]), dg = dgr[k];
          da[k] = dg * s;
          dgt[k] = dg * a[k] * s * (1.f - s);
        }
        stv<8>(dz1 + r * 2 * C + ce, da);
        stv<8>(dz1 + r * 2 * C + C + ce, dgt);
      } else {
        for (int k = 0; k < 8 && ce + k < C; k += 2) {
          float a[2], gt[2];
          ldv<2>(z1 + r * 2 * C + ce + k, a);
          ldv<2>(z1 + r * 2 * C + C + ce + k, gt);
          const float s0 = sigmoidf_(gt[0]), s1 = sigmoidf_(gt[1]);
          const float da[2] = {dgr[k] * s0, dgr[k + 1] * s1};
          const float dgt[2] = {dgr[k] * a[0] * s0 * (1.f - s0), dgr[k + 1] * a[1] * s1 * (1.f - s1)};
          stv<2>(dz1 + r * 2 * C + ce + k, da);
          stv<2>(dz1 + r * 2 * C + C + ce + k, dgt);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < DW_K; ++k) {
    sp[grp][k][2 * cp] = dw0[k];
    sp[grp][k][2 * cp + 1] = dw1[k];
  }
  sp[grp][DW_K][2 * cp] = db0;
  sp[grp][DW_K][2 * cp + 1] = db1;
  __syncthreads();
  // partial row of this block in the parameters' own layout: [C][K] weight taps, then [C]
  // bias, so the reduction writes dw / db directly (or is deferred as one segment)
  float* pp = part + (int64_t)blockIdx.x * (DW_K + 1) * C;
  for (int e = threadIdx.x; e < (DW_K + 1) * 2 * DW_CP; e += DW_NT) {
    const int cl = e / (DW_K + 1), k = e % (DW_K + 1);
    const int cg = blockIdx.y * 2 * DW_CP + cl;
    if (cg >= C) continue;
    float v = sp[0][k][cl];
#pragma unroll
    for (int q = 1; q < DW_G; ++q) v += sp[q][k][cl];
    pp[k < DW_K ? (int64_t)cg * DW_K + k : (int64_t)DW_K * C + cg] = v;
  }
}

// Channel c's outputs from the combined statistics (explicit fmaf / products: the roundings do
// not depend on what hipcc contracts).
LASR_DEV void bn_final_write(int c, double n, double mu, double m2, float eps, float momentum, const float* gamma,
                             const float* beta, float* rmean, float* rvar, float* mean, float* rstd, float* scale,
                             float* shift, int update) {
  const float var = (float)(m2 / n);
  const float rs = rsqrtf(var + eps);
  mean[c] = (float)mu;
  rstd[c] = rs;
  const float sc = __fmul_rn(gamma[c], rs);
  scale[c] = sc;
  shift[c] = fmaf(-(float)mu, sc, beta[c]);
  if (update == 1) {
    const float uvar = n > 1.0 ? (float)(m2 / (n - 1.0)) : var;
    rmean[c] = fmaf(momentum, (float)mu, __fmul_rn(1.f - momentum, rmean[c]));
    rvar[c] = fmaf(momentum, uvar, __fmul_rn(1.f - momentum, rvar[c]));
  }
}

// ------------------------------- BatchNorm ---------------------------------------
// 1024 threads = BNF_C channels x BNF_G partial-groups, combined in double by a fixed
// pairwise tree, then one thread per channel finalises.
constexpr int BNF_C = 16, BNF_G = 1024 / BNF_C;
__global__ __launch_bounds__(1024) void bn_finalize_par_kernel(
    const float* stats, int nparts, int C, float eps, float momentum, const float* gamma,
    const float* beta, float* rmean, float* rvar, int64_t* nbt, float* mean, float* rstd,
    float* scale, float* shift, int update) {
  __shared__ double sn[BNF_G][BNF_C + 1], smu[BNF_G][BNF_C + 1], sm2[BNF_G][BNF_C + 1];
  const int tx = threadIdx.x % BNF_C, ty = threadIdx.x / BNF_C;
  const int c = blockIdx.x * BNF_C + tx;
  if (blockIdx.x == 0 && threadIdx.x == 0 && update == 1 && nbt) nbt[0] += 1;
  if (update == 2) {  // eval mode: normalise with the running statistics
    if (ty == 0 && c < C) {
      const float rs = rsqrtf(rvar[c] + eps);
      mean[c] = rmean[c];
      rstd[c] = rs;
      const float sc = __fmul_rn(gamma[c], rs);
      scale[c] = sc;
      shift[c] = fmaf(-rmean[c], sc, beta[c]);
    }
    return;
  }
  // two-pass exact combine in double: (N, sum n_b mu_b) -> mu; then
  // M2 = sum_b [m2_b + n_b (mu_b - mu)^2]; fixed partial order, no per-partial division.
  double n = 0.0, s = 0.0;
  if (c < C)
    for (int p = ty; p < nparts; p += BNF_G) {
      const float* st = stats + (int64_t)p * 3 * C;
      const double nb = st[c];
      n += nb;
      s += nb * (double)st[C + c];
    }
  sn[ty][tx] = n;
  smu[ty][tx] = s;
  __syncthreads();
  // fixed pairwise tree over the partial groups (6 LDS steps instead of a 64-long chain)
  for (int w = BNF_G / 2; w >= 1; w >>= 1) {
    if (ty < w) {
      sn[ty][tx] += sn[ty + w][tx];
      smu[ty][tx] += smu[ty + w][tx];
    }
    __syncthreads();
  }
  n = sn[0][tx];
  s = smu[0][tx];
  const double mu = n > 0.0 ? s / n : 0.0;
  double m2 = 0.0;
  if (c < C)
    for (int p = ty; p < nparts; p += BNF_G) {
      const float* st = stats + (int64_t)p * 3 * C;
      const double nb = st[c], dl = (double)st[C + c] - mu;
      m2 += (double)st[2 * C + c] + nb * dl * dl;
    }
  sm2[ty][tx] = m2;
  __syncthreads();
  for (int w = BNF_G / 2; w >= 1; w >>= 1) {
    if (ty < w) sm2[ty][tx] += sm2[ty + w][tx];
    __syncthreads();
  }
  if (ty != 0 || c >= C) return;
  m2 = sm2[0][tx];
  bn_final_write(c, n, mu, m2, eps, momentum, gamma, beta, rmean, rvar, mean, rstd, scale, shift, update);
}

// The conv module's activation after the BatchNorm (conformer_convolution.py:56): Swish
// (the default) or ReLU (encoder activation "relu", transformer_encoder.py:77-80).
template <bool RELU>
LASR_DEV float bn_act(float u) {
  if constexpr (RELU) return fmaxf(u, 0.f);
  else return swishf(u);
}
template <bool RELU>
LASR_DEV float bn_act_grad(float u) {
  if constexpr (RELU) return u > 0.f ? 1.f : 0.f;
  else return swish_grad(u);
}

// The BatchNorm + activation backward of one element (train mode: the batch-mean terms; eval
// mode: inv_n = 0): dy from the BN input y, the activation-output gradient dh and the channel's
// statistics / column totals.  One definition for bn_act_bwd_apply_kernel and BnDyWin.
template <bool RELU>
LASR_DEV float bn_dy(float yv, float gv, float sc, float sf, float mu, float rs, float ga, float t1, float t2,
                     float inv_n) {
  const float du = gv * bn_act_grad<RELU>(yv * sc + sf);
  const float xh = (yv - mu) * rs;
  return ga * rs * (du - t1 * inv_n - xh * t2 * inv_n);
}

// glu_dwconv_bwd's dy window computed on the fly from y and dh (lasr_bn_act_glu_dwconv_bwd): the
// values bn_act_bwd_apply_kernel would have stored, without the fp32 dy round trip or its launch
template <typename TY, typename TH, bool RELU>
struct BnDyWin {
  const TY* y;
  const TH* dh;
  const float *scale, *shift, *mean, *rstd, *gamma, *tot;
  float* dgamma;
  float* dbeta;
  float inv_n;
  int C;
  LASR_DEV float one(float yv, float gv, int c) const {
    return bn_dy<RELU>(yv, gv, scale[c], shift[c], mean[c], rstd[c], gamma[c], tot[c], tot[C + c], inv_n);
  }
  LASR_DEV void load8(const TY* row, int ce, float* v, float* u) const {
    float yv[8], gv[8];
    ldv<8>(row + ce, yv);
    ldv<8>(dh + (row - y) + ce, gv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = one(yv[k], gv[k], ce + k);
      u[k] = 0.f;
    }
  }
  LASR_DEV void load2(const TY* row, int ce, float* v, float* u) const {
    float yv[2], gv[2];
    ldv<2>(row + ce, yv);
    ldv<2>(dh + (row - y) + ce, gv);
    v[0] = one(yv[0], gv[0], ce);
    v[1] = one(yv[1], gv[1], ce + 1);
    u[0] = u[1] = 0.f;
  }
  LASR_DEV float2 pair(const float* v, const float*) const { return make_float2(v[0], v[1]); }
  // the parameter gradients (bn_act_bwd_apply_kernel's block-0 job: the totals are final here)
  LASR_DEV void finish(int) const {
    if (blockIdx.x == 0 && blockIdx.y == 0)
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        dbeta[c] += tot[c];
        dgamma[c] += tot[C + c];
      }
  }
};

// Elementwise BN + activation, 8 channels per thread (C % 8 == 0; the host checks).
template <typename TY, typename TH, bool RELU>
__global__ void bn_act_fwd_kernel(const TY* y, int64_t rows, int C, const float* scale,
                                  const float* shift, TH* h) {
  const int64_t n8 = rows * C / 8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)((e * 8) % C);
    float v[8], sc[8], sf[8];
    ldv<8>(y + e * 8, v);
    ldv<8>(scale + c, sc);
    ldv<8>(shift + c, sf);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = bn_act<RELU>(v[q] * sc[q] + sf[q]);
    stv<8>(h + e * 8, v);
  }
}

constexpr int BN_ROWS = 64;
// 256 threads = BN_G row groups x BN_CP channel pairs; a block reduces BN_ROWS rows of
// 2*BN_CP channels and combines its row groups in LDS (fixed order).
constexpr int BN_G = 8, BN_CP = 32;
template <typename TY, typename TH, bool RELU>
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(const TY* y, const TH* dh, int64_t rows, int C,
                                                                const float* scale, const float* shift,
                                                                const float* mean, const float* rstd, float* part) {
  __shared__ float sp[BN_G][2][2 * BN_CP];
  const int cp = threadIdx.x % BN_CP, grp = threadIdx.x / BN_CP;
  const int c = (blockIdx.x * BN_CP + cp) * 2;
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  if (c < C) {
    const float sc[2] = {scale[c], scale[c + 1]}, sf[2] = {shift[c], shift[c + 1]};
    const float mu[2] = {mean[c], mean[c + 1]}, rs[2] = {rstd[c], rstd[c + 1]};
    const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
    const int64_t r1 = r0 + BN_ROWS < rows ? r0 + BN_ROWS : rows;
    for (int64_t r = r0 + grp; r < r1; r += BN_G) {
      float yv[2], gv[2];
      ldv<2>(y + r * C + c, yv);
      ldv<2>(dh + r * C + c, gv);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float du = gv[q] * bn_act_grad<RELU>(yv[q] * sc[q] + sf[q]);
        s1[q] += du;
        s2[q] += du * (yv[q] - mu[q]) * rs[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    sp[grp][0][2 * cp + q] = s1[q];
    sp[grp][1][2 * cp + q] = s2[q];
  }
  __syncthreads();
  if (threadIdx.x >= 2 * 2 * BN_CP) return;
  const int which = threadIdx.x / (2 * BN_CP), cl = threadIdx.x % (2 * BN_CP);
  const int cc = blockIdx.x * 2 * BN_CP + cl;
  if (cc >= C) return;
  float v = sp[0][which][cl];
#pragma unroll
  for (int q = 1; q < BN_G; ++q) v += sp[q][which][cl];
  part[(int64_t)blockIdx.y * 2 * C + (int64_t)which * C + cc] = v;
}
__global__ void bn_bwd_total_kernel(const float* part, int nparts, int C, float* tot,
                                    float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
  for (int p = 0; p < nparts; ++p) {
    s1 += part[(int64_t)p * 2 * C + c];
    s2 += part[(int64_t)p * 2 * C + C + c];
  }
  tot[c] = s1;
  tot[C + c] = s2;
  dbeta[c] += s1;
  dgamma[c] += s2;
}
template <typename TY, typename TH, typename TD, bool RELU>
__global__ void bn_act_bwd_apply_kernel(const TY* y, const TH* dh, int64_t rows, int C,
                                        const float* scale, const float* shift,
                                        const float* mean, const float* rstd,
                                        const float* gamma, const float* tot, TD* dy,
                                        float* dgamma, float* dbeta, int batch_stats) {
  if (blockIdx.x == 0)  // parameter gradients (the column totals are final here)
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      dbeta[c] += tot[c];
      dgamma[c] += tot[C + c];
    }
  const int64_t n8 = rows * C / 8;
  // eval mode (running statistics): mean / rstd are constants, so the batch-mean terms
  // of the train-mode gradient vanish and dx = gamma * rstd * du
  const float inv_n = batch_stats ? 1.f / (float)rows : 0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)((e * 8) % C);
    float yv[8], gv[8], o[8];
    ldv<8>(y + e * 8, yv);
    ldv<8>(dh + e * 8, gv);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + q;
      o[q] = bn_dy<RELU>(yv[q], gv[q], scale[c], shift[c], mean[c], rstd[c], gamma[c], tot[c], tot[C + c], inv_n);
    }
    stv<8>(dy + e * 8, o);
  }
}

// ================================ host API =========================================
static unsigned gridn(int64_t n) { return (unsigned)std::min<int64_t>(cdiv(n, 256), 16384); }

extern "C" int lasr_conv1_fwd(const float* x, int B, int T, int F, int C, const float* w,
                              const float* bias, void* y1, int dt, void* stream) {
  LASR_CHECK_ARG(T >= 3 && F >= 3 && C > 0, "lasr_conv1_fwd: bad sizes");
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const size_t shm = (size_t)(3 * F + 10 * C) * sizeof(float);
  LASR_CHECK_ARG(shm <= 64 * 1024, "lasr_conv1_fwd: too much LDS");
  hipStream_t st = (hipStream_t)stream;
  constexpr int rpb = C1F_ROWS;  // rows per block
  if (C % 8 == 0 && 256 % (C / 8) == 0 && ((uintptr_t)y1 & 15) == 0 &&
      (size_t)rpb * 3 * F * sizeof(float) <= 64 * 1024) {
    const size_t shv = (size_t)rpb * 3 * F * sizeof(float);
    const int nrows = B * T1;
    const unsigned nb = (unsigned)cdiv(nrows, rpb);
    if (dt == LASR_F32) conv1_fwd_v8_kernel<float><<<nb, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, w, bias, (float*)y1, rpb);
    else conv1_fwd_v8_kernel<bf16_t><<<nb, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, w, bias, (bf16_t*)y1, rpb);
    return lasr_check_launch("conv1_fwd");
  }
  if (dt == LASR_F32) conv1_fwd_kernel<float><<<B * T1, 256, shm, st>>>(x, T, F, C, T1, F1, w, bias, (float*)y1);
  else conv1_fwd_kernel<bf16_t><<<B * T1, 256, shm, st>>>(x, T, F, C, T1, F1, w, bias, (bf16_t*)y1);
  return lasr_check_launch("conv1_fwd");
}

extern "C" int lasr_conv1_bwd(const float* x, int B, int T, int F, int C, const void* dy1, int dt,
                              float* dw, float* db, float* ws, int64_t ws_floats, void* stream) {
  const int T1 = (T - 3) / 2 + 1, F1 = (F - 3) / 2 + 1;
  const int nrows = B * T1;
  // rows per block: 16 (998 blocks at config 2, four per CU: twice the loads in flight of
  // 32-row blocks, 143 -> 108 us standalone, tools/conv1_bench.py)
  constexpr int rpb = C1B_ROWS;
  const bool vec = C % 8 == 0 && 256 % (C / 8) == 0 && ((uintptr_t)dy1 & 15) == 0 &&
                   (size_t)(rpb * 3 * F + 8 * 256) * sizeof(float) <= 64 * 1024;
  const int nparts = (int)cdiv(nrows, vec ? rpb : C1B_ROWS);
  LASR_CHECK_ARG(ws_floats >= (int64_t)(nparts + 1) * 10 * C, "lasr_conv1_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (vec) {
    const size_t shv = (size_t)(rpb * 3 * F + 8 * 256) * sizeof(float);
    if (dt == LASR_F32) conv1_bwd_v8_kernel<float><<<nparts, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, (const float*)dy1, ws, rpb);
    else conv1_bwd_v8_kernel<bf16_t><<<nparts, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, (const bf16_t*)dy1, ws, rpb);
  } else {
    const size_t shm = (size_t)C1B_ROWS * 3 * F * sizeof(float);
    if (dt == LASR_F32) conv1_bwd_kernel<float><<<nparts, 256, shm, st>>>(x, T, F, C, T1, F1, nrows, (const float*)dy1, ws);
    else conv1_bwd_kernel<bf16_t><<<nparts, 256, shm, st>>>(x, T, F, C, T1, F1, nrows, (const bf16_t*)dy1, ws);
  }
  int rc = lasr_check_launch("conv1_bwd");
  if (rc) return rc;
  // partials [nparts][10][C] -> tot[10*C] (after the partials) -> dw[c*9+k], db[c]
  float* tot = ws + (int64_t)nparts * 10 * C;
  rc = lasr_reduce_cols(ws, nparts, (int64_t)10 * C, tot, nullptr, 10 * C, 0, st);
  if (rc) return rc;
  return lasr_scatter_kc(tot, 9, C, 9, dw, db, st);
}

extern "C" int lasr_im2col3x3s2(const void* y1, int dt, int B, int T1, int F1, int C, void* col,
                                void* stream) {
  LASR_CHECK_ARG(C % 8 == 0, "lasr_im2col3x3s2: C %% 8 != 0");
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const int64_t n8 = (int64_t)B * T2 * F2 * 9 * C / 8;
  LASR_CHECK_ARG(n8 * 8 < (1ll << 31), "lasr_im2col3x3s2: column matrix too large");
  hipStream_t st = (hipStream_t)stream;
  if (dt == LASR_F32) im2col_kernel<float><<<gridn(n8), 256, 0, st>>>((const float*)y1, B, T1, F1, C, T2, F2, (float*)col);
  else im2col_kernel<bf16_t><<<gridn(n8), 256, 0, st>>>((const bf16_t*)y1, B, T1, F1, C, T2, F2, (bf16_t*)col);
  return lasr_check_launch("im2col");
}

extern "C" int lasr_col2im3x3s2(const void* dcol, int dt, int B, int T1, int F1, int C,
                                const void* y1, void* dy1, void* stream) {
  LASR_CHECK_ARG(C % 8 == 0, "lasr_col2im3x3s2: C %% 8 != 0");
  const int T2 = (T1 - 3) / 2 + 1, F2 = (F1 - 3) / 2 + 1;
  const int64_t n = (int64_t)B * T1 * F1 * (C / 8);
  LASR_CHECK_ARG((int64_t)B * T2 * F2 * 9 * C < (1ll << 31), "lasr_col2im3x3s2: column matrix too large");
  hipStream_t st = (hipStream_t)stream;
  if (dt == LASR_F32) col2im_kernel<float><<<gridn(n), 256, 0, st>>>((const float*)dcol, B, T1, F1, C, T2, F2, (const float*)y1, (float*)dy1);
  else col2im_kernel<bf16_t><<<gridn(n), 256, 0, st>>>((const bf16_t*)dcol, B, T1, F1, C, T2, F2, (const bf16_t*)y1, (bf16_t*)dy1);
  return lasr_check_launch("col2im");
}

extern "C" int lasr_permute_last2(const void* src, int sdt, int64_t N, int64_t A, int64_t Bd,
                                  void* dst, int ddt, int reverse, int accumulate, void* stream) {
  const int64_t n = N * A * Bd;
  if (n == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
#define PL(TS, TD) permute_last2_kernel<TS, TD><<<gridn(n), 256, 0, st>>>((const TS*)src, N, A, Bd, (TD*)dst, reverse, accumulate)
  if (sdt == LASR_F32 && ddt == LASR_F32) PL(float, float);
  else if (sdt == LASR_F32) PL(float, bf16_t);
  else if (ddt == LASR_F32) PL(bf16_t, float);
  else PL(bf16_t, bf16_t);
#undef PL
  return lasr_check_launch("permute_last2");
}

extern "C" int lasr_glu_dwconv_fwd(const void* z1, int dt, int B, int T, int C, int K,
                                   const float* w, const float* bias, void* y, int ydt,
                                   float* stats_ws, void* stream) {
  LASR_CHECK_ARG(K == DW_K, "lasr_glu_dwconv_fwd: only kernel size %d is built (got %d)", DW_K, K);
  LASR_CHECK_ARG(C % 2 == 0, "lasr_glu_dwconv_fwd: C must be even");
  const int nchunk = (int)cdiv(T, DW_TT);
  dim3 g((unsigned)(B * nchunk), (unsigned)cdiv(C, 2 * DW_CP));
  hipStream_t st = (hipStream_t)stream;
  const int vec = C % 8 == 0 && ((uintptr_t)z1 & 15) == 0;
#define GF(TT, TY) glu_dwconv_fwd_kernel<TT, TY><<<g, DW_NT, 0, st>>>((const TT*)z1, T, C, w, bias, (TY*)y, stats_ws, vec)
  if (dt == LASR_F32 && ydt == LASR_F32) GF(float, float);
  else if (dt == LASR_F32) GF(float, bf16_t);
  else if (ydt == LASR_F32) GF(bf16_t, float);
  else GF(bf16_t, bf16_t);
#undef GF
  return lasr_check_launch("glu_dwconv_fwd");
}

extern "C" int lasr_dwconv_nparts(int B, int T) { return (int)(B * cdiv(T, DW_TT)); }

extern "C" int lasr_bn_finalize(const float* stats_ws, int nparts, int C, float eps,
                                float momentum, const float* gamma, const float* beta,
                                float* running_mean, float* running_var, int64_t* num_batches,
                                float* mean, float* rstd, float* scale, float* shift,
                                int update_running, void* stream) {
  bn_finalize_par_kernel<<<(unsigned)cdiv(C, BNF_C), BNF_C * BNF_G, 0, (hipStream_t)stream>>>(
      stats_ws, nparts, C, eps, momentum, gamma, beta, running_mean, running_var, num_batches,
      mean, rstd, scale, shift, update_running);
  return lasr_check_launch("bn_finalize");
}

template <bool RELU>
static void bn_act_fwd_launch(const void* y, int ydt, int64_t rows, int C, const float* scale, const float* shift,
                              void* h, int hdt, int64_t n, hipStream_t st) {
#define BF(TY, TH) bn_act_fwd_kernel<TY, TH, RELU><<<gridn(n), 256, 0, st>>>((const TY*)y, rows, C, scale, shift, (TH*)h)
  if (ydt == LASR_F32 && hdt == LASR_F32) BF(float, float);
  else if (ydt == LASR_F32) BF(float, bf16_t);
  else if (hdt == LASR_F32) BF(bf16_t, float);
  else BF(bf16_t, bf16_t);
#undef BF
}

extern "C" int lasr_bn_act_fwd(const void* y, int ydt, int64_t rows, int C, const float* scale,
                               const float* shift, void* h, int hdt, int act, void* stream) {
  LASR_CHECK_ARG(C % 8 == 0, "lasr_bn_act_fwd: C must be a multiple of 8");
  LASR_CHECK_ARG(act == LASR_ACT_SWISH || act == LASR_ACT_RELU, "lasr_bn_act_fwd: act must be SWISH or RELU");
  const int64_t n = rows * C / 8;
  if (n == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (act == LASR_ACT_RELU) bn_act_fwd_launch<true>(y, ydt, rows, C, scale, shift, h, hdt, n, st);
  else bn_act_fwd_launch<false>(y, ydt, rows, C, scale, shift, h, hdt, n, st);
  return lasr_check_launch("bn_act_fwd");
}

template <bool RELU>
static int bn_act_bwd_launch(const void* y, int ydt, const void* dh, int hdt, int64_t rows, int C,
                             const float* scale, const float* shift, const float* mean, const float* rstd,
                             const float* gamma, float* dgamma, float* dbeta, void* dy, int dydt, float* ws,
                             int64_t nparts, int batch_stats, hipStream_t st) {
  float* tot = ws + nparts * 2 * C;
  dim3 g((unsigned)cdiv(C, 2 * BN_CP), (unsigned)nparts);
#define BR(TY, TH) bn_act_bwd_reduce_kernel<TY, TH, RELU><<<g, 256, 0, st>>>((const TY*)y, (const TH*)dh, rows, C, scale, shift, mean, rstd, ws)
  if (ydt == LASR_F32 && hdt == LASR_F32) BR(float, float);
  else if (ydt == LASR_F32) BR(float, bf16_t);
  else if (hdt == LASR_F32) BR(bf16_t, float);
  else BR(bf16_t, bf16_t);
#undef BR
  int rc = lasr_check_launch("bn_act_bwd/reduce");
  if (rc) return rc;
  rc = lasr_reduce_cols(ws, (int)nparts, 2 * C, tot, nullptr, 2 * C, 0, st);
  if (rc) return rc;
  const int64_t n = rows * C / 8;
#define BA(TY, TH, TD) bn_act_bwd_apply_kernel<TY, TH, TD, RELU><<<gridn(n), 256, 0, st>>>((const TY*)y, (const TH*)dh, rows, C, scale, shift, mean, rstd, gamma, tot, (TD*)dy, dgamma, dbeta, batch_stats)
  const bool yf = ydt == LASR_F32, hf = hdt == LASR_F32, df = dydt == LASR_F32;
  if (yf && hf && df) BA(float, float, float);
  else if (yf && hf) BA(float, float, bf16_t);
  else if (yf && df) BA(float, bf16_t, float);
  else if (yf) BA(float, bf16_t, bf16_t);
  else if (hf && df) BA(bf16_t, float, float);
  else if (hf) BA(bf16_t, float, bf16_t);
  else if (df) BA(bf16_t, bf16_t, float);
  else BA(bf16_t, bf16_t, bf16_t);
#undef BA
  return lasr_check_launch("bn_act_bwd/apply");
}

extern "C" int lasr_bn_act_bwd(const void* y, int ydt, const void* dh, int hdt, int64_t rows,
                               int C, const float* scale, const float* shift, const float* mean,
                               const float* rstd, const float* gamma, float* dgamma,
                               float* dbeta, void* dy, int dydt, float* ws, int64_t ws_floats,
                               int batch_stats, int act, void* stream) {
  const int64_t nparts = cdiv(rows, BN_ROWS);
  LASR_CHECK_ARG(ws_floats >= (nparts + 1) * 2 * C, "lasr_bn_act_bwd: workspace too small");
  LASR_CHECK_ARG(nparts <= 65535, "lasr_bn_act_bwd: too many rows");
  LASR_CHECK_ARG(act == LASR_ACT_SWISH || act == LASR_ACT_RELU, "lasr_bn_act_bwd: act must be SWISH or RELU");
  if (rows == 0) return LASR_OK;
  LASR_CHECK_ARG(C % 8 == 0, "lasr_bn_act_bwd: C must be a multiple of 8");
  hipStream_t st = (hipStream_t)stream;
  if (act == LASR_ACT_RELU)
    return bn_act_bwd_launch<true>(y, ydt, dh, hdt, rows, C, scale, shift, mean, rstd, gamma, dgamma, dbeta, dy,
                                   dydt, ws, nparts, batch_stats, st);
  return bn_act_bwd_launch<false>(y, ydt, dh, hdt, rows, C, scale, shift, mean, rstd, gamma, dgamma, dbeta, dy,
                                  dydt, ws, nparts, batch_stats, st);
}

extern "C" int lasr_glu_dwconv_bwd(const void* z1, int dt, const void* dy, int dydt, int B, int T,
                                   int C, int K, const float* w, void* dz1, float* dw, float* db,
                                   float* ws, int64_t ws_floats, void* stream) {
  LASR_CHECK_ARG(K == DW_K, "lasr_glu_dwconv_bwd: only kernel size %d is built", DW_K);
  const int nchunk = (int)cdiv(T, DW_TT);
  const int nparts = B * nchunk;
  LASR_CHECK_ARG(ws_floats >= (int64_t)nparts * (DW_K + 1) * C, "lasr_glu_dwconv_bwd: workspace too small");
  LASR_CHECK_ARG(C % 2 == 0, "lasr_glu_dwconv_bwd: C must be even");
  dim3 g((unsigned)nparts, (unsigned)cdiv(C, 2 * DW_CP));
  hipStream_t st = (hipStream_t)stream;
  const int vec = C % 8 == 0 && ((uintptr_t)z1 & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dz1 & 15) == 0;
#define GB(TT, TD) glu_dwconv_bwd_kernel<TT, TD><<<g, DW_NT, 0, st>>>((const TT*)z1, (const TD*)dy, T, C, w, (TT*)dz1, ws, vec)
  if (dt == LASR_F32 && dydt == LASR_F32) GB(float, float);
  else if (dt == LASR_F32) GB(float, bf16_t);
  else if (dydt == LASR_F32) GB(bf16_t, float);
  else GB(bf16_t, bf16_t);
#undef GB
  int rc = lasr_check_launch("glu_dwconv_bwd");
  if (rc || (!dw && !db)) return rc;  // no outputs: partials left in ws (deferred reduction)
  LASR_CHECK_ARG(dw && db, "lasr_glu_dwconv_bwd: dw and db go together");
  return lasr_reduce_cols(ws, nparts, (int64_t)(DW_K + 1) * C, dw, db, (int64_t)DW_K * C, 1, st);
}

// lasr_bn_act_bwd + lasr_glu_dwconv_bwd with the BN backward's elementwise pass folded into the
// depthwise-conv backward's dy window (BnDyWin): one launch and the fp32 dy round trip fewer, the
// same dz1 / dw / db / dgamma / dbeta bits.
template <typename TT, typename TY, typename TH, bool RELU>
static void bn_glu_launch(dim3 g, hipStream_t st, const void* z1, const void* y, const void* dh, int T, int C,
                          const float* w, void* dz1, float* ws, int vec, const BnDyWin<TY, TH, RELU>& f) {
  glu_dwconv_bwd_kernel<TT, TY, BnDyWin<TY, TH, RELU>><<<g, DW_NT, 0, st>>>((const TT*)z1, (const TY*)y, T, C, w,
                                                                          (TT*)dz1, ws, vec, f);
}

template <typename TT, typename TY, typename TH>
static void bn_glu_dispatch(bool relu, dim3 g, hipStream_t st, const void* z1, const void* y, const void* dh, int T,
                            int C, const float* w, void* dz1, float* ws, int vec, const float* scale,
                            const float* shift, const float* mean, const float* rstd, const float* gamma,
                            const float* tot, float* dgamma, float* dbeta, float inv_n) {
  if (relu)
    bn_glu_launch<TT, TY, TH, true>(g, st, z1, y, dh, T, C, w, dz1, ws, vec,
                                    BnDyWin<TY, TH, true>{(const TY*)y, (const TH*)dh, scale, shift, mean, rstd,
                                                          gamma, tot, dgamma, dbeta, inv_n, C});
  else
    bn_glu_launch<TT, TY, TH, false>(g, st, z1, y, dh, T, C, w, dz1, ws, vec,
                                     BnDyWin<TY, TH, false>{(const TY*)y, (const TH*)dh, scale, shift, mean, rstd,
                                                            gamma, tot, dgamma, dbeta, inv_n, C});
}

extern "C" int lasr_bn_act_glu_dwconv_bwd(const void* y, int ydt, const void* dh, int hdt, int B, int T, int C,
                                          const float* scale, const float* shift, const float* mean,
                                          const float* rstd, const float* gamma, float* dgamma, float* dbeta,
                                          float* bn_ws, int64_t bn_ws_floats, int batch_stats, int act,
                                          const void* z1, int dt, int K, const float* w, void* dz1, float* dw,
                                          float* db, float* ws, int64_t ws_floats, void* stream) {
  const int64_t rows = (int64_t)B * T;
  const int64_t nparts_bn = cdiv(rows, BN_ROWS);
  LASR_CHECK_ARG(bn_ws_floats >= (nparts_bn + 1) * 2 * C, "lasr_bn_act_glu_dwconv_bwd: BN workspace too small");
  LASR_CHECK_ARG(nparts_bn <= 65535, "lasr_bn_act_glu_dwconv_bwd: too many rows");
  LASR_CHECK_ARG(act == LASR_ACT_SWISH || act == LASR_ACT_RELU, "lasr_bn_act_glu_dwconv_bwd: act must be SWISH or RELU");
  LASR_CHECK_ARG(K == DW_K, "lasr_bn_act_glu_dwconv_bwd: only kernel size %d is built", DW_K);
  LASR_CHECK_ARG(C % 8 == 0 && rows > 0, "lasr_bn_act_glu_dwconv_bwd: C must be a multiple of 8, rows > 0");
  LASR_CHECK_ARG((ydt == LASR_F32 || ydt == LASR_BF16) && (hdt == LASR_F32 || hdt == LASR_BF16) &&
                     (dt == LASR_F32 || dt == LASR_BF16), "lasr_bn_act_glu_dwconv_bwd: bad dtype");
  const int nchunk = (int)cdiv(T, DW_TT);
  const int nparts = B * nchunk;
  LASR_CHECK_ARG(ws_floats >= (int64_t)nparts * (DW_K + 1) * C, "lasr_bn_act_glu_dwconv_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  // BN column totals, exactly as lasr_bn_act_bwd computes them
  float* tot = bn_ws + nparts_bn * 2 * C;
  {
    dim3 g((unsigned)cdiv(C, 2 * BN_CP), (unsigned)nparts_bn);
#define BR(RL, TY, TH) bn_act_bwd_reduce_kernel<TY, TH, RL><<<g, 256, 0, st>>>((const TY*)y, (const TH*)dh, rows, C, scale, shift, mean, rstd, bn_ws)
    const bool relu = act == LASR_ACT_RELU, yf = ydt == LASR_F32, hf = hdt == LASR_F32;
    if (relu) {
      if (yf && hf) BR(true, float, float); else if (yf) BR(true, float, bf16_t);
      else if (hf) BR(true, bf16_t, float); else BR(true, bf16_t, bf16_t);
    } else {
      if (yf && hf) BR(false, float, float); else if (yf) BR(false, float, bf16_t);
      else if (hf) BR(false, bf16_t, float); else BR(false, bf16_t, bf16_t);
    }
#undef BR
    if (int rc = lasr_check_launch("bn_act_glu_dwconv_bwd/reduce")) return rc;
    if (int rc = lasr_reduce_cols(bn_ws, (int)nparts_bn, 2 * C, tot, nullptr, 2 * C, 0, st)) return rc;
  }
  const float inv_n = batch_stats ? 1.f / (float)rows : 0.f;
  dim3 g((unsigned)nparts, (unsigned)cdiv(C, 2 * DW_CP));
  const int vec = ((uintptr_t)z1 & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)dh & 15) == 0 &&
                  ((uintptr_t)dz1 & 15) == 0;
  const bool relu = act == LASR_ACT_RELU;
#define BG(TT, TY, TH) bn_glu_dispatch<TT, TY, TH>(relu, g, st, z1, y, dh, T, C, w, dz1, ws, vec, scale, shift, mean, rstd, gamma, tot, dgamma, dbeta, inv_n)
  const bool zf = dt == LASR_F32, yf = ydt == LASR_F32, hf = hdt == LASR_F32;
  if (zf) {
    if (yf && hf) BG(float, float, float); else if (yf) BG(float, float, bf16_t);
    else if (hf) BG(float, bf16_t, float); else BG(float, bf16_t, bf16_t);
  } else {
    if (yf && hf) BG(bf16_t, float, float); else if (yf) BG(bf16_t, float, bf16_t);
    else if (hf) BG(bf16_t, bf16_t, float); else BG(bf16_t, bf16_t, bf16_t);
  }
#undef BG
  int rc = lasr_check_launch("bn_act_glu_dwconv_bwd");
  if (rc || (!dw && !db)) return rc;  // no outputs: partials left in ws (deferred reduction)
  LASR_CHECK_ARG(dw && db, "lasr_bn_act_glu_dwconv_bwd: dw and db go together");
  return lasr_reduce_cols(ws, nparts, (int64_t)(DW_K + 1) * C, dw, db, (int64_t)DW_K * C, 1, st);
}
