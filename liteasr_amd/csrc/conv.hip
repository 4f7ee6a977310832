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
      for (int kw = 0; kw < 3; ++kw) acc += wc[kh * 3 + kw] * xs[kh * F + 2 * f1 + kw];
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
// Same per-output arithmetic order as the scalar kernels above.
template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_v8_kernel(const float* __restrict__ x, int T_, int F,
                                                           int C, int T1, int F1, const float* w,
                                                           const float* bias, T* y1) {
  extern __shared__ float xs[];  // the 3 contiguous input rows 2*t1 .. 2*t1+2
  const int bt = blockIdx.x;
  const int b = bt / T1, t1 = bt - b * T1;
  const float* src = x + ((int64_t)b * T_ + 2 * t1) * F;
  for (int i = threadIdx.x; i < 3 * F; i += 256) xs[i] = src[i];
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
  T* out = y1 + (int64_t)bt * F1 * C + c0;
  for (int f1 = fg; f1 < F1; f1 += NFG) {
    float xv[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) xv[kh * 3 + kw] = xs[kh * F + 2 * f1 + kw];
    float o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float acc = bv[q];
#pragma unroll
      for (int k = 0; k < 9; ++k) acc += wr[q][k] * xv[k];
      o[q] = fmaxf(acc, 0.f);
    }
    st8(out + (int64_t)f1 * C, o);
  }
}

constexpr int C1V_ROWS = 32;  // (b,t1) rows per vectorised conv1-bwd block
template <typename T>
__global__ __launch_bounds__(256) void conv1_bwd_v8_kernel(const float* __restrict__ x, int T_, int F,
                                                           int C, int T1, int F1, int nrows,
                                                           const T* __restrict__ dy1, float* part) {
  extern __shared__ float sh[];  // C1V_ROWS x 3F input rows, then the 8*256 reduce slab
  float* xs = sh;
  float* red = sh + C1V_ROWS * 3 * F;
  const int r0 = blockIdx.x * C1V_ROWS;
  const int nr = min(C1V_ROWS, nrows - r0);
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
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t el = e * 8;
    const int64_t m = el / (9 * C);
    const int k = (int)(el - m * 9 * C);
    const int tap = k / C, cin = k - tap * C;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int64_t b = m / (T2 * F2);
    const int rem = (int)(m - b * T2 * F2);
    const int t2 = rem / F2, f2 = rem - t2 * F2;
    const T* src = y1 + ((b * T1 + 2 * t2 + kh) * F1 + 2 * f2 + kw) * C + cin;
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
    const int cin = (int)(e % C8) * 8;
    const int64_t pix = e / C8;
    const int fi = (int)(pix % F1);
    const int64_t bt = pix / F1;
    const int ti = (int)(bt % T1);
    const int64_t b = bt / T1;
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

template <typename T, typename TY>
__global__ __launch_bounds__(256) void glu_dwconv_fwd_kernel(const T* __restrict__ z1, int T_,
                                                             int C, const float* w,
                                                             const float* bias, TY* y,
                                                             float* stats) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  const int nchunk = (T_ + DW_TT - 1) / DW_TT;
  const int b = blockIdx.x / nchunk, t0 = (blockIdx.x - b * nchunk) * DW_TT;
  if (c >= C) return;
  float g[DW_WIN];
#pragma unroll
  for (int i = 0; i < DW_WIN; ++i) {
    const int t = t0 - DW_P + i;
    float v = 0.f;
    if (t >= 0 && t < T_) {
      const T* zr = z1 + ((int64_t)b * T_ + t) * 2 * C;
      v = to_f(zr[c]) * sigmoidf_(to_f(zr[C + c]));
    }
    g[i] = v;
  }
  float wk[DW_K];
#pragma unroll
  for (int k = 0; k < DW_K; ++k) wk[k] = w[c * DW_K + k];
  const float bs = bias[c];
  int cnt = 0;
  float mean = 0.f, m2 = 0.f;
#pragma unroll
  for (int i = 0; i < DW_TT; ++i) {
    const int t = t0 + i;
    if (t < T_) {
      float acc = bs;
#pragma unroll
      for (int k = 0; k < DW_K; ++k) acc += wk[k] * g[i + k];
      y[((int64_t)b * T_ + t) * C + c] = from_f<TY>(acc);
      const float yv = to_f(from_f<TY>(acc));  // stats on the stored value
      ++cnt;
      const float dlt = yv - mean;
      mean += dlt / cnt;
      m2 += dlt * (yv - mean);
    }
  }
  float* st = stats + (int64_t)blockIdx.x * 3 * C;
  st[c] = (float)cnt;
  st[C + c] = mean;
  st[2 * C + c] = m2;
}

template <typename T, typename TD>
__global__ __launch_bounds__(256) void glu_dwconv_bwd_kernel(const T* __restrict__ z1,
                                                             const TD* __restrict__ dy, int T_,
                                                             int C, const float* w, T* dz1,
                                                             float* part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  const int nchunk = (T_ + DW_TT - 1) / DW_TT;
  const int b = blockIdx.x / nchunk, t0 = (blockIdx.x - b * nchunk) * DW_TT;
  if (c >= C) return;
  float g[DW_WIN], d[DW_WIN];
#pragma unroll
  for (int i = 0; i < DW_WIN; ++i) {
    const int t = t0 - DW_P + i;
    float gv = 0.f, dv = 0.f;
    if (t >= 0 && t < T_) {
      const int64_t r = (int64_t)b * T_ + t;
      gv = to_f(z1[r * 2 * C + c]) * sigmoidf_(to_f(z1[r * 2 * C + C + c]));
      dv = to_f(dy[r * C + c]);
    }
    g[i] = gv;
    d[i] = dv;
  }
  float wk[DW_K], dw[DW_K];
#pragma unroll
  for (int k = 0; k < DW_K; ++k) { wk[k] = w[c * DW_K + k]; dw[k] = 0.f; }
  float db = 0.f;
#pragma unroll
  for (int i = 0; i < DW_TT; ++i) {
    const int t = t0 + i;
    if (t < T_) {
      const float dyt = d[i + DW_P];
      db += dyt;
#pragma unroll
      for (int k = 0; k < DW_K; ++k) dw[k] += dyt * g[i + k];
      // dg[t] = sum_k w[k] * dy[t - k + P]
      float dg = 0.f;
#pragma unroll
      for (int k = 0; k < DW_K; ++k) dg += wk[k] * d[i + 2 * DW_P - k];
      const int64_t r = (int64_t)b * T_ + t;
      const float a = to_f(z1[r * 2 * C + c]);
      const float s = sigmoidf_(to_f(z1[r * 2 * C + C + c]));
      dz1[r * 2 * C + c] = from_f<T>(dg * s);
      dz1[r * 2 * C + C + c] = from_f<T>(dg * a * s * (1.f - s));
    }
  }
  float* pp = part + (int64_t)blockIdx.x * (DW_K + 1) * C;
#pragma unroll
  for (int k = 0; k < DW_K; ++k) pp[k * C + c] = dw[k];
  pp[DW_K * C + c] = db;
}

__global__ void dw_reduce_kernel(const float* part, int nparts, int C, float* dw, float* db) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // e = c*(K+1) + k
  if (e >= C * (DW_K + 1)) return;
  const int c = e / (DW_K + 1), k = e - c * (DW_K + 1);
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[((int64_t)p * (DW_K + 1) + k) * C + c];
  if (k < DW_K) dw[c * DW_K + k] += s;
  else db[c] += s;
}

// ------------------------------- BatchNorm ---------------------------------------
// 1024 threads = 32 channels x BNF_G partial-groups, combined exactly in double (fixed
// order), then one thread per channel finalises.
constexpr int BNF_G = 32;
__global__ __launch_bounds__(1024) void bn_finalize_par_kernel(
    const float* stats, int nparts, int C, float eps, float momentum, const float* gamma,
    const float* beta, float* rmean, float* rvar, int64_t* nbt, float* mean, float* rstd,
    float* scale, float* shift, int update) {
  __shared__ double sn[BNF_G][33], smu[BNF_G][33], sm2[BNF_G][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + tx;
  if (blockIdx.x == 0 && threadIdx.x == 0 && update == 1 && nbt) nbt[0] += 1;
  if (update == 2) {  // eval mode: normalise with the running statistics
    if (ty == 0 && c < C) {
      const float rs = rsqrtf(rvar[c] + eps);
      mean[c] = rmean[c];
      rstd[c] = rs;
      const float sc = gamma[c] * rs;
      scale[c] = sc;
      shift[c] = beta[c] - rmean[c] * sc;
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
  n = 0.0;
  s = 0.0;
#pragma unroll
  for (int g = 0; g < BNF_G; ++g) { n += sn[g][tx]; s += smu[g][tx]; }
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
  if (ty != 0 || c >= C) return;
  m2 = 0.0;
#pragma unroll
  for (int g = 0; g < BNF_G; ++g) m2 += sm2[g][tx];
  const float var = (float)(m2 / n);
  const float rs = rsqrtf(var + eps);
  mean[c] = (float)mu;
  rstd[c] = rs;
  const float sc = gamma[c] * rs;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mu * sc;
  if (update == 1) {
    const float uvar = n > 1.0 ? (float)(m2 / (n - 1.0)) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * uvar;
  }
}

template <typename TY, typename TH>
__global__ void bn_swish_fwd_kernel(const TY* y, int64_t rows, int C, const float* scale,
                                    const float* shift, TH* h) {
  const int64_t n = rows * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    h[e] = from_f<TH>(swishf(to_f(y[e]) * scale[c] + shift[c]));
  }
}

constexpr int BN_ROWS = 64;
template <typename TY, typename TH>
__global__ void bn_swish_bwd_reduce_kernel(const TY* y, const TH* dh, int64_t rows, int C,
                                           const float* scale, const float* shift,
                                           const float* mean, const float* rstd, float* part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
  const int64_t r1 = r0 + BN_ROWS < rows ? r0 + BN_ROWS : rows;
  const float sc = scale[c], sf = shift[c], mu = mean[c], rs = rstd[c];
  float s1 = 0.f, s2 = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    const float yv = to_f(y[r * C + c]);
    const float du = to_f(dh[r * C + c]) * swish_grad(yv * sc + sf);
    s1 += du;
    s2 += du * (yv - mu) * rs;
  }
  part[(int64_t)blockIdx.y * 2 * C + c] = s1;
  part[(int64_t)blockIdx.y * 2 * C + C + c] = s2;
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
__global__ void bn_bwd_accum_kernel(const float* tot, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  dbeta[c] += tot[c];
  dgamma[c] += tot[C + c];
}

template <typename TY, typename TH, typename TD>
__global__ void bn_swish_bwd_apply_kernel(const TY* y, const TH* dh, int64_t rows, int C,
                                          const float* scale, const float* shift,
                                          const float* mean, const float* rstd,
                                          const float* gamma, const float* tot, TD* dy) {
  const int64_t n = rows * C;
  const float inv_n = 1.f / (float)rows;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const float yv = to_f(y[e]);
    const float du = to_f(dh[e]) * swish_grad(yv * scale[c] + shift[c]);
    const float xh = (yv - mean[c]) * rstd[c];
    dy[e] = from_f<TD>(gamma[c] * rstd[c] * (du - tot[c] * inv_n - xh * tot[C + c] * inv_n));
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
  if (C % 8 == 0 && 256 % (C / 8) == 0 && ((uintptr_t)y1 & 15) == 0) {
    const size_t shv = (size_t)3 * F * sizeof(float);
    if (dt == LASR_F32) conv1_fwd_v8_kernel<float><<<B * T1, 256, shv, st>>>(x, T, F, C, T1, F1, w, bias, (float*)y1);
    else conv1_fwd_v8_kernel<bf16_t><<<B * T1, 256, shv, st>>>(x, T, F, C, T1, F1, w, bias, (bf16_t*)y1);
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
  const bool vec = C % 8 == 0 && 256 % (C / 8) == 0 && ((uintptr_t)dy1 & 15) == 0 &&
                   (size_t)(C1V_ROWS * 3 * F + 8 * 256) * sizeof(float) <= 64 * 1024;
  const int nparts = (int)cdiv(nrows, vec ? C1V_ROWS : C1B_ROWS);
  LASR_CHECK_ARG(ws_floats >= (int64_t)(nparts + 1) * 10 * C, "lasr_conv1_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (vec) {
    const size_t shv = (size_t)(C1V_ROWS * 3 * F + 8 * 256) * sizeof(float);
    if (dt == LASR_F32) conv1_bwd_v8_kernel<float><<<nparts, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, (const float*)dy1, ws);
    else conv1_bwd_v8_kernel<bf16_t><<<nparts, 256, shv, st>>>(x, T, F, C, T1, F1, nrows, (const bf16_t*)dy1, ws);
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
  const int nchunk = (int)cdiv(T, DW_TT);
  dim3 g((unsigned)(B * nchunk), (unsigned)cdiv(C, 256));
  hipStream_t st = (hipStream_t)stream;
#define GF(TT, TY) glu_dwconv_fwd_kernel<TT, TY><<<g, 256, 0, st>>>((const TT*)z1, T, C, w, bias, (TY*)y, stats_ws)
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
  bn_finalize_par_kernel<<<(unsigned)cdiv(C, 32), 32 * BNF_G, 0, (hipStream_t)stream>>>(
      stats_ws, nparts, C, eps, momentum, gamma, beta, running_mean, running_var, num_batches,
      mean, rstd, scale, shift, update_running);
  return lasr_check_launch("bn_finalize");
}

extern "C" int lasr_bn_swish_fwd(const void* y, int ydt, int64_t rows, int C, const float* scale,
                                 const float* shift, void* h, int hdt, void* stream) {
  const int64_t n = rows * C;
  if (n == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
#define BF(TY, TH) bn_swish_fwd_kernel<TY, TH><<<gridn(n), 256, 0, st>>>((const TY*)y, rows, C, scale, shift, (TH*)h)
  if (ydt == LASR_F32 && hdt == LASR_F32) BF(float, float);
  else if (ydt == LASR_F32) BF(float, bf16_t);
  else if (hdt == LASR_F32) BF(bf16_t, float);
  else BF(bf16_t, bf16_t);
#undef BF
  return lasr_check_launch("bn_swish_fwd");
}

extern "C" int lasr_bn_swish_bwd(const void* y, int ydt, const void* dh, int hdt, int64_t rows,
                                 int C, const float* scale, const float* shift, const float* mean,
                                 const float* rstd, const float* gamma, float* dgamma,
                                 float* dbeta, void* dy, int dydt, float* ws, int64_t ws_floats,
                                 void* stream) {
  const int64_t nparts = cdiv(rows, BN_ROWS);
  LASR_CHECK_ARG(ws_floats >= (nparts + 1) * 2 * C, "lasr_bn_swish_bwd: workspace too small");
  LASR_CHECK_ARG(nparts <= 65535, "lasr_bn_swish_bwd: too many rows");
  if (rows == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  float* tot = ws + nparts * 2 * C;
  dim3 g((unsigned)cdiv(C, 256), (unsigned)nparts);
#define BR(TY, TH) bn_swish_bwd_reduce_kernel<TY, TH><<<g, 256, 0, st>>>((const TY*)y, (const TH*)dh, rows, C, scale, shift, mean, rstd, ws)
  if (ydt == LASR_F32 && hdt == LASR_F32) BR(float, float);
  else if (ydt == LASR_F32) BR(float, bf16_t);
  else if (hdt == LASR_F32) BR(bf16_t, float);
  else BR(bf16_t, bf16_t);
#undef BR
  int rc = lasr_check_launch("bn_swish_bwd/reduce");
  if (rc) return rc;
  rc = lasr_reduce_cols(ws, (int)nparts, 2 * C, tot, nullptr, 2 * C, 0, st);
  if (rc) return rc;
  bn_bwd_accum_kernel<<<(unsigned)cdiv(C, 256), 256, 0, st>>>(tot, C, dgamma, dbeta);
  rc = lasr_check_launch("bn_swish_bwd/accum");
  if (rc) return rc;
  const int64_t n = rows * C;
#define BA(TY, TH, TD) bn_swish_bwd_apply_kernel<TY, TH, TD><<<gridn(n), 256, 0, st>>>((const TY*)y, (const TH*)dh, rows, C, scale, shift, mean, rstd, gamma, tot, (TD*)dy)
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
  return lasr_check_launch("bn_swish_bwd/apply");
}

extern "C" int lasr_glu_dwconv_bwd(const void* z1, int dt, const void* dy, int dydt, int B, int T,
                                   int C, int K, const float* w, void* dz1, float* dw, float* db,
                                   float* ws, int64_t ws_floats, void* stream) {
  LASR_CHECK_ARG(K == DW_K, "lasr_glu_dwconv_bwd: only kernel size %d is built", DW_K);
  const int nchunk = (int)cdiv(T, DW_TT);
  const int nparts = B * nchunk;
  LASR_CHECK_ARG(ws_floats >= (int64_t)(nparts + 1) * (DW_K + 1) * C, "lasr_glu_dwconv_bwd: workspace too small");
  dim3 g((unsigned)nparts, (unsigned)cdiv(C, 256));
  hipStream_t st = (hipStream_t)stream;
#define GB(TT, TD) glu_dwconv_bwd_kernel<TT, TD><<<g, 256, 0, st>>>((const TT*)z1, (const TD*)dy, T, C, w, (TT*)dz1, ws)
  if (dt == LASR_F32 && dydt == LASR_F32) GB(float, float);
  else if (dt == LASR_F32) GB(float, bf16_t);
  else if (dydt == LASR_F32) GB(bf16_t, float);
  else GB(bf16_t, bf16_t);
#undef GB
  int rc = lasr_check_launch("glu_dwconv_bwd");
  if (rc) return rc;
  float* tot = ws + (int64_t)nparts * (DW_K + 1) * C;
  rc = lasr_reduce_cols(ws, nparts, (int64_t)(DW_K + 1) * C, tot, nullptr, (DW_K + 1) * C, 0, st);
  if (rc) return rc;
  return lasr_scatter_kc(tot, DW_K, C, DW_K, dw, db, st);
}
