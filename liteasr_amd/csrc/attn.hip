// Attention pieces for the materialised-score MHA path.
// Reference: liteasr/nets/attention.py — project_qkv :27-44, apply_attention :46-59
// (masked_fill(mask, -1e38) -> softmax -> dropout -> matmul), RelativeMultiHeadAttention
// :120-154 with pos_bias_u/v :94-97 and the legacy rel_shift :99-118.
//
// rel_shift closed form (verified against the reference by golden vectors): for
// query row i and key column j of a T x T score matrix,
//   j <= i   : bd[i,   T-1-i+j]
//   j == i+1 : 0
//   j >  i+1 : bd[i+1, j-i-2]
// The softmax kernels apply it by index arithmetic (no padded copy), one wave per
// row, the row held in registers (Tk <= 1024).
#include "common.h"
#include "qbias.h"

// qu = q + u, qv = q + v  (q = first D columns of the fused qkv projection)
template <typename T>
__global__ void qbias_fwd_kernel(const T* qkv, int64_t rows, int H, int dk, int64_t ld,
                                 const float* bu, const float* bv, T* qu, T* qv) {
  const int D = H * dk;
  const int64_t n = rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D;
    const int c = (int)(i - r * D);
    const float q = to_f(qkv[r * ld + c]);
    qu[i] = from_f<T>(q + bu[c]);
    qv[i] = from_f<T>(q + bv[c]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void qbias_bwd_kernel(const T* dqu, const T* dqv, int64_t rows, int D,
                                                        T* dqkv, int64_t ld, float* part) {
  qbias_bwd_body<T>(dqu, dqv, rows, D, dqkv, ld, part, blockIdx.x, blockIdx.y);
}
__global__ void qbias_reduce_kernel(const float* part, int nchunk, int D, float* du, float* dv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nchunk; ++k) {
    a += part[(int64_t)k * 2 * D + c];
    b += part[(int64_t)k * 2 * D + D + c];
  }
  du[c] += a;
  dv[c] += b;
}

LASR_DEV float relpos_bd(const float* bd, int i, int j, int T, int ldS) {
  if (j <= i) return bd[(int64_t)i * ldS + (T - 1 - i + j)];
  if (j == i + 1) return 0.f;
  return bd[(int64_t)(i + 1) * ldS + (j - i - 2)];
}

constexpr int SM_MAXC = 16;  // 16 * 64 = 1024 columns max

template <typename TP>
__global__ __launch_bounds__(256) void attn_softmax_fwd_kernel(
    const float* __restrict__ s_ac, const float* __restrict__ s_bd, int relpos, int H, int Tq,
    int Tk, int ldS, int64_t Zrows, const uint8_t* mask, int64_t msb, int64_t msq, TP* P, TP* Praw,
    DropCfg d) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Zrows) return;
  const int64_t z = row / Tq;
  const int i = (int)(row - z * Tq);
  const int b = (int)(z / H);
  const float* ac = s_ac + (z * Tq) * ldS;
  const float* bd = relpos ? s_bd + (z * Tq) * ldS : nullptr;
  const uint8_t* mr = mask ? mask + b * msb + (int64_t)i * msq : nullptr;
  float v[SM_MAXC];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    float s = -INFINITY;
    if (j < Tk) {
      s = ac[(int64_t)i * ldS + j];
      if (relpos) s += relpos_bd(bd, i, j, Tk, ldS);
      if (mr && mr[j]) s = -1e38f;
    }
    v[k] = s;
    m = fmaxf(m, s);
  }
  m = wave_max(m);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    const float e = (j < Tk) ? __expf(v[k] - m) : 0.f;
    v[k] = e;
    sum += e;
  }
  const float inv = 1.f / wave_sum(sum);
  TP* pr = P + row * ldS;
  TP* prr = Praw ? Praw + row * ldS : nullptr;
  const uint32_t key = drop_key_if(d);
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    if (j < Tk) {
      const float p = v[k] * inv;
      pr[j] = from_f<TP>(p * drop_mul_if(d, key, (uint64_t)row * Tk + j));
      if (prr) prr[j] = from_f<TP>(p);
    } else if (j < ldS) {
      pr[j] = from_f<TP>(0.f);
      if (prr) prr[j] = from_f<TP>(0.f);
    }
  }
}

template <typename TP, typename TS>
__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(
    const TP* __restrict__ P, const float* __restrict__ dPd, int H, int Tq, int Tk, int ldS,
    int64_t Zrows, const uint8_t* mask, int64_t msb, int64_t msq, DropCfg d, TS* dS) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Zrows) return;
  const int64_t z = row / Tq;
  const int i = (int)(row - z * Tq);
  const int b = (int)(z / H);
  const uint8_t* mr = mask ? mask + b * msb + (int64_t)i * msq : nullptr;
  const TP* pr = P + row * ldS;
  const float* gr = dPd + row * ldS;
  float p[SM_MAXC], g[SM_MAXC];
  float s = 0.f;
  const uint32_t key = drop_key_if(d);
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    p[k] = 0.f;
    g[k] = 0.f;
    if (j < Tk) {
      p[k] = to_f(pr[j]);
      g[k] = gr[j] * drop_mul_if(d, key, (uint64_t)row * Tk + j);
      s += p[k] * g[k];
    }
  }
  s = wave_sum(s);
  TS* out = dS + row * ldS;
#pragma unroll
  for (int k = 0; k < SM_MAXC; ++k) {
    const int j = lane + 64 * k;
    if (j < Tk) {
      float v = p[k] * (g[k] - s);
      if (mr && mr[j]) v = 0.f;  // masked_fill backward
      out[j] = from_f<TS>(v);
    } else if (j < ldS) {
      out[j] = from_f<TS>(0.f);
    }
  }
}

// dBD[z,r,c] = dS[z,i,j] where k = r*(T+1)+c+1, i = k/T-1, j = k%T (0 if i < 0)
template <typename T>
__global__ void relshift_bwd_kernel(const T* dS, int64_t Z, int Tn, int ldS, T* dBD) {
  const int64_t n = Z * Tn * (int64_t)ldS;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t zr = e / ldS;
    const int c = (int)(e - zr * ldS);
    const int64_t z = zr / Tn;
    const int r = (int)(zr - z * Tn);
    float v = 0.f;
    if (c < Tn) {
      const int64_t k = (int64_t)r * (Tn + 1) + c + 1;
      const int i = (int)(k / Tn) - 1;
      const int j = (int)(k % Tn);
      if (i >= 0 && i < Tn) v = to_f(dS[(z * Tn + i) * ldS + j]);
    }
    dBD[e] = from_f<T>(v);
  }
}

template <typename T>
__global__ void reduce_batch_kernel(const float* src, int B, int H, int Tn, int dk, T* dst) {
  const int64_t n = (int64_t)Tn * H * dk;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / (H * dk);
    const int hc = (int)(e - t * H * dk);
    const int h = hc / dk, c = hc - h * dk;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += src[(((int64_t)b * H + h) * Tn + t) * dk + c];
    dst[e] = from_f<T>(s);
  }
}

static unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>(cdiv(n, 256), 16384); }

extern "C" int lasr_qbias_fwd(const void* qkv, int dt, int B, int T, int H, int dk, int64_t ld,
                              const float* bu, const float* bv, void* qu, void* qv, void* stream) {
  const int64_t rows = (int64_t)B * T;
  if (rows == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = grid_for(rows * H * dk);
  if (dt == LASR_F32) qbias_fwd_kernel<float><<<g, 256, 0, st>>>((const float*)qkv, rows, H, dk, ld, bu, bv, (float*)qu, (float*)qv);
  else qbias_fwd_kernel<bf16_t><<<g, 256, 0, st>>>((const bf16_t*)qkv, rows, H, dk, ld, bu, bv, (bf16_t*)qu, (bf16_t*)qv);
  return lasr_check_launch("qbias_fwd");
}

extern "C" int lasr_qbias_bwd(const void* dqu, const void* dqv, int dt, int B, int T, int H,
                              int dk, void* dqkv, int64_t ld, float* du, float* dv, float* ws,
                              int64_t ws_floats, void* stream) {
  const int64_t rows = (int64_t)B * T;
  const int D = H * dk;
  const int64_t nchunk = cdiv(rows, QB_ROWS);
  LASR_CHECK_ARG(ws_floats >= nchunk * 2 * D, "lasr_qbias_bwd: workspace too small");
  LASR_CHECK_ARG(nchunk <= 65535, "lasr_qbias_bwd: too many rows");
  if (rows == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  LASR_CHECK_ARG(D % 2 == 0 && ld % 2 == 0, "lasr_qbias_bwd: D and ld must be even");
  dim3 g((unsigned)cdiv(D, 2 * QB_CP), (unsigned)nchunk);
  if (dt == LASR_F32) qbias_bwd_kernel<float><<<g, 256, 0, st>>>((const float*)dqu, (const float*)dqv, rows, D, (float*)dqkv, ld, ws);
  else qbias_bwd_kernel<bf16_t><<<g, 256, 0, st>>>((const bf16_t*)dqu, (const bf16_t*)dqv, rows, D, (bf16_t*)dqkv, ld, ws);
  int rc = lasr_check_launch("qbias_bwd");
  if (rc || (!du && !dv)) return rc;  // no outputs: partials left in ws (deferred reduction)
  return lasr_reduce_cols(ws, (int)nchunk, 2 * D, du, dv, D, 1, st);
}

extern "C" int lasr_attn_softmax_fwd(const float* s_ac, const float* s_bd, int relpos, int B,
                                     int H, int Tq, int Tk, int ldS, const uint8_t* mask,
                                     int64_t mask_sb, int64_t mask_sq, void* P, int pdt,
                                     float drop_p, uint64_t seed, void* Praw, void* stream) {
  LASR_CHECK_ARG(Tk <= 64 * SM_MAXC, "lasr_attn_softmax_fwd: Tk=%d > %d", Tk, 64 * SM_MAXC);
  LASR_CHECK_ARG(ldS >= Tk, "lasr_attn_softmax_fwd: ldS < Tk");
  LASR_CHECK_ARG(!relpos || Tq == Tk, "lasr_attn_softmax_fwd: relpos needs Tq == Tk");
  const int64_t rows = (int64_t)B * H * Tq;
  if (rows == 0) return LASR_OK;
  DropCfg d = mkdrop(drop_p, seed);
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = (unsigned)cdiv(rows, 4);
  if (pdt == LASR_F32)
    attn_softmax_fwd_kernel<float><<<g, 256, 0, st>>>(s_ac, s_bd, relpos, H, Tq, Tk, ldS, rows, mask, mask_sb, mask_sq, (float*)P, (float*)Praw, d);
  else
    attn_softmax_fwd_kernel<bf16_t><<<g, 256, 0, st>>>(s_ac, s_bd, relpos, H, Tq, Tk, ldS, rows, mask, mask_sb, mask_sq, (bf16_t*)P, (bf16_t*)Praw, d);
  return lasr_check_launch("attn_softmax_fwd");
}

extern "C" int lasr_attn_softmax_bwd(const void* P, int pdt, const float* dPd, int B, int H,
                                     int Tq, int Tk, int ldS, const uint8_t* mask, int64_t mask_sb,
                                     int64_t mask_sq, float drop_p, uint64_t seed, void* dS,
                                     int dsdt, void* stream) {
  LASR_CHECK_ARG(Tk <= 64 * SM_MAXC, "lasr_attn_softmax_bwd: Tk too large");
  const int64_t rows = (int64_t)B * H * Tq;
  if (rows == 0) return LASR_OK;
  DropCfg d = mkdrop(drop_p, seed);
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = (unsigned)cdiv(rows, 4);
#define SMB(TP, TS)                                                                            \
  attn_softmax_bwd_kernel<TP, TS><<<g, 256, 0, st>>>((const TP*)P, dPd, H, Tq, Tk, ldS, rows, \
                                                     mask, mask_sb, mask_sq, d, (TS*)dS)
  if (pdt == LASR_F32 && dsdt == LASR_F32) SMB(float, float);
  else if (pdt == LASR_F32) SMB(float, bf16_t);
  else if (dsdt == LASR_F32) SMB(bf16_t, float);
  else SMB(bf16_t, bf16_t);
#undef SMB
  return lasr_check_launch("attn_softmax_bwd");
}

extern "C" int lasr_relshift_bwd(const void* dS, int dt, int Z, int T, int ldS, void* dBD,
                                 void* stream) {
  const int64_t n = (int64_t)Z * T * ldS;
  if (n == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dt == LASR_F32) relshift_bwd_kernel<float><<<grid_for(n), 256, 0, st>>>((const float*)dS, Z, T, ldS, (float*)dBD);
  else relshift_bwd_kernel<bf16_t><<<grid_for(n), 256, 0, st>>>((const bf16_t*)dS, Z, T, ldS, (bf16_t*)dBD);
  return lasr_check_launch("relshift_bwd");
}

extern "C" int lasr_reduce_batch(const float* src, int B, int H, int T, int dk, void* dst, int dt,
                                 void* stream) {
  const int64_t n = (int64_t)T * H * dk;
  if (n == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dt == LASR_F32) reduce_batch_kernel<float><<<grid_for(n), 256, 0, st>>>(src, B, H, T, dk, (float*)dst);
  else reduce_batch_kernel<bf16_t><<<grid_for(n), 256, 0, st>>>(src, B, H, T, dk, (bf16_t*)dst);
  return lasr_check_launch("reduce_batch");
}
