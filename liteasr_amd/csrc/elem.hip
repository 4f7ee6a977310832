// Elementwise kernels: casts, scaled adds, positional encodings, decoder embedding.
// Reference: liteasr/nets/positional_encoding.py:49-56 (x*sqrt(d) + pe, dropout) and
// :68-75 (relative: dropout(x*sqrt(d)), dropout(pe[:, :T])); decoder embedding
// liteasr/nets/transformer_decoder.py:77-78.
#include "common.h"

static unsigned gridn(int64_t n) { return (unsigned)std::min<int64_t>(cdiv(n, 256), 16384); }

template <typename TS, typename TD>
__global__ void cast_kernel(const TS* s, TD* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = from_f<TD>(to_f(s[i]));
}

template <typename TA, typename TB, typename TO>
__global__ void scale_add_kernel(const TA* a, const TB* b, float sa, float sb, TO* o, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = sa * to_f(a[i]);
    if (b) v += sb * to_f(b[i]);
    o[i] = from_f<TO>(v);
  }
}

template <typename TX, typename TY>
__global__ void pe_fwd_kernel(const TX* x, int64_t rows, int T, int D, const float* pe,
                              float xscale, DropCfg d, TY* y) {
  const int64_t n = rows * D;
  const uint32_t key = drop_key_if(d);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    const int c = (int)(e - r * D);
    float v = x ? to_f(x[e]) * xscale : 0.f;
    if (pe) v += pe[(r % T) * D + c];
    y[e] = from_f<TY>(v * drop_mul_if(d, key, (uint64_t)e));
  }
}

template <typename TY>
__global__ void embed_pe_fwd_kernel(const int32_t* ids, int R, int L, int D, const float* E,
                                    const float* pe, float xscale, DropCfg d, TY* y) {
  const int64_t n = (int64_t)R * D;
  const uint32_t key = drop_key_if(d);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / D), c = (int)(e - (int64_t)r * D);
    const float v = E[(int64_t)ids[r] * D + c] * xscale + (pe ? pe[(int64_t)(r % L) * D + c] : 0.f);
    y[e] = from_f<TY>(v * drop_mul_if(d, key, (uint64_t)e));
  }
}

// Deterministic embedding backward: the workgroup of the first row holding an id sums
// every row with that id and adds it to dE[id].  The rows holding the id are found in
// parallel (ballot compaction, row order kept); the sum runs over EMB_NW row groups (one per
// wave) x 8 accumulators per column and is combined in a fixed order (run-to-run identical).
// 16 waves: a frequent id (the eos padding of the decoder input: hundreds of rows) is one
// chain of dependent load rounds per row group, so its workgroup's time scales with
// rows / (8 x EMB_NW).
constexpr int EMB_EC = 4;   // 64-column chunks per pass of embed_bwd_kernel
constexpr int EMB_NW = 16;  // waves (row groups) per workgroup

template <typename TD>
__global__ __launch_bounds__(EMB_NW * 64) void embed_bwd_kernel(const int32_t* ids, int R, int D, const TD* dy,
                                                                float xscale, DropCfg d, float* dE) {
  extern __shared__ int sid[];  // R ids, up to R matching rows, EMB_NW x EMB_EC x 64 partial sums
  __shared__ int wcnt[EMB_NW];
  int* rows = sid + R;
  for (int i = threadIdx.x; i < R; i += blockDim.x) sid[i] = ids[i];
  __syncthreads();
  const int r = blockIdx.x, id = sid[r];
  if (id < 0) return;  // a negative id contributes nothing (padding_idx rows, rnn_decoder.py:20)
  int earlier = 0;
  for (int k = threadIdx.x; k < r; k += blockDim.x) earlier |= sid[k] == id;
  if (__syncthreads_or(earlier)) return;  // not the first occurrence (uniform)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int n = 0;
  for (int base = r; base < R; base += EMB_NW * 64) {
    const int k = base + threadIdx.x;
    const bool m = k < R && sid[k] == id;
    const uint64_t bal = __ballot(m);
    if (lane == 0) wcnt[w] = __popcll(bal);
    __syncthreads();
    int off = n, tot = 0;
    for (int q = 0; q < EMB_NW; ++q) {
      off += q < w ? wcnt[q] : 0;
      tot += wcnt[q];
    }
    if (m) rows[off + __popcll(bal & ((1ull << lane) - 1))] = k;
    n += tot;
    __syncthreads();
  }
  // 4 row groups x 64 columns per chunk, EC chunks (EC * 64 columns) per pass so a frequent
  // id's long row list is walked once per pass with EC x 8 independent loads in flight (a
  // frequent id, e.g. the eos padding, has hundreds of rows: the latency chain, not
  // bandwidth, bounds this block); per column the same summation order as one chunk a pass
  const uint32_t key = d.p > 0.f ? drop_key(d) : 0u;
  float* part = reinterpret_cast<float*>(rows + R);  // [EMB_NW][EC * 64]
  if ((D & 1) == 0) {
    // even D: a lane takes a column PAIR (one 4/8-B load, one dropout draw for both halves,
    // as the forward drew them); per column the same order as below, so the same bits
    constexpr int PC = EMB_EC / 2, S = 64 * EMB_EC;
    for (int c0 = 0; c0 < D; c0 += S) {
      float a[PC][2][8];
#pragma unroll
      for (int pc = 0; pc < PC; ++pc)
#pragma unroll
        for (int u = 0; u < 8; ++u) a[pc][0][u] = a[pc][1][u] = 0.f;
      for (int q0 = w; q0 < n; q0 += 8 * EMB_NW) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = q0 + EMB_NW * u;
          if (q < n) {
            const int64_t rb = (int64_t)rows[q] * D;
#pragma unroll
            for (int pc = 0; pc < PC; ++pc) {
              const int c = c0 + 128 * pc + 2 * lane;
              if (c < D) {
                float v2[2];
                ldv<2>(dy + rb + c, v2);
                const uint32_t bits = drop_bits(key, (uint64_t)(rb + c) >> 1);
                a[pc][0][u] += v2[0] * ((bits & 0xFFFFu) >= d.thr ? d.scale : 0.f);
                a[pc][1][u] += v2[1] * ((bits >> 16) >= d.thr ? d.scale : 0.f);
              }
            }
          }
        }
      }
#pragma unroll
      for (int pc = 0; pc < PC; ++pc)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          part[w * S + 128 * pc + 2 * lane + j] = ((a[pc][j][0] + a[pc][j][1]) + (a[pc][j][2] + a[pc][j][3])) +
                                                  ((a[pc][j][4] + a[pc][j][5]) + (a[pc][j][6] + a[pc][j][7]));
      __syncthreads();
      if (w == 0) {
#pragma unroll
        for (int pc = 0; pc < PC; ++pc)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int o = 128 * pc + 2 * lane + j, c = c0 + o;
            float t = 0.f;
#pragma unroll
            for (int g = 0; g < EMB_NW; ++g) t += part[g * S + o];
            if (c < D) dE[(int64_t)id * D + c] += t * xscale;
          }
      }
      __syncthreads();
    }
    return;
  }
  for (int c0 = 0; c0 < D; c0 += 64 * EMB_EC) {
    float a[EMB_EC][8];
#pragma unroll
    for (int cc = 0; cc < EMB_EC; ++cc)
#pragma unroll
      for (int u = 0; u < 8; ++u) a[cc][u] = 0.f;
    for (int q0 = w; q0 < n; q0 += 8 * EMB_NW) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + EMB_NW * u;
        if (q < n) {
          const int64_t rb = (int64_t)rows[q] * D;
#pragma unroll
          for (int cc = 0; cc < EMB_EC; ++cc) {
            const int c = c0 + 64 * cc + lane;
            if (c < D) a[cc][u] += to_f(dy[rb + c]) * drop_mul_k(d, key, (uint64_t)(rb + c));
          }
        }
      }
    }
#pragma unroll
    for (int cc = 0; cc < EMB_EC; ++cc)
      part[w * 64 * EMB_EC + 64 * cc + lane] =
          ((a[cc][0] + a[cc][1]) + (a[cc][2] + a[cc][3])) + ((a[cc][4] + a[cc][5]) + (a[cc][6] + a[cc][7]));
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int cc = 0; cc < EMB_EC; ++cc) {
        const int c = c0 + 64 * cc + lane, o = 64 * cc + lane, S = 64 * EMB_EC;
        float t = 0.f;
#pragma unroll
        for (int g = 0; g < EMB_NW; ++g) t += part[g * S + o];
        if (c < D) dE[(int64_t)id * D + c] += t * xscale;
      }
    }
    __syncthreads();
  }
}

template <typename T>
__global__ void fill_kernel(T* d, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = from_f<T>(v);
}

extern "C" int lasr_cast(const void* src, int sdt, void* dst, int ddt, int64_t n, void* stream) {
  if (n <= 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (sdt == LASR_F32 && ddt == LASR_F32) cast_kernel<float, float><<<gridn(n), 256, 0, st>>>((const float*)src, (float*)dst, n);
  else if (sdt == LASR_F32) cast_kernel<float, bf16_t><<<gridn(n), 256, 0, st>>>((const float*)src, (bf16_t*)dst, n);
  else if (ddt == LASR_F32) cast_kernel<bf16_t, float><<<gridn(n), 256, 0, st>>>((const bf16_t*)src, (float*)dst, n);
  else cast_kernel<bf16_t, bf16_t><<<gridn(n), 256, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, n);
  return lasr_check_launch("cast");
}

extern "C" int lasr_scale_add(const void* a, int adt, const void* b, int bdt, float sa, float sb,
                              void* out, int odt, int64_t n, void* stream) {
  if (n <= 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = gridn(n);
#define SA(TA, TB, TO) scale_add_kernel<TA, TB, TO><<<g, 256, 0, st>>>((const TA*)a, (const TB*)b, sa, sb, (TO*)out, n)
  const bool af = adt == LASR_F32, bf = bdt == LASR_F32, of = odt == LASR_F32;
  if (af && bf && of) SA(float, float, float);
  else if (af && bf) SA(float, float, bf16_t);
  else if (af && of) SA(float, bf16_t, float);
  else if (af) SA(float, bf16_t, bf16_t);
  else if (bf && of) SA(bf16_t, float, float);
  else if (bf) SA(bf16_t, float, bf16_t);
  else if (of) SA(bf16_t, bf16_t, float);
  else SA(bf16_t, bf16_t, bf16_t);
#undef SA
  return lasr_check_launch("scale_add");
}

extern "C" int lasr_pe_fwd(const void* x, int xdt, int64_t rows, int T, int D, const float* pe,
                           float xscale, float p, uint64_t seed, void* y, int ydt, void* stream) {
  const int64_t n = rows * D;
  if (n <= 0) return LASR_OK;
  DropCfg d = mkdrop(p, seed);
  hipStream_t st = (hipStream_t)stream;
#define PF(TX, TY) pe_fwd_kernel<TX, TY><<<gridn(n), 256, 0, st>>>((const TX*)x, rows, T, D, pe, xscale, d, (TY*)y)
  if (xdt == LASR_F32 && ydt == LASR_F32) PF(float, float);
  else if (xdt == LASR_F32) PF(float, bf16_t);
  else if (ydt == LASR_F32) PF(bf16_t, float);
  else PF(bf16_t, bf16_t);
#undef PF
  return lasr_check_launch("pe_fwd");
}

extern "C" int lasr_embed_pe_fwd(const int32_t* ids, int R, int L, int D, const float* E,
                                 const float* pe, float xscale, float p, uint64_t seed, void* y,
                                 int ydt, void* stream) {
  const int64_t n = (int64_t)R * D;
  if (n <= 0) return LASR_OK;
  DropCfg d = mkdrop(p, seed);
  hipStream_t st = (hipStream_t)stream;
  if (ydt == LASR_F32) embed_pe_fwd_kernel<float><<<gridn(n), 256, 0, st>>>(ids, R, L, D, E, pe, xscale, d, (float*)y);
  else embed_pe_fwd_kernel<bf16_t><<<gridn(n), 256, 0, st>>>(ids, R, L, D, E, pe, xscale, d, (bf16_t*)y);
  return lasr_check_launch("embed_pe_fwd");
}

extern "C" int lasr_embed_bwd(const int32_t* ids, int R, int D, const void* dy, int dydt,
                              float xscale, float p, uint64_t seed, float* dE, void* stream) {
  if (R <= 0) return LASR_OK;
  LASR_CHECK_ARG(R <= 16384, "lasr_embed_bwd: R=%d > 16384", R);  // 2 R ints + 16 KB of LDS
  DropCfg d = mkdrop(p, seed);
  hipStream_t st = (hipStream_t)stream;
  const size_t shm = ((size_t)2 * R + EMB_NW * 64 * EMB_EC) * sizeof(int);
  if (dydt == LASR_F32) embed_bwd_kernel<float><<<R, EMB_NW * 64, shm, st>>>(ids, R, D, (const float*)dy, xscale, d, dE);
  else embed_bwd_kernel<bf16_t><<<R, EMB_NW * 64, shm, st>>>(ids, R, D, (const bf16_t*)dy, xscale, d, dE);
  return lasr_check_launch("embed_bwd");
}

extern "C" int lasr_fill(void* dst, int dt, int64_t n, float value, void* stream) {
  if (n <= 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dt == LASR_F32) fill_kernel<float><<<gridn(n), 256, 0, st>>>((float*)dst, n, value);
  else fill_kernel<bf16_t><<<gridn(n), 256, 0, st>>>((bf16_t*)dst, n, value);
  return lasr_check_launch("fill");
}
