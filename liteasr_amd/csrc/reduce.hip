// Deterministic reduction of per-block partial sums: out[n] (+)= sum_p part[p*N + n].
// 256-thread blocks cover 16 columns x 16 partial-groups (coalesced 64-B reads per
// group row); each thread sums its strided partials, then a fixed-order LDS combine.
// Used by every "partials -> parameter gradient" epilogue (LayerNorm, bias colsums,
// BatchNorm, depthwise conv, conv1, positional biases).
#include "common.h"

constexpr int RC_COLS = 16;
constexpr int RC_GROUPS = 16;

__global__ __launch_bounds__(256) void reduce_cols_kernel(const float* __restrict__ part, int P,
                                                          int64_t N, float* out0, float* out1,
                                                          int64_t split, int accumulate) {
  __shared__ float sh[RC_GROUPS][RC_COLS + 1];
  const int tx = threadIdx.x & (RC_COLS - 1), ty = threadIdx.x / RC_COLS;
  const int64_t n = (int64_t)blockIdx.x * RC_COLS + tx;
  // 4 independent accumulators (4 loads in flight per thread), combined in fixed order
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (n < N) {
    int p = ty;
    for (; p + 3 * RC_GROUPS < P; p += 4 * RC_GROUPS) {
      s0 += part[(int64_t)p * N + n];
      s1 += part[(int64_t)(p + RC_GROUPS) * N + n];
      s2 += part[(int64_t)(p + 2 * RC_GROUPS) * N + n];
      s3 += part[(int64_t)(p + 3 * RC_GROUPS) * N + n];
    }
    for (; p < P; p += RC_GROUPS) s0 += part[(int64_t)p * N + n];
  }
  sh[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < RC_GROUPS; ++g) t += sh[g][tx];
    float* o = n < split ? out0 + n : out1 + (n - split);
    *o = accumulate ? *o + t : t;
  }
}

int lasr_reduce_cols(const float* part, int P, int64_t N, float* out0, float* out1, int64_t split,
                     int accumulate, hipStream_t st) {
  if (N <= 0) return LASR_OK;
  if (!out1) split = N;
  reduce_cols_kernel<<<(unsigned)cdiv(N, RC_COLS), 256, 0, st>>>(part, P, N, out0, out1, split,
                                                                 accumulate);
  return lasr_check_launch("reduce_cols");
}

// ---- batched ("deferred") reductions ------------------------------------------------
// One launch finishes many partial -> gradient reductions of a backward node (LayerNorm
// gamma/beta, positional biases, split-K weight gradients and their bias rowsums), each
// with the summation order of its single-launch counterpart:
//   mode 0 (many partials, P large): reduce_cols' 16 columns x 16 partial groups
//   mode 1 (few partials, P <= 64): 4 columns per thread, partials summed in order 0..P-1
//                                   (splitk_reduce_kernel's order)
constexpr int RM_MAXSEG = 32;
struct RSeg {
  const float* part;
  float* out0;
  float* out1;
  int64_t N, split;
  int P, accumulate, mode, blk0;
};
struct RSegs {
  RSeg s[RM_MAXSEG];
  int nseg;
};

__global__ __launch_bounds__(256) void reduce_multi_kernel(RSegs a) {
  __shared__ float sh[RC_GROUPS][RC_COLS + 1];
  int si = 0;
  for (int i = 1; i < a.nseg; ++i)
    if ((int)blockIdx.x >= a.s[i].blk0) si = i;
  const RSeg& g = a.s[si];
  const int b = blockIdx.x - g.blk0;
  if (g.mode == 1) {
    const int64_t n = ((int64_t)b * 256 + threadIdx.x) * 4;
    if (n >= g.N) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const float* src = g.part + n;
    int p = 0;
    for (; p + 4 <= g.P; p += 4) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const float4*)(src + (int64_t)(p + u) * g.N);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[0] += v[u].x; acc[1] += v[u].y; acc[2] += v[u].z; acc[3] += v[u].w;
      }
    }
    for (; p < g.P; ++p) {
      const float4 v = *(const float4*)(src + (int64_t)p * g.N);
      acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
    }
    float* o4 = n + 4 <= g.split ? g.out0 + n : (n >= g.split ? g.out1 + (n - g.split) : nullptr);
    if (o4 && ((uintptr_t)o4 & 15) == 0) {  // the 4 columns in one aligned output run: 16-B RMW
      float4 r = make_float4(acc[0], acc[1], acc[2], acc[3]);
      if (g.accumulate) {
        const float4 c = *(const float4*)o4;
        r = make_float4(c.x + acc[0], c.y + acc[1], c.z + acc[2], c.w + acc[3]);
      }
      *(float4*)o4 = r;
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float* o = n + q < g.split ? g.out0 + n + q : g.out1 + (n + q - g.split);
      *o = g.accumulate ? *o + acc[q] : acc[q];
    }
    return;
  }
  const int tx = threadIdx.x & (RC_COLS - 1), ty = threadIdx.x / RC_COLS;
  const int64_t n = (int64_t)b * RC_COLS + tx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (n < g.N) {
    int p = ty;
    for (; p + 3 * RC_GROUPS < g.P; p += 4 * RC_GROUPS) {
      s0 += g.part[(int64_t)p * g.N + n];
      s1 += g.part[(int64_t)(p + RC_GROUPS) * g.N + n];
      s2 += g.part[(int64_t)(p + 2 * RC_GROUPS) * g.N + n];
      s3 += g.part[(int64_t)(p + 3 * RC_GROUPS) * g.N + n];
    }
    for (; p < g.P; p += RC_GROUPS) s0 += g.part[(int64_t)p * g.N + n];
  }
  sh[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && n < g.N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < RC_GROUPS; ++q) t += sh[q][tx];
    float* o = n < g.split ? g.out0 + n : g.out1 + (n - g.split);
    *o = g.accumulate ? *o + t : t;
  }
}

extern "C" int lasr_reduce_multi(const lasr_reduce_seg* segs, int nseg, void* stream) {
  LASR_CHECK_ARG(nseg >= 0 && (nseg == 0 || segs), "lasr_reduce_multi: bad segment list");
  hipStream_t st = (hipStream_t)stream;
  for (int base = 0; base < nseg; base += RM_MAXSEG) {
    RSegs a = {};
    int nblk = 0;
    for (int i = 0; i < RM_MAXSEG && base + i < nseg; ++i) {
      const lasr_reduce_seg& q = segs[base + i];
      LASR_CHECK_ARG(q.part && q.out0 && q.N > 0 && q.P > 0, "lasr_reduce_multi: segment %d invalid", base + i);
      const int64_t split = q.out1 ? q.split : q.N;
      LASR_CHECK_ARG(split > 0 && split <= q.N, "lasr_reduce_multi: segment %d split", base + i);
      const bool vec = q.P <= 64 && q.N % 4 == 0 && split % 4 == 0 && ((uintptr_t)q.part & 15) == 0;
      RSeg& g = a.s[a.nseg++];
      g.part = q.part; g.out0 = q.out0; g.out1 = q.out1; g.N = q.N; g.split = split;
      g.P = q.P; g.accumulate = q.accumulate; g.mode = vec ? 1 : 0; g.blk0 = nblk;
      const int64_t nb = vec ? cdiv(q.N / 4, 256) : cdiv(q.N, RC_COLS);
      LASR_CHECK_ARG(nblk + nb < (1ll << 31), "lasr_reduce_multi: too many blocks");
      nblk += (int)nb;
    }
    if (nblk == 0) continue;
    reduce_multi_kernel<<<nblk, 256, 0, st>>>(a);
    const int rc = lasr_check_launch("reduce_multi");
    if (rc) return rc;
  }
  return LASR_OK;
}

// dst[c*ld + k] (+)= src[k*C + c] for k < K (the [K][C] -> [C][ld] reshuffle of weight
// grads reduced in a [.][K][C] partial layout); also src[K*C + c] -> bias[c] if given.
__global__ void scatter_kc_kernel(const float* src, int K, int C, int ld, float* dst,
                                  float* bias) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (K + (bias ? 1 : 0)) * C) return;
  const int k = e / C, c = e - k * C;
  if (k < K) dst[(int64_t)c * ld + k] += src[e];
  else bias[c] += src[e];
}

int lasr_scatter_kc(const float* src, int K, int C, int ld, float* dst, float* bias,
                    hipStream_t st) {
  const int n = (K + (bias ? 1 : 0)) * C;
  scatter_kc_kernel<<<(unsigned)cdiv(n, 256), 256, 0, st>>>(src, K, C, ld, dst, bias);
  return lasr_check_launch("scatter_kc");
}
