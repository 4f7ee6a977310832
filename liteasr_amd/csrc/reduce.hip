// Deterministic reduction of per-block partial sums: out[n] (+)= sum_p part[p*N + n].
// 256-thread blocks cover 16 columns x 16 partial-groups (coalesced 64-B reads per
// group row); each thread sums its strided partials (cols_psum), then a fixed-order LDS
// combine.
// Used by every "partials -> parameter gradient" epilogue (LayerNorm, bias colsums,
// BatchNorm, depthwise conv, conv1, positional biases).
#include "common.h"

constexpr int RC_COLS = 16;
constexpr int RC_GROUPS = 16;
constexpr int RC_ACC = 8;

// Column n's partials p = ty, ty + 16, ... summed into RC_ACC accumulators (accumulator k takes
// every RC_ACC-th of them), combined by a fixed pairwise tree.  Every iteration issues its
// RC_ACC loads together (out-of-range ones read nothing): with P = 498 (a LayerNorm's
// 16-row blocks over B*T' = 7968 rows) a thread waits for 4 rounds of loads, not 31 serial
// ones -- these reductions are latency-bound, the bytes are few.
LASR_DEV float cols_psum(const float* __restrict__ part, int P, int64_t N, int64_t n, int ty) {
  float s[RC_ACC];
#pragma unroll
  for (int k = 0; k < RC_ACC; ++k) s[k] = 0.f;
  for (int p = ty; p < P; p += RC_ACC * RC_GROUPS) {
    float v[RC_ACC];
#pragma unroll
    for (int k = 0; k < RC_ACC; ++k) {
      const int q = p + k * RC_GROUPS;
      v[k] = q < P ? part[(int64_t)q * N + n] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < RC_ACC; ++k) s[k] += v[k];
  }
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

__global__ __launch_bounds__(256) void reduce_cols_kernel(const float* __restrict__ part, int P,
                                                          int64_t N, float* out0, float* out1,
                                                          int64_t split, int accumulate) {
  __shared__ float sh[RC_GROUPS][RC_COLS + 1];
  const int tx = threadIdx.x & (RC_COLS - 1), ty = threadIdx.x / RC_COLS;
  const int64_t n = (int64_t)blockIdx.x * RC_COLS + tx;
  sh[ty][tx] = n < N ? cols_psum(part, P, N, n, ty) : 0.f;
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
// 64 segments = 3588 B of kernel arguments (under the 4 KB kernarg budget); a longer list runs
// in ceil(nseg / 64) launches
constexpr int RM_MAXSEG = 64;
constexpr int RM_VEC = 2;  // mode 1: 4-column runs per thread
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
  // the segment of this block: the last one whose blk0 <= blockIdx.x (blk0 strictly increasing)
  int lo = 0, hi = a.nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)blockIdx.x >= a.s[mid].blk0) lo = mid; else hi = mid - 1;
  }
  const RSeg& g = a.s[lo];
  const int b = blockIdx.x - g.blk0;
  if (g.mode == 1) {
    // RM_VEC runs of 4 columns per thread, 1024 columns apart (coalesced per run); every
    // load -- the output's old value for the RMW included -- is issued before the first add,
    // so a thread waits for one round of loads, not two
    float acc[RM_VEC][4], c[RM_VEC][4];
    float* o4[RM_VEC];
    int64_t n[RM_VEC];
#pragma unroll
    for (int j = 0; j < RM_VEC; ++j) {
      n[j] = ((int64_t)b * 256 * RM_VEC + j * 256 + threadIdx.x) * 4;
      o4[j] = n[j] + 4 <= g.split ? g.out0 + n[j] : (n[j] >= g.split ? g.out1 + (n[j] - g.split) : nullptr);
      if (o4[j] && ((uintptr_t)o4[j] & 15) != 0) o4[j] = nullptr;  // unaligned run: element-wise below
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[j][q] = c[j][q] = 0.f;
      if (n[j] < g.N && o4[j] && g.accumulate) {
        const float4 v = *(const float4*)o4[j];
        c[j][0] = v.x; c[j][1] = v.y; c[j][2] = v.z; c[j][3] = v.w;
      }
    }
    int p = 0;
    for (; p + 4 <= g.P; p += 4) {
      float4 v[RM_VEC][4];
#pragma unroll
      for (int j = 0; j < RM_VEC; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[j][u] = n[j] < g.N ? *(const float4*)(g.part + n[j] + (int64_t)(p + u) * g.N) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < RM_VEC; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc[j][0] += v[j][u].x; acc[j][1] += v[j][u].y; acc[j][2] += v[j][u].z; acc[j][3] += v[j][u].w;
        }
    }
    for (; p < g.P; ++p) {
#pragma unroll
      for (int j = 0; j < RM_VEC; ++j) {
        if (n[j] >= g.N) continue;
        const float4 v = *(const float4*)(g.part + n[j] + (int64_t)p * g.N);
        acc[j][0] += v.x; acc[j][1] += v.y; acc[j][2] += v.z; acc[j][3] += v.w;
      }
    }
#pragma unroll
    for (int j = 0; j < RM_VEC; ++j) {
      if (n[j] >= g.N) continue;
      if (o4[j]) {  // the 4 columns in one aligned output run: 16-B RMW
        *(float4*)o4[j] = g.accumulate ? make_float4(c[j][0] + acc[j][0], c[j][1] + acc[j][1], c[j][2] + acc[j][2],
                                                      c[j][3] + acc[j][3])
                                       : make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
        continue;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* o = n[j] + q < g.split ? g.out0 + n[j] + q : g.out1 + (n[j] + q - g.split);
        *o = g.accumulate ? *o + acc[j][q] : acc[j][q];
      }
    }
    return;
  }
  const int tx = threadIdx.x & (RC_COLS - 1), ty = threadIdx.x / RC_COLS;
  const int64_t n = (int64_t)b * RC_COLS + tx;
  sh[ty][tx] = n < g.N ? cols_psum(g.part, g.P, g.N, n, ty) : 0.f;
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
    const int cnt = nseg - base < RM_MAXSEG ? nseg - base : RM_MAXSEG;
    // the many-partial (mode 0) segments' blocks first: they are latency-bound chains of loads,
    // the few-partial slabs' blocks stream around them (blocks are dispatched in index order);
    // every output is written by one segment, so the order changes no value
    int ord[RM_MAXSEG], no = 0;
    for (int pass = 0; pass < 2; ++pass)
      for (int i = 0; i < cnt; ++i) {
        const lasr_reduce_seg& q = segs[base + i];
        const bool v = q.P <= 64 && q.N % 4 == 0 && (q.out1 ? q.split : q.N) % 4 == 0 && ((uintptr_t)q.part & 15) == 0;
        if (v == (pass == 1)) ord[no++] = i;
      }
    for (int oi = 0; oi < cnt; ++oi) {
      const int i = ord[oi];
      const lasr_reduce_seg& q = segs[base + i];
      LASR_CHECK_ARG(q.part && q.out0 && q.N > 0 && q.P > 0, "lasr_reduce_multi: segment %d invalid", base + i);
      const int64_t split = q.out1 ? q.split : q.N;
      LASR_CHECK_ARG(split > 0 && split <= q.N, "lasr_reduce_multi: segment %d split", base + i);
      const bool vec = q.P <= 64 && q.N % 4 == 0 && split % 4 == 0 && ((uintptr_t)q.part & 15) == 0;
      RSeg& g = a.s[a.nseg++];
      g.part = q.part; g.out0 = q.out0; g.out1 = q.out1; g.N = q.N; g.split = split;
      g.P = q.P; g.accumulate = q.accumulate; g.mode = vec ? 1 : 0; g.blk0 = nblk;
      const int64_t nb = vec ? cdiv(q.N / 4, 256 * RM_VEC) : cdiv(q.N, RC_COLS);
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
