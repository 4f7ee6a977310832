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
