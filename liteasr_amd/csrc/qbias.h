// Positional-bias gradient body (liteasr/nets/attention.py:131-135: q + pos_bias_u / v, so
// du / dv are column sums of dqu / dqv and dq = dqu + dqv), shared by lasr_qbias_bwd (attn.hip)
// and the launch that runs it beside a split-K reduction (gemm_ln.hip).
#pragma once
#include "common.h"

// 256 threads = QB_G row groups x QB_CP column pairs; a block covers QB_ROWS rows of
// 2*QB_CP columns and writes one (du, dv) partial per column (groups combined in LDS in a
// fixed order).
constexpr int QB_ROWS = 64, QB_G = 8, QB_CP = 32;
template <typename T>
LASR_DEV void qbias_bwd_body(const T* dqu, const T* dqv, int64_t rows, int D, T* dqkv, int64_t ld, float* part,
                             int bx, int by) {
  __shared__ float sp[QB_G][2][2 * QB_CP];
  const int cp = threadIdx.x % QB_CP, grp = threadIdx.x / QB_CP;
  const int c = (bx * QB_CP + cp) * 2;
  float su[2] = {0.f, 0.f}, sv[2] = {0.f, 0.f};
  if (c < D) {
    const int64_t r0 = (int64_t)by * QB_ROWS;
    const int64_t r1 = r0 + QB_ROWS < rows ? r0 + QB_ROWS : rows;
    for (int64_t r = r0 + grp; r < r1; r += QB_G) {
      float a[2], b[2], o[2];
      ldv<2>(dqu + r * D + c, a);
      ldv<2>(dqv + r * D + c, b);
      su[0] += a[0]; su[1] += a[1];
      sv[0] += b[0]; sv[1] += b[1];
      o[0] = a[0] + b[0];
      o[1] = a[1] + b[1];
      stv<2>(dqkv + r * ld + c, o);
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    sp[grp][0][2 * cp + q] = su[q];
    sp[grp][1][2 * cp + q] = sv[q];
  }
  __syncthreads();
  if (threadIdx.x >= 4 * QB_CP) return;
  const int which = threadIdx.x / (2 * QB_CP), cl = threadIdx.x % (2 * QB_CP);
  const int cc = bx * 2 * QB_CP + cl;
  if (cc >= D) return;
  float v = sp[0][which][cl];
#pragma unroll
  for (int q = 1; q < QB_G; ++q) v += sp[q][which][cl];
  part[(int64_t)by * 2 * D + (int64_t)which * D + cc] = v;
}
