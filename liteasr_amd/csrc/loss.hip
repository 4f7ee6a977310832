// Label-smoothed KL attention loss + hybrid loss combine.
// Reference: liteasr/criterions/hybrid_ctc_attn.py:49-64 (true_dist = s/(V-1) everywhere,
// 1-s at the target; KLDivLoss(reduction="none") on log_softmax(h); ignored rows zeroed;
// sum / B) and :78 (ctc_weight * ctc + (1 - ctc_weight) * att).
// One workgroup per row; a row is read once in fwd (online max/sum-exp + sum of logits)
// and once in bwd (grad = g * (softmax - true_dist)).
#include "common.h"

LASR_DEV float xlogx(float x) { return x > 0.f ? x * __logf(x) : 0.f; }

template <typename T>
__global__ __launch_bounds__(256) void lsm_kl_fwd_kernel(const T* __restrict__ logits, int V, int64_t ld,
                                                         const int32_t* target, int ignore,
                                                         float smoothing, float* lse, float* loss) {
  __shared__ float red[32];
  const int r = blockIdx.x;
  const int tg = target[r];
  if (tg == ignore) {
    if (threadIdx.x == 0) { loss[r] = 0.f; lse[r] = 0.f; }
    return;
  }
  const T* x = logits + (int64_t)r * ld;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float v = to_f(x[c]);
    sx += v;
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
  }
  const float M = block_max(m, red);
  const float S = block_sum(m == -INFINITY ? 0.f : s * __expf(m - M), red + 16);
  const float SX = block_sum(sx, red);
  if (threadIdx.x == 0) {
    const float l = M + __logf(S);
    const float eps = smoothing / (float)(V - 1), conf = 1.f - smoothing;
    const float lpt = to_f(x[tg]) - l;
    const float sum_lp = SX - (float)V * l;
    const float ent = (float)(V - 1) * xlogx(eps) + xlogx(conf);
    // sum_c td_c * lp_c, with td = eps everywhere except conf at the target
    const float cross = eps * (sum_lp - lpt) + conf * lpt;
    loss[r] = ent - cross;
    lse[r] = l;
  }
}

template <typename T, typename TG>
__global__ __launch_bounds__(256) void lsm_kl_bwd_kernel(const T* __restrict__ logits, int V, int64_t ld,
                                                         const int32_t* target, int ignore,
                                                         float smoothing, const float* lse,
                                                         TG* grad, float gscale,
                                                         const float* gdev) {
  const int r = blockIdx.x;
  const int tg = target[r];
  TG* g = grad + (int64_t)r * ld;
  if (tg == ignore) {
    for (int c = threadIdx.x; c < V; c += blockDim.x) g[c] = from_f<TG>(0.f);
    return;
  }
  const float gs = gscale * (gdev ? gdev[0] : 1.f);
  const float eps = smoothing / (float)(V - 1), conf = 1.f - smoothing;
  const float l = lse[r];
  const T* x = logits + (int64_t)r * ld;
  for (int c = threadIdx.x; c < V; c += blockDim.x) {
    const float td = (c == tg) ? conf : eps;
    g[c] = from_f<TG>(gs * (__expf(to_f(x[c]) - l) - td));
  }
}

__global__ void loss_combine_kernel(const float* a, int na, float wa, const float* b, int nb,
                                    float wb, float* out) {
  __shared__ float red[32];
  float sa = 0.f, sb = 0.f;
  for (int i = threadIdx.x; i < na; i += blockDim.x) sa += a[i];
  for (int i = threadIdx.x; i < nb; i += blockDim.x) sb += b[i];
  sa = block_sum(sa, red);
  sb = block_sum(sb, red + 16);
  if (threadIdx.x == 0) out[0] = wa * sa + wb * sb;
}

extern "C" int lasr_lsm_kl_fwd(const void* logits, int ldt, int R, int V, int64_t ld,
                               const int32_t* target,
                               int ignore, float smoothing, float* lse, float* loss_rows,
                               void* stream) {
  LASR_CHECK_ARG(R >= 0 && V > 1 && ld >= V, "lasr_lsm_kl_fwd: bad sizes");
  if (R == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
  if (ldt == LASR_F32)
    lsm_kl_fwd_kernel<float><<<R, 256, 0, st>>>((const float*)logits, V, ld, target, ignore, smoothing, lse, loss_rows);
  else
    lsm_kl_fwd_kernel<bf16_t><<<R, 256, 0, st>>>((const bf16_t*)logits, V, ld, target, ignore, smoothing, lse, loss_rows);
  return lasr_check_launch("lsm_kl_fwd");
}

extern "C" int lasr_lsm_kl_bwd(const void* logits, int ldt, int R, int V, int64_t ld,
                               const int32_t* target,
                               int ignore, float smoothing, const float* lse, void* grad, int gdt,
                               float gscale, const float* gdev, void* stream) {
  LASR_CHECK_ARG(R >= 0 && V > 1 && ld >= V, "lasr_lsm_kl_bwd: bad sizes");
  if (R == 0) return LASR_OK;
  hipStream_t st = (hipStream_t)stream;
#define KLB(TT, TGG)                                                                      \
  lsm_kl_bwd_kernel<TT, TGG><<<R, 256, 0, st>>>((const TT*)logits, V, ld, target, ignore, smoothing, \
                                                lse, (TGG*)grad, gscale, gdev)
  if (ldt == LASR_F32 && gdt == LASR_F32) KLB(float, float);
  else if (ldt == LASR_F32) KLB(float, bf16_t);
  else if (gdt == LASR_F32) KLB(bf16_t, float);
  else KLB(bf16_t, bf16_t);
#undef KLB
  return lasr_check_launch("lsm_kl_bwd");
}

extern "C" int lasr_loss_combine(const float* a, int na, float wa, const float* b, int nb, float wb,
                                 float* out, void* stream) {
  loss_combine_kernel<<<1, 256, 0, (hipStream_t)stream>>>(a, na, wa, b, nb, wb, out);
  return lasr_check_launch("loss_combine");
}
