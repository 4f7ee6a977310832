// Gradient clipping + NaN-skip + Noam/Adam over flat fp32 buffers, all on the device.
// Reference: liteasr/trainer.py:152-171 (clip_grad_norm_(params, clip); skip the step
// when the norm is NaN), liteasr/optims/noam.py:33-46 (lr = factor * d^-0.5 *
// min(s^-0.5, s * warmup^-1.5), s counts *taken* steps), liteasr/optims/adam.py:24-34
// (torch.optim.Adam: bias-corrected moments, eps outside the sqrt).
// The host never reads the norm: step count, lr, norm and the skip flag live in a
// small device `state` vector, so the whole step can be captured in a hipGraph.
#include "common.h"

constexpr int SQ_CHUNK = 16384;  // elements per partial

// The Adam operands are streamed once per step (30 B per parameter, ~1.4 GB), so they are
// loaded and stored non-temporally: 250 -> 230 us per step at 46.2 M parameters, bit identical
// (profiles/r05/adam_ab.jsonl).  Timing ablation (tools/gemm_exp.sh with EXP_FILES=optim; 0 in
// the product): bit 1 goes back to plain loads and stores; bit 2 reads the gradient
// non-temporally in the sum of squares too (slower: sum of squares + Adam 262-270 us with plain
// loads there, 288-297 us with non-temporal ones, 325 us before; profiles/r05/adam_sumsq_ab.jsonl).
#ifndef LASR_EXP
#define LASR_EXP 0
#endif
typedef float adam_f4 __attribute__((ext_vector_type(4)));
LASR_DEV float4 adam_ld(const float4* q) {
  if constexpr ((LASR_EXP & 1) == 0) {
    const adam_f4 x = __builtin_nontemporal_load((const adam_f4*)q);
    return make_float4(x[0], x[1], x[2], x[3]);
  } else {
    return *q;
  }
}
LASR_DEV void adam_st(float4* q, float4 x) {
  if constexpr ((LASR_EXP & 1) == 0) {
    const adam_f4 y = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(y, (adam_f4*)q);
  } else {
    *q = x;
  }
}

// One partial per SQ_CHUNK elements.  Full chunks: 16-B loads, all 16 per thread issued
// before the sums (4 accumulators, fixed order); the ragged last chunk: scalar loads.
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* g, int64_t n, float* ws) {
  __shared__ float red[32];
  const int64_t base = (int64_t)blockIdx.x * SQ_CHUNK;
  float s = 0.f;
  if (base + SQ_CHUNK <= n && (((uintptr_t)g) & 15) == 0) {
    constexpr int NV = SQ_CHUNK / (256 * 4);
    float4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const float4* q = (const float4*)(g + base + ((int64_t)k * 256 + threadIdx.x) * 4);
      if constexpr ((LASR_EXP & 2) != 0) {
        const adam_f4 x = __builtin_nontemporal_load((const adam_f4*)q);
        v[k] = make_float4(x[0], x[1], x[2], x[3]);
      } else {
        v[k] = *q;
      }
    }
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      a[0] += v[k].x * v[k].x;
      a[1] += v[k].y * v[k].y;
      a[2] += v[k].z * v[k].z;
      a[3] += v[k].w * v[k].w;
    }
    s = (a[0] + a[1]) + (a[2] + a[3]);
  } else {
    for (int64_t i = base + threadIdx.x; i < base + SQ_CHUNK && i < n; i += 256) {
      const float v = g[i];
      s += v * v;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// state: [0] taken steps, [1] lr, [2] grad norm, [3] skipped flag, [4] clip coefficient
__global__ __launch_bounds__(256) void opt_finalize_kernel(const float* ws, int nparts,
                                                           float* state, float max_norm,
                                                           int lr_mode, float lr, float factor,
                                                           float model_dim, float warmup) {
  __shared__ float red[32];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += ws[i];
  s = block_sum(s, red);
  if (threadIdx.x != 0) return;
  const float norm = sqrtf(s);
  // torch.nn.utils.clip_grad_norm_: clip_coef = max_norm / (norm + 1e-6) clamped to <= 1
  // for ANY max_norm (0 zeroes the gradients, as the reference does with the dataclass
  // default clip_grad_norm = 0.0); "no clipping" is max_norm = +inf (coef 1; fminf
  // drops the NaN of inf/inf)
  const float coef = fminf(max_norm / (norm + 1e-6f), 1.f);
  const bool skip = isnan(norm);
  state[2] = norm;
  state[3] = skip ? 1.f : 0.f;
  state[4] = coef;
  if (!skip) {
    const float step = state[0] + 1.f;
    state[0] = step;
    float r = lr;
    if (lr_mode == 1) r = factor * powf(model_dim, -0.5f) * fminf(powf(step, -0.5f), step * powf(warmup, -1.5f));
    state[1] = r;
  }
}

template <typename TL>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, TL* __restrict__ plp,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, const float* __restrict__ state,
                                                   float beta1, float beta2, float eps, float wd) {
  if (state[3] != 0.f) return;  // NaN norm: step skipped (reference trainer.py:157)
  const float step = state[0], lr = state[1], coef = state[4];
  const float bc1 = 1.f - powf(beta1, step);
  const float bc2 = 1.f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  // the multiply-adds are spelled out (fmaf / __fmul_rn), so the rounding does not depend on
  // how the compiler contracts the expression in each copy of it
  auto upd = [&](float gi, float pi, float& mi, float& vi) {
    gi = __fmul_rn(gi, coef);
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    mi = fmaf(1.f - beta1, gi - mi, mi);  // lerp, as torch.optim.Adam
    vi = fmaf(__fmul_rn(1.f - beta2, gi), gi, __fmul_rn(vi, beta2));
    return pi - __fmul_rn(step_size, mi) / (sqrtf(vi) / bc2s + eps);
  };
  // 16-B accesses, 4 parameters per thread and group; two groups (i, i + stride) per iteration
  // so eight 16-B loads per thread are in flight (the same per-element arithmetic)
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (((uintptr_t)plp) & (4 * sizeof(TL) - 1)) == 0;
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;
    auto group = [&](int64_t i, float4 g4, float4 p4, float4 m4, float4 v4) {
      float o[4];
      o[0] = upd(g4.x, p4.x, m4.x, v4.x);
      o[1] = upd(g4.y, p4.y, m4.y, v4.y);
      o[2] = upd(g4.z, p4.z, m4.z, v4.z);
      o[3] = upd(g4.w, p4.w, m4.w, v4.w);
      adam_st((float4*)m + i, m4);
      adam_st((float4*)v + i, v4);
      adam_st((float4*)p + i, make_float4(o[0], o[1], o[2], o[3]));
      if (plp) stv<4>(plp + 4 * i, o);
    };
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
      const int64_t k = i + stride;
      const float4 ga = adam_ld((const float4*)g + i), pa = adam_ld((const float4*)p + i);
      const float4 ma = adam_ld((const float4*)m + i), va = adam_ld((const float4*)v + i);
      const float4 gb = adam_ld((const float4*)g + k), pb = adam_ld((const float4*)p + k);
      const float4 mb = adam_ld((const float4*)m + k), vb = adam_ld((const float4*)v + k);
      group(i, ga, pa, ma, va);
      group(k, gb, pb, mb, vb);
    }
    for (; i < n4; i += stride)
      group(i, adam_ld((const float4*)g + i), adam_ld((const float4*)p + i), adam_ld((const float4*)m + i),
            adam_ld((const float4*)v + i));
    done = n4 * 4;
  }
  for (int64_t i = done + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float mi = m[i], vi = v[i];
    const float pi = upd(g[i], p[i], mi, vi);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (plp) plp[i] = from_f<TL>(pi);
  }
}

extern "C" int lasr_sumsq_nparts(int64_t n) { return (int)cdiv(n, SQ_CHUNK); }

extern "C" int lasr_sumsq_partial(const float* g, int64_t n, float* ws, int64_t ws_floats,
                                  void* stream) {
  const int64_t np = cdiv(n, SQ_CHUNK);
  LASR_CHECK_ARG(ws_floats >= np, "lasr_sumsq_partial: workspace too small");
  if (np == 0) return LASR_OK;
  sumsq_partial_kernel<<<(unsigned)np, 256, 0, (hipStream_t)stream>>>(g, n, ws);
  return lasr_check_launch("sumsq_partial");
}

extern "C" int lasr_adam_step(float* param, void* param_lp, int lp_dtype, const float* grad,
                              float* m, float* v, int64_t n, const float* ws, int nparts,
                              float* state, float max_norm, int lr_mode, float lr, float factor,
                              float model_dim, float warmup, float beta1, float beta2, float eps,
                              float weight_decay, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  opt_finalize_kernel<<<1, 256, 0, st>>>(ws, nparts, state, max_norm, lr_mode, lr, factor,
                                         model_dim, warmup);
  int rc = lasr_check_launch("adam/finalize");
  if (rc || n <= 0) return rc;
  const unsigned g = (unsigned)std::min<int64_t>(cdiv(n, 256), 8192);
  if (param_lp && lp_dtype == LASR_BF16)
    adam_kernel<bf16_t><<<g, 256, 0, st>>>(param, (bf16_t*)param_lp, grad, m, v, n, state, beta1, beta2, eps, weight_decay);
  else
    adam_kernel<float><<<g, 256, 0, st>>>(param, (float*)param_lp, grad, m, v, n, state, beta1, beta2, eps, weight_decay);
  return lasr_check_launch("adam");
}
