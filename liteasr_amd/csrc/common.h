// Shared device helpers for the liteasr_amd HIP kernels (gfx950 / CDNA4).
// Storage types: fp32 (`float`) and bf16 (`bf16_t`, raw 16-bit); all arithmetic
// is done in fp32.  Wave = 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/liteasr_hip.h"

typedef uint16_t bf16_t;

#define LASR_DEV __device__ __forceinline__

LASR_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
LASR_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, b);
}

// Two floats -> one dword of two bf16 (low = a), one v_cvt_pk_bf16_f32 (RNE, as f2bf): packing
// two f2bf results with shifts / ors made the compiler convert, split and re-merge halves.
typedef float lasr_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 lasr_bf2 __attribute__((ext_vector_type(2)));
LASR_DEV uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((lasr_f2){a, b}, lasr_bf2));
}

LASR_DEV float to_f(float x) { return x; }
LASR_DEV float to_f(bf16_t x) { return bf2f(x); }
template <typename T> LASR_DEV T from_f(float x);
template <> LASR_DEV float from_f<float>(float x) { return x; }
template <> LASR_DEV bf16_t from_f<bf16_t>(float x) { return f2bf(x); }

template <typename T> LASR_DEV float ldf(const T* p, int64_t i) { return to_f(p[i]); }
template <typename T> LASR_DEV void stf(T* p, int64_t i, float v) { p[i] = from_f<T>(v); }

// ---- 8-wide vector load/store (16-B aligned for bf16, 32-B for fp32) ----------
LASR_DEV void ld8(const float* p, float v[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
LASR_DEV void ld8(const bf16_t* p, float v[8]) {
  const uint4 u = *(const uint4*)p;
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
LASR_DEV void st8(float* p, const float v[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
LASR_DEV void st8(bf16_t* p, const float v[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pk_bf16(v[2 * i], v[2 * i + 1]);
  *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
}

// N consecutive elements (N in 1,2,4,8,16; pointer aligned to N elements) <-> fp32.
template <int N>
LASR_DEV void ldv(const float* p, float* v) {
  if constexpr (N == 1) v[0] = p[0];
  else if constexpr (N == 2) { const float2 a = *(const float2*)p; v[0] = a.x; v[1] = a.y; }
  else {
#pragma unroll
    for (int j = 0; j < N; j += 4) {
      const float4 a = *(const float4*)(p + j);
      v[j] = a.x; v[j + 1] = a.y; v[j + 2] = a.z; v[j + 3] = a.w;
    }
  }
}
template <int N>
LASR_DEV void ldv(const bf16_t* p, float* v) {
  if constexpr (N == 1) v[0] = bf2f(p[0]);
  else if constexpr (N == 2) {
    const uint32_t w = *(const uint32_t*)p;
    v[0] = __uint_as_float(w << 16); v[1] = __uint_as_float(w & 0xFFFF0000u);
  } else if constexpr (N == 4) {
    const uint2 w = *(const uint2*)p;
    v[0] = __uint_as_float(w.x << 16); v[1] = __uint_as_float(w.x & 0xFFFF0000u);
    v[2] = __uint_as_float(w.y << 16); v[3] = __uint_as_float(w.y & 0xFFFF0000u);
  } else {
#pragma unroll
    for (int j = 0; j < N; j += 8) ld8(p + j, v + j);
  }
}
template <int N>
LASR_DEV void stv(float* p, const float* v) {
  if constexpr (N == 1) p[0] = v[0];
  else if constexpr (N == 2) *(float2*)p = make_float2(v[0], v[1]);
  else {
#pragma unroll
    for (int j = 0; j < N; j += 4) *(float4*)(p + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  }
}
template <int N>
LASR_DEV void stv(bf16_t* p, const float* v) {
  if constexpr (N == 1) p[0] = f2bf(v[0]);
  else if constexpr (N == 2) *(uint32_t*)p = pk_bf16(v[0], v[1]);
  else if constexpr (N == 4)
    *(uint2*)p = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
  else {
#pragma unroll
    for (int j = 0; j < N; j += 8) st8(p + j, v + j);
  }
}

// ---- wave (64-lane) reductions ------------------------------------------------
LASR_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
LASR_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
LASR_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block reduction (blockDim.x multiple of 64, <= 1024). `red` holds >= 16 floats.
LASR_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += red[i];  // fixed order -> deterministic
  return r;
}
LASR_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
  return r;
}

// ---- counter-based dropout RNG -----------------------------------------------
// keep(seed, idx) is a pure function of (seed, device step counter, logical element
// index), so the backward pass regenerates the forward mask instead of storing it.
// One 32-bit draw serves a PAIR of elements (2k, 2k+1: its low / high 16 bits); element
// idx is kept iff its 16-bit half >= thr = round(p * 65536), and kept values are scaled
// by 65536 / (65536 - thr), so E[mask * scale] = 1 exactly (p is realised to 2^-16).
struct DropCfg {
  float p;              // drop probability (0 = off)
  uint32_t thr;         // 16-bit keep threshold
  float scale;          // multiplier of kept elements
  uint64_t seed;        // per-site seed (host)
  const uint64_t* ctr;  // optional device step counter (read at run time, graph-safe)
};
// Host: the process-wide device counter registered by lasr_set_dropout_counter().
const uint64_t* lasr_dropout_counter();
static inline DropCfg mkdrop(float p, uint64_t seed) {
  DropCfg d;
  d.p = p;
  d.seed = seed;
  d.ctr = p > 0.f ? lasr_dropout_counter() : nullptr;
  uint32_t thr = 0;
  if (p > 0.f) {
    const float t = p * 65536.f + 0.5f;
    thr = t >= 65536.f ? 65536u : (uint32_t)t;
  }
  d.thr = thr;
  d.scale = thr >= 65536u ? 0.f : 65536.f / (float)(65536u - thr);
  return d;
}
// 32-bit finaliser (lowbias32: 2 multiplies, 3 xor-shifts).
LASR_DEV uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// Per-site/step key (wave-uniform: derived from kernel args + the device counter).
LASR_DEV uint32_t drop_key(const DropCfg& d) {
  const uint64_t s = d.seed + (d.ctr ? d.ctr[0] * 0xD1B54A32D192ED03ull : 0ull);
  return mix32((uint32_t)s ^ mix32((uint32_t)(s >> 32) + 0x9E3779B9u));
}
// The draw of element pair k (elements 2k and 2k+1).
LASR_DEV uint32_t drop_bits(uint32_t key, uint64_t pair) {
  const uint32_t hi = (uint32_t)(pair >> 32);
  return mix32((uint32_t)pair ^ key ^ ((hi << 16) | (hi >> 16)));
}
// 1 (kept) or 0 for element idx.
LASR_DEV float drop_keep_k(const DropCfg& d, uint32_t key, uint64_t idx) {
  const uint32_t b = drop_bits(key, idx >> 1);
  const uint32_t h = (idx & 1) ? (b >> 16) : (b & 0xFFFFu);
  return h >= d.thr ? 1.f : 0.f;
}
// Multiplier of element idx (0 or scale).
LASR_DEV float drop_mul_k(const DropCfg& d, uint32_t key, uint64_t idx) {
  return drop_keep_k(d, key, idx) * d.scale;
}
// Keep flags (1 / 0) of the N consecutive elements idx0 .. idx0+N-1, one draw per pair
// when idx0 is even (the vector epilogues' case).
template <int N>
LASR_DEV void drop_keep_n(const DropCfg& d, uint32_t key, uint64_t idx0, float* k) {
  if (idx0 & 1) {
#pragma unroll
    for (int q = 0; q < N; ++q) k[q] = drop_keep_k(d, key, idx0 + q);
    return;
  }
#pragma unroll
  for (int q = 0; q < N; q += 2) {
    const uint32_t b = drop_bits(key, (idx0 >> 1) + (q >> 1));
    k[q] = (b & 0xFFFFu) >= d.thr ? 1.f : 0.f;
    if (q + 1 < N) k[q + 1] = (b >> 16) >= d.thr ? 1.f : 0.f;
  }
}
// The same keep flags as a bit mask (bit q = element idx0 + q), N <= 32.
template <int N>
LASR_DEV uint32_t drop_keep_mask(const DropCfg& d, uint32_t key, uint64_t idx0) {
  uint32_t km = 0u;
  if (idx0 & 1) {
#pragma unroll
    for (int q = 0; q < N; ++q) km |= (drop_keep_k(d, key, idx0 + q) != 0.f ? 1u : 0u) << q;
    return km;
  }
#pragma unroll
  for (int q = 0; q < N; q += 2) {
    const uint32_t b = drop_bits(key, (idx0 >> 1) + (q >> 1));
    km |= ((b & 0xFFFFu) >= d.thr ? 1u : 0u) << q;
    if (q + 1 < N) km |= ((b >> 16) >= d.thr ? 1u : 0u) << (q + 1);
  }
  return km;
}
// The same for an even idx0 (the specialised vector epilogues: N % 8 == 0 host-checked, so a
// row's 8-column vector starts on an even element): no per-element fallback code.
template <int N>
LASR_DEV uint32_t drop_keep_mask_even(const DropCfg& d, uint32_t key, uint64_t idx0) {
  static_assert(N % 2 == 0, "pairs");
  uint32_t km = 0u;
  const uint64_t pair0 = idx0 >> 1;
#pragma unroll
  for (int q = 0; q < N; q += 2) {
    const uint32_t b = drop_bits(key, pair0 + (q >> 1));
    km |= ((b & 0xFFFFu) >= d.thr ? 1u : 0u) << q;
    km |= ((b >> 16) >= d.thr ? 1u : 0u) << (q + 1);
  }
  return km;
}
template <int N>
LASR_DEV void drop_mul_n(const DropCfg& d, uint32_t key, uint64_t idx0, float* m) {
  drop_keep_n<N>(d, key, idx0, m);
#pragma unroll
  for (int q = 0; q < N; ++q) m[q] *= d.scale;
}
// Key / multiplier pair for loops: take the key once before the loop (drop_key reads the
// device step counter; inside a loop with stores that load is re-issued every iteration).
LASR_DEV uint32_t drop_key_if(const DropCfg& d) { return d.p > 0.f ? drop_key(d) : 0u; }
LASR_DEV float drop_mul_if(const DropCfg& d, uint32_t key, uint64_t idx) {
  return d.p > 0.f ? drop_mul_k(d, key, idx) : 1.f;
}
// Multiplier for element idx; 1 when dropout is off (one element: loops use the pair above).
LASR_DEV float drop_mul(const DropCfg& d, uint64_t idx) {
  if (d.p <= 0.f) return 1.f;
  return drop_mul_k(d, drop_key(d), idx);
}

LASR_DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }  // v_rcp_f32 (1 ulp)
LASR_DEV float swishf(float x) { return x * sigmoidf_(x); }
LASR_DEV float swish_grad(float z) {
  const float s = sigmoidf_(z);
  return s * (1.f + z * (1.f - s));
}

// ---- error plumbing (defined in capi.cpp) ------------------------------------
void lasr_set_error(const char* fmt, ...);
int lasr_check_launch(const char* what);

#define LASR_CHECK_ARG(cond, ...)          \
  do {                                     \
    if (!(cond)) {                         \
      lasr_set_error(__VA_ARGS__);         \
      return LASR_ERR_INVALID;             \
    }                                      \
  } while (0)

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// reduce.hip: out[n] (+)= sum_p part[p*N+n]; columns >= split go to out1[n-split].
int lasr_reduce_cols(const float* part, int P, int64_t N, float* out0, float* out1, int64_t split,
                     int accumulate, hipStream_t st);
// dst[c*ld+k] += src[k*C+c] (k<K); bias[c] += src[K*C+c] when bias != nullptr.
int lasr_scatter_kc(const float* src, int K, int C, int ld, float* dst, float* bias,
                    hipStream_t st);
