// Transducer head (liteasr/models/transducer.py) and the RNN-T loss (liteasr/criterions/
// rnnt.py: warp-transducer / warp-rnnt, blank 0, batch mean, log-softmax applied to the raw
// joint logits).
//
//   rnnt_lse_gather_kernel : one wave per lattice row (b, t, u): log-sum-exp over V and the
//                            blank / next-label log-probs (rows past (T_b, U_b) skipped)
//   rnnt_alpha_beta_kernel : per utterance, the anti-diagonal wavefront over the (T_b, U_b+1)
//                            lattice, one thread per label position u; alpha blocks and
//                            beta blocks run side by side (2B workgroups)
//   rnnt_grad_kernel       : one wave per row: softmax * occupancy - (blank, label) terms,
//                            one coalesced write over V
//   joint_tanh_fwd_kernel  : z(b,t,u) = tanh(lin_enc(h_enc)(b,t) + lin_dec(h_dec)(u,b))
//   joint_reduce_kernels   : the joint's input gradients: sums of dz over u (encoder side)
//                            and over t (prediction-network side), fixed order
//   lstm_cell_fwd / bwd    : torch.nn.LSTMCell's gate arithmetic (rnn_decoder.py:49-67) around
//                            the recurrent GEMM the host issues per step
// The algorithm (Graves 2012, §2.3-2.5) is restated in oracle/rnnt_ref.py, which the tests
// pin by path enumeration and finite differences (the reference's own loss package is not
// available: parity against it is unpinned).
#include "common.h"

namespace {

LASR_DEV float lse2f(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

// ------------------------------------------------------------ lse + gather -------
template <typename TL>
__global__ __launch_bounds__(256) void rnnt_lse_gather_kernel(const TL* __restrict__ logits, int64_t ld, int B,
                                                              int T_, int U1, int V, const int32_t* __restrict__ targets,
                                                              int Lmax, const int32_t* ilen, const int32_t* tlen,
                                                              int blank, float* lse, float2* lp, bool vec) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * T_ * U1) return;
  const int lane = threadIdx.x & 63;
  const int u = (int)(row % U1);
  const int64_t bt = row / U1;
  const int t = (int)(bt % T_), b = (int)(bt / T_);
  const int Tb = ilen[b], Ub = tlen[b];
  if (t >= Tb || u > Ub) {  // outside the utterance's lattice: never read
    if (lane == 0) {
      lse[row] = 0.f;
      lp[row] = make_float2(0.f, -INFINITY);
    }
    return;
  }
  const TL* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  if (vec) {
    for (int c0 = lane * 8; c0 < V; c0 += 512) {
      if (c0 + 8 <= V) {
        float v[8];
        ldv<8>(x + c0, v);
        float mx = v[0];
#pragma unroll
        for (int q = 1; q < 8; ++q) mx = fmaxf(mx, v[q]);
        float e = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) e += __expf(v[q] - mx);
        if (mx > m) { s = s * __expf(m - mx) + e; m = mx; }
        else s += e * __expf(mx - m);
      } else {
        for (int c = c0; c < V; ++c) {
          const float v = to_f(x[c]);
          if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
          else s += __expf(v - m);
        }
      }
    }
  } else {
    for (int c = lane; c < V; c += 64) {
      const float v = to_f(x[c]);
      if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
      else s += __expf(v - m);
    }
  }
  const float M = wave_max(m);
  const float S = wave_sum(m == -INFINITY ? 0.f : s * __expf(m - M));
  const float l = M + __logf(S);
  if (lane == 0) {
    lse[row] = l;
    const float ly = u < Ub ? to_f(x[targets[(int64_t)b * Lmax + u]]) - l : -INFINITY;
    lp[row] = make_float2(to_f(x[blank]) - l, ly);
  }
}

// ---------------------------------------------------------------- lattice --------
// Diagonal n holds the nodes t + u = n; thread u owns node (n - u, u).  Each step needs the
// previous diagonal (LDS, ping-pong) and emission log-probs that are known ahead of time,
// so they are prefetched RN_PF diagonals ahead into a register ring (off the serial chain).
constexpr int RN_PF = 4;

__global__ void rnnt_alpha_beta_kernel(int B, int T_, int U1, const int32_t* ilen, const int32_t* tlen,
                                       const float2* __restrict__ lp, float* alpha, float* beta, float* nll) {
  extern __shared__ float sh[];  // two diagonals of U1 + 1 entries
  const bool isb = blockIdx.x >= (unsigned)B;
  const int b = isb ? blockIdx.x - B : blockIdx.x;
  const int Tb = ilen[b], Ub = tlen[b];
  const int u = threadIdx.x;
  float* d0 = sh;
  float* d1 = sh + U1 + 1;
  for (int i = threadIdx.x; i < 2 * (U1 + 1); i += blockDim.x) sh[i] = -INFINITY;
  if (Tb <= 0) {  // no frames: no alignment (warp-transducer requires T >= 1)
    if (!isb && threadIdx.x == 0) nll[b] = INFINITY;
    return;
  }
  const float2* lpu = lp + (int64_t)b * T_ * U1;
  float* out = (isb ? beta : alpha) + (int64_t)b * T_ * U1;
  const int ND = Tb + Ub;  // diagonals 0 .. ND-1
  const bool act = u <= Ub;
  __syncthreads();
  float* prev = d0;
  float* cur = d1;
  if (!isb) {
    // alpha(t,u) = lse(alpha(t-1,u) + lpb(t-1,u), alpha(t,u-1) + lpy(t,u-1))
    auto fetch = [&](int n, float& eb, float& ey) {
      const int t = n - u;
      eb = (act && t >= 1 && t < Tb) ? lpu[(int64_t)(t - 1) * U1 + u].x : -INFINITY;
      ey = (act && u >= 1 && t >= 0 && t < Tb) ? lpu[(int64_t)t * U1 + u - 1].y : -INFINITY;
    };
    float rb[RN_PF], ry[RN_PF];
#pragma unroll
    for (int k = 0; k < RN_PF; ++k) fetch(k, rb[k], ry[k]);
    for (int n0 = 0; n0 < ND; n0 += RN_PF) {
#pragma unroll
      for (int k = 0; k < RN_PF; ++k) {
        const int n = n0 + k;
        if (n >= ND) break;  // uniform
        const float eb = rb[k], ey = ry[k];
        fetch(n + RN_PF, rb[k], ry[k]);
        const int t = n - u;
        float v = -INFINITY;
        if (act && t >= 0 && t < Tb) {
          v = n == 0 ? 0.f : lse2f(prev[u] + eb, (u > 0 ? prev[u - 1] : -INFINITY) + ey);
          out[(int64_t)t * U1 + u] = v;
        }
        if (u < U1) cur[u] = v;
        __syncthreads();
        float* tmp = prev; prev = cur; cur = tmp;
      }
    }
    if (u == Ub) nll[b] = -(prev[Ub] + lpu[(int64_t)(Tb - 1) * U1 + Ub].x);
  } else {
    // beta(t,u) = lse(beta(t+1,u) + lpb(t,u), beta(t,u+1) + lpy(t,u)); beta(Tb-1,Ub) = lpb
    auto fetch = [&](int n, float2& e) {
      const int t = n - u;
      e = (act && n >= 0 && t >= 0 && t < Tb) ? lpu[(int64_t)t * U1 + u] : make_float2(-INFINITY, -INFINITY);
    };
    float2 re[RN_PF];
#pragma unroll
    for (int k = 0; k < RN_PF; ++k) fetch(ND - 1 - k, re[k]);
    for (int n0 = ND - 1; n0 >= 0; n0 -= RN_PF) {
#pragma unroll
      for (int k = 0; k < RN_PF; ++k) {
        const int n = n0 - k;
        if (n < 0) break;  // uniform
        const float2 e = re[k];
        fetch(n - RN_PF, re[k]);
        const int t = n - u;
        float v = -INFINITY;
        if (act && t >= 0 && t < Tb) {
          if (t == Tb - 1 && u == Ub) v = e.x;
          else v = lse2f((t + 1 < Tb ? prev[u] : -INFINITY) + e.x, (u < Ub ? prev[u + 1] : -INFINITY) + e.y);
          out[(int64_t)t * U1 + u] = v;
        }
        if (u < U1) cur[u] = v;
        __syncthreads();
        float* tmp = prev; prev = cur; cur = tmp;
      }
    }
  }
}

// -------------------------------------------------------------------- grad -------
template <typename TL, typename TG>
__global__ __launch_bounds__(256) void rnnt_grad_kernel(const TL* __restrict__ logits, int64_t ld, int B, int T_,
                                                        int U1, int V, const int32_t* __restrict__ targets, int Lmax,
                                                        const int32_t* ilen, const int32_t* tlen, int blank,
                                                        const float* lse, const float2* lp, const float* alpha,
                                                        const float* beta, const float* nll, TG* grad, float gscale,
                                                        const float* gdev, bool vec) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * T_ * U1) return;
  const int lane = threadIdx.x & 63;
  const int u = (int)(row % U1);
  const int64_t bt = row / U1;
  const int t = (int)(bt % T_), b = (int)(bt / T_);
  const int Tb = ilen[b], Ub = tlen[b];
  TG* g = grad + row * ld;
  if (t >= Tb || u > Ub || !(nll[b] < INFINITY)) {
    for (int c = lane; c < V; c += 64) g[c] = from_f<TG>(0.f);
    return;
  }
  const float gs = gscale * (gdev ? gdev[0] : 1.f);
  const float lP = -nll[b];
  const float a = alpha[row], l = lse[row];
  const float2 e = lp[row];
  const float occ = __expf(a + beta[row] - lP);
  const float bn = t + 1 < Tb ? beta[row + U1] : (u == Ub ? 0.f : -INFINITY);
  const float cb = __expf(a + e.x + bn - lP);
  const float cy = u < Ub ? __expf(a + e.y + beta[row + 1] - lP) : 0.f;
  const int y = u < Ub ? targets[(int64_t)b * Lmax + u] : -1;
  const TL* x = logits + row * ld;
  auto gv = [&](int c, float xv) {
    float v = __expf(xv - l) * occ;
    if (c == blank) v -= cb;
    if (c == y) v -= cy;
    return gs * v;
  };
  if (vec) {
    for (int c0 = lane * 8; c0 < V; c0 += 512) {
      if (c0 + 8 <= V) {
        float v[8];
        ldv<8>(x + c0, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = gv(c0 + q, v[q]);
        stv<8>(g + c0, v);
      } else {
        for (int c = c0; c < V; ++c) g[c] = from_f<TG>(gv(c, to_f(x[c])));
      }
    }
  } else {
    for (int c = lane; c < V; c += 64) g[c] = from_f<TG>(gv(c, to_f(x[c])));
  }
}

// ------------------------------------------------------------------- joint -------
// z[((b T + t) U1 + u) J + j] = tanh(e[(b T + t) J + j] + d[(u B + b) J + j]); d is
// time-major (the prediction network runs [U1][B] rows).  J % 8 == 0.
template <typename TZ>
__global__ void joint_tanh_fwd_kernel(const float* __restrict__ e, const float* __restrict__ d, int B, int T_,
                                      int U1, int J, TZ* z) {
  const int J8 = J / 8;
  const int64_t n = (int64_t)B * T_ * U1 * J8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % J8) * 8;
    const int64_t row = i / J8;
    const int u = (int)(row % U1);
    const int64_t bt = row / U1;
    const int b = (int)(bt / T_);
    float ev[8], dv[8];
    ldv<8>(e + bt * J + j, ev);
    ldv<8>(d + ((int64_t)u * B + b) * J + j, dv);
#pragma unroll
    for (int q = 0; q < 8; ++q) ev[q] = tanhf(ev[q] + dv[q]);
    stv<8>(z + row * J + j, ev);
  }
}

// de[(b T + t), j] = sum_u dz[((b T + t) U1 + u), j]   (one thread per (bt, j), u in order)
template <typename TZ, typename TO>
__global__ void joint_reduce_enc_kernel(const TZ* __restrict__ dz, int64_t BT, int U1, int J, TO* de) {
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  const int64_t bt = blockIdx.x;
  if (j >= J || bt >= BT) return;
  const TZ* p = dz + bt * U1 * J + j;
  float s = 0.f;
  for (int u = 0; u < U1; ++u) s += to_f(p[(int64_t)u * J]);
  de[bt * J + j] = from_f<TO>(s);
}
// dd[(u B + b), j] = sum_t dz[((b T + t) U1 + u), j]   (4 interleaved partial sums over t,
// combined in a fixed order)
template <typename TZ, typename TO>
__global__ void joint_reduce_dec_kernel(const TZ* __restrict__ dz, int B, int T_, int U1, int J, TO* dd) {
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  const int ub = blockIdx.x, u = ub / B, b = ub % B;
  if (j >= J || u >= U1) return;
  const TZ* p = dz + ((int64_t)b * T_ * U1 + u) * J + j;
  const int64_t st = (int64_t)U1 * J;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int t = 0;
  for (; t + 4 <= T_; t += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] += to_f(p[(t + q) * st]);
  }
  for (; t < T_; ++t) s[0] += to_f(p[t * st]);
  dd[(int64_t)ub * J + j] = from_f<TO>((s[0] + s[1]) + (s[2] + s[3]));
}

// -------------------------------------------------------------------- LSTM -------
// torch.nn.LSTMCell (rnn_decoder.py:21-24,49-67): gates = x W_ih^T + b_ih + h W_hh^T + b_hh
// (pre-activations, fp32, chunks i | f | g | o), c = sigm(f) c_prev + sigm(i) tanh(g),
// h = sigm(o) tanh(c).  One thread per (b, j).
LASR_DEV float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// bias (nullable, [4H]): a second bias added to every row's gates (b_hh when the input GEMM
// carried b_ih)
LASR_DEV void lstm_gates(const float* g, const float* bias, int H, int j, float& ig, float& fg, float& gg, float& og) {
  float a = g[j], f = g[H + j], c = g[2 * H + j], o = g[3 * H + j];
  if (bias) { a += bias[j]; f += bias[H + j]; c += bias[2 * H + j]; o += bias[3 * H + j]; }
  ig = sigm(a); fg = sigm(f); gg = tanhf(c); og = sigm(o);
}

template <typename TH>
__global__ void lstm_cell_fwd_kernel(const float* __restrict__ gates, int64_t ldg, const float* bias,
                                     const float* c_prev, int B, int H, float* c_out, TH* h_out, int64_t ldh) {
  const int64_t n = (int64_t)B * H;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / H), j = (int)(i % H);
    float ig, fg, gg, og;
    lstm_gates(gates + b * ldg, bias, H, j, ig, fg, gg, og);
    const float c = fg * (c_prev ? c_prev[i] : 0.f) + ig * gg;
    c_out[i] = c;
    h_out[b * ldh + j] = from_f<TH>(og * tanhf(c));
  }
}

// dh = dh_out (+ dh_rec); dc = dc_next + dh o (1 - tanh(c)^2); dgates (pre-activation):
// di = dc g i (1-i), df = dc c_prev f (1-f), dg = dc i (1 - g^2), do = dh tanh(c) o (1-o);
// dc_prev = dc f.
template <typename TD, typename TG>
__global__ void lstm_cell_bwd_kernel(const float* __restrict__ gates, int64_t ldg, const float* bias, const float* c,
                                     const float* c_prev, const TD* dh_out, int64_t lddh, const float* dh_rec,
                                     const float* dc_next, int B, int H, TG* dgates, int64_t lddg, float* dc_prev) {
  const int64_t n = (int64_t)B * H;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / H), j = (int)(i % H);
    float ig, fg, gg, og;
    lstm_gates(gates + b * ldg, bias, H, j, ig, fg, gg, og);
    const float tc = tanhf(c[i]);
    float dh = dh_out ? to_f(dh_out[b * lddh + j]) : 0.f;
    if (dh_rec) dh += dh_rec[i];
    const float dc = (dc_next ? dc_next[i] : 0.f) + dh * og * (1.f - tc * tc);
    const float cp = c_prev ? c_prev[i] : 0.f;
    TG* dg = dgates + b * lddg;
    dg[j] = from_f<TG>(dc * gg * ig * (1.f - ig));
    dg[H + j] = from_f<TG>(dc * cp * fg * (1.f - fg));
    dg[2 * H + j] = from_f<TG>(dc * ig * (1.f - gg * gg));
    dg[3 * H + j] = from_f<TG>(dh * tc * og * (1.f - og));
    if (dc_prev) dc_prev[i] = dc * fg;
  }
}

unsigned gridn(int64_t n) { return (unsigned)std::min<int64_t>(cdiv(n, 256), 16384); }
bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int lasr_rnnt_fwd(const void* logits, int ldt, int B, int T, int U1, int V, int64_t ld,
                             const int32_t* targets, int Lmax, const int32_t* ilen, const int32_t* tlen, int blank,
                             float* lse, float* lp, float* alpha, float* beta, float* nll, void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && U1 > 0 && V > 0 && ld >= V && Lmax >= U1 - 1, "lasr_rnnt_fwd: bad sizes");
  LASR_CHECK_ARG(U1 <= 1024, "lasr_rnnt_fwd: U+1 = %d > 1024 (one lattice column per thread)", U1);
  LASR_CHECK_ARG(ldt == LASR_F32 || ldt == LASR_BF16, "lasr_rnnt_fwd: bad dtype");
  LASR_CHECK_ARG(blank >= 0 && blank < V, "lasr_rnnt_fwd: blank out of range");
  LASR_CHECK_ARG(logits && lse && lp && alpha && beta && nll, "lasr_rnnt_fwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * T * U1;
  const bool vec = ld % 8 == 0 && al16(logits);
  if (ldt == LASR_F32)
    rnnt_lse_gather_kernel<float><<<(unsigned)cdiv(rows, 4), 256, 0, st>>>(
        (const float*)logits, ld, B, T, U1, V, targets, Lmax, ilen, tlen, blank, lse, (float2*)lp, vec);
  else
    rnnt_lse_gather_kernel<bf16_t><<<(unsigned)cdiv(rows, 4), 256, 0, st>>>(
        (const bf16_t*)logits, ld, B, T, U1, V, targets, Lmax, ilen, tlen, blank, lse, (float2*)lp, vec);
  int rc = lasr_check_launch("rnnt_lse_gather");
  if (rc) return rc;
  const int nt = (int)std::min<int64_t>(1024, std::max<int64_t>(64, cdiv(U1, 64) * 64));
  rnnt_alpha_beta_kernel<<<2 * B, nt, 2 * (U1 + 1) * sizeof(float), st>>>(B, T, U1, ilen, tlen, (const float2*)lp,
                                                                          alpha, beta, nll);
  return lasr_check_launch("rnnt_alpha_beta");
}

extern "C" int lasr_rnnt_bwd(const void* logits, int ldt, int B, int T, int U1, int V, int64_t ld,
                             const int32_t* targets, int Lmax, const int32_t* ilen, const int32_t* tlen, int blank,
                             const float* lse, const float* lp, const float* alpha, const float* beta,
                             const float* nll, void* grad, int gdt, float gscale, const float* gdev, void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && U1 > 0 && V > 0 && ld >= V && Lmax >= U1 - 1, "lasr_rnnt_bwd: bad sizes");
  LASR_CHECK_ARG(logits && grad && lse && lp && alpha && beta && nll, "lasr_rnnt_bwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * T * U1;
  const bool vec = ld % 8 == 0 && al16(logits) && al16(grad);
#define RG(TL, TG)                                                                                          \
  rnnt_grad_kernel<TL, TG><<<(unsigned)cdiv(rows, 4), 256, 0, st>>>((const TL*)logits, ld, B, T, U1, V, targets, \
                                                                    Lmax, ilen, tlen, blank, lse,            \
                                                                    (const float2*)lp, alpha, beta, nll,     \
                                                                    (TG*)grad, gscale, gdev, vec)
  if (ldt == LASR_F32 && gdt == LASR_F32) RG(float, float);
  else if (ldt == LASR_F32) RG(float, bf16_t);
  else if (gdt == LASR_F32) RG(bf16_t, float);
  else RG(bf16_t, bf16_t);
#undef RG
  return lasr_check_launch("rnnt_grad");
}

extern "C" int lasr_joint_fwd(const float* e, const float* d, int B, int T, int U1, int J, void* z, int zdt,
                              void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && U1 > 0 && J > 0 && J % 8 == 0, "lasr_joint_fwd: bad sizes (J %% 8 == 0)");
  LASR_CHECK_ARG(al16(e) && al16(d) && al16(z), "lasr_joint_fwd: 16-B alignment");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)B * T * U1 * (J / 8);
  if (zdt == LASR_F32) joint_tanh_fwd_kernel<float><<<gridn(n), 256, 0, st>>>(e, d, B, T, U1, J, (float*)z);
  else joint_tanh_fwd_kernel<bf16_t><<<gridn(n), 256, 0, st>>>(e, d, B, T, U1, J, (bf16_t*)z);
  return lasr_check_launch("joint_fwd");
}

extern "C" int lasr_joint_reduce(const void* dz, int dzdt, int B, int T, int U1, int J, void* de, void* dd, int odt,
                                 void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && U1 > 0 && J > 0, "lasr_joint_reduce: bad sizes");
  LASR_CHECK_ARG(dz && de && dd, "lasr_joint_reduce: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const dim3 ge((unsigned)((int64_t)B * T), (unsigned)cdiv(J, 256)), gd((unsigned)(B * U1), (unsigned)cdiv(J, 256));
#define JR(TZ, TO)                                                                                              \
  do {                                                                                                          \
    joint_reduce_enc_kernel<TZ, TO><<<ge, 256, 0, st>>>((const TZ*)dz, (int64_t)B * T, U1, J, (TO*)de);          \
    joint_reduce_dec_kernel<TZ, TO><<<gd, 256, 0, st>>>((const TZ*)dz, B, T, U1, J, (TO*)dd);                    \
  } while (0)
  if (dzdt == LASR_F32 && odt == LASR_F32) JR(float, float);
  else if (dzdt == LASR_F32) JR(float, bf16_t);
  else if (odt == LASR_F32) JR(bf16_t, float);
  else JR(bf16_t, bf16_t);
#undef JR
  return lasr_check_launch("joint_reduce");
}

extern "C" int lasr_lstm_cell_fwd(const float* gates, int64_t ldg, const float* bias, const float* c_prev, int B, int H,
                                  float* c_out, void* h_out, int hdt, int64_t ldh, void* stream) {
  LASR_CHECK_ARG(B > 0 && H > 0 && ldg >= 4 * H && ldh >= H, "lasr_lstm_cell_fwd: bad sizes");
  LASR_CHECK_ARG(gates && c_out && h_out, "lasr_lstm_cell_fwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)B * H;
  if (hdt == LASR_F32)
    lstm_cell_fwd_kernel<float><<<gridn(n), 256, 0, st>>>(gates, ldg, bias, c_prev, B, H, c_out, (float*)h_out, ldh);
  else
    lstm_cell_fwd_kernel<bf16_t><<<gridn(n), 256, 0, st>>>(gates, ldg, bias, c_prev, B, H, c_out, (bf16_t*)h_out, ldh);
  return lasr_check_launch("lstm_cell_fwd");
}

extern "C" int lasr_lstm_cell_bwd(const float* gates, int64_t ldg, const float* bias, const float* c,
                                  const float* c_prev, const void* dh_out, int dhdt, int64_t lddh, const float* dh_rec,
                                  const float* dc_next, int B, int H, void* dgates, int gdt, int64_t lddg,
                                  float* dc_prev, void* stream) {
  LASR_CHECK_ARG(B > 0 && H > 0 && ldg >= 4 * H && lddg >= 4 * H, "lasr_lstm_cell_bwd: bad sizes");
  LASR_CHECK_ARG(gates && c && dgates, "lasr_lstm_cell_bwd: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)B * H;
#define LB(TD, TG)                                                                                            \
  lstm_cell_bwd_kernel<TD, TG><<<gridn(n), 256, 0, st>>>(gates, ldg, bias, c, c_prev, (const TD*)dh_out, lddh,    \
                                                         dh_rec, dc_next, B, H, (TG*)dgates, lddg, dc_prev)
  if (dhdt == LASR_BF16 && gdt == LASR_BF16) LB(bf16_t, bf16_t);
  else if (dhdt == LASR_BF16) LB(bf16_t, float);
  else if (gdt == LASR_BF16) LB(float, bf16_t);
  else LB(float, float);
#undef LB
  return lasr_check_launch("lstm_cell_bwd");
}
