// CTC loss (blank = 0, reduction = sum) fused with log_softmax over the vocabulary.
//
// Reference call site: liteasr/criterions/hybrid_ctc_attn.py:67-75
//   h_ctc.transpose(0,1).log_softmax(-1) -> nn.CTCLoss(reduction="sum")(..., get_pred_len(xlens), ylens)
// whose arithmetic lives in PyTorch aten (ctc_loss / _ctc_loss_backward).  The
// composed gradient w.r.t. the *logits* is softmax - gamma (gamma = posterior of the
// extended-label lattice), which is what lasr_ctc_bwd writes directly.
//
// Work split (per utterance b, lattice S_b = 2*L_b + 1 states):
//   ctc_lse_gather_kernel : one workgroup per (b,t) row: online max/sum-exp over V
//                           (one HBM read of the row) + gather of the L_b+1 label
//                           log-probs the lattice needs.
//   ctc_alpha_kernel      : one workgroup per utterance, threads over states, LDS
//                           ping-pong across the serial t recursion.
//   ctc_beta_kernel       : same, backward in t.
//   ctc_grad_kernel       : one workgroup per (b,t) row: gamma from alpha+beta (summed
//                           per distinct label once per row), then a single coalesced
//                           write of g*(softmax - gamma) over V.
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void ctc_lse_gather_kernel(const T* __restrict__ logits, int B,
                                                             int T_, int V, int64_t ld,
                                                             const int32_t* __restrict__ targets,
                                                             int Lmax, const int32_t* ilen,
                                                             const int32_t* tlen, float* lse,
                                                             float* lp) {
  __shared__ float red[32];
  const int row = blockIdx.x;
  const int b = row / T_, t = row - b * T_;
  float* lprow = lp + (int64_t)row * (Lmax + 1);
  const int Tb = ilen[b];
  if (t >= Tb) {  // rows past the input length never enter the lattice
    if (threadIdx.x == 0) lse[row] = 0.f;
    for (int j = threadIdx.x; j <= Lmax; j += blockDim.x) lprow[j] = 0.f;
    return;
  }
  const T* x = logits + (int64_t)row * ld;
  float m = -INFINITY, s = 0.f;
  auto acc = [&](float v) {
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
  };
  if (ld % 8 == 0 && ((uintptr_t)logits & 15) == 0) {  // 16-B loads, 8 columns per thread
    for (int c0 = threadIdx.x * 8; c0 < V; c0 += blockDim.x * 8) {
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
        for (int c = c0; c < V; ++c) acc(to_f(x[c]));
      }
    }
  } else {
    for (int c = threadIdx.x; c < V; c += blockDim.x) acc(to_f(x[c]));
  }
  const float M = block_max(m, red);
  const float S = block_sum(m == -INFINITY ? 0.f : s * __expf(m - M), red + 16);
  const float l = M + __logf(S);
  if (threadIdx.x == 0) lse[row] = l;
  const int Lb = tlen[b];
  for (int j = threadIdx.x; j <= Lmax; j += blockDim.x) {
    float v = 0.f;
    if (j == 0) v = to_f(x[0]) - l;
    else if (j <= Lb) v = to_f(x[targets[(int64_t)b * Lmax + (j - 1)]]) - l;
    lprow[j] = v;
  }
}

LASR_DEV float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}
LASR_DEV float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

// label id of extended state s (blank for even s)
LASR_DEV int ext_label(const int32_t* tg, int s) { return (s & 1) ? tg[s >> 1] : 0; }

// The recursions run one state per thread (S <= blockDim <= 1024).  Everything a step
// needs from HBM is off the serial chain: the skip rule is decided once, and each
// thread's emission log-probs are prefetched CTC_PF steps ahead into a register ring.
constexpr int CTC_PF = 8;

LASR_DEV void ctc_alpha(int b, int T_, int Lmax, const int32_t* __restrict__ targets,
                        const int32_t* ilen, const int32_t* tlen, const float* lp, float* alpha,
                        float* nll) {
  extern __shared__ float sh[];
  const int Tb = ilen[b], Lb = tlen[b], S = 2 * Lb + 1, Smax = 2 * Lmax + 1;
  const int32_t* tg = targets + (int64_t)b * Lmax;
  float* buf0 = sh;
  float* buf1 = sh + Smax;
  if (Tb <= 0) {
    if (threadIdx.x == 0) nll[b] = (Lb == 0) ? 0.f : INFINITY;
    return;
  }
  const int s = threadIdx.x;
  const bool act = s < S;
  const bool skip = act && s >= 2 && (s & 1) && ext_label(tg, s) != ext_label(tg, s - 2);
  const int eix = (s & 1) ? 1 + (s >> 1) : 0;
  const int64_t ld = Lmax + 1;
  const float* lpb = lp + (int64_t)b * T_ * ld + eix;
  float* al = alpha + (int64_t)b * T_ * Smax;
  if (act) {
    const float v = (s == 0) ? lpb[0] : (s == 1) ? lpb[0] : -INFINITY;
    buf0[s] = v;
    al[s] = v;
  }
  float epf[CTC_PF];
#pragma unroll
  for (int k = 0; k < CTC_PF; ++k) epf[k] = (act && 1 + k < Tb) ? lpb[(1 + k) * ld] : 0.f;
  __syncthreads();
  float* prev = buf0;
  float* cur = buf1;
  for (int t0 = 1; t0 < Tb; t0 += CTC_PF) {
#pragma unroll
    for (int k = 0; k < CTC_PF; ++k) {
      const int t = t0 + k;
      if (t >= Tb) break;  // uniform
      const float e = epf[k];
      epf[k] = (act && t + CTC_PF < Tb) ? lpb[(t + CTC_PF) * ld] : 0.f;
      if (act) {
        const float a0 = prev[s];
        const float a1 = s >= 1 ? prev[s - 1] : -INFINITY;
        const float a2 = skip ? prev[s - 2] : -INFINITY;
        const float v = lse3(a0, a1, a2) + e;
        cur[s] = v;
        al[(int64_t)t * Smax + s] = v;
      }
      __syncthreads();
      float* tmp = prev; prev = cur; cur = tmp;
    }
  }
  if (threadIdx.x == 0) {
    const float ll = (S >= 2) ? lse2(prev[S - 1], prev[S - 2]) : prev[0];
    nll[b] = -ll;
  }
}

LASR_DEV void ctc_beta(int b, int T_, int Lmax, const int32_t* __restrict__ targets,
                       const int32_t* ilen, const int32_t* tlen, const float* lp, float* beta) {
  extern __shared__ float sh[];
  const int Tb = ilen[b], Lb = tlen[b], S = 2 * Lb + 1, Smax = 2 * Lmax + 1;
  if (Tb <= 0) return;
  const int32_t* tg = targets + (int64_t)b * Lmax;
  float* buf0 = sh;
  float* buf1 = sh + Smax;
  const int s = threadIdx.x;
  const bool act = s < S;
  const bool skip = act && s + 2 < S && (s & 1) && ext_label(tg, s) != ext_label(tg, s + 2);
  const int eix = (s & 1) ? 1 + (s >> 1) : 0;
  const int64_t ld = Lmax + 1;
  const float* lpb = lp + (int64_t)b * T_ * ld + eix;
  float* be = beta + (int64_t)b * T_ * Smax;
  if (act) {
    const float e = lpb[(int64_t)(Tb - 1) * ld];
    const float v = (s >= S - 2) ? e : -INFINITY;
    buf0[s] = v;
    be[(int64_t)(Tb - 1) * Smax + s] = v;
  }
  float epf[CTC_PF];
#pragma unroll
  for (int k = 0; k < CTC_PF; ++k) epf[k] = (act && Tb - 2 - k >= 0) ? lpb[(int64_t)(Tb - 2 - k) * ld] : 0.f;
  __syncthreads();
  float* nxt = buf0;
  float* cur = buf1;
  for (int t0 = Tb - 2; t0 >= 0; t0 -= CTC_PF) {
#pragma unroll
    for (int k = 0; k < CTC_PF; ++k) {
      const int t = t0 - k;
      if (t < 0) break;  // uniform
      const float e = epf[k];
      epf[k] = (act && t - CTC_PF >= 0) ? lpb[(int64_t)(t - CTC_PF) * ld] : 0.f;
      if (act) {
        const float b0 = nxt[s];
        const float b1 = (s + 1 < S) ? nxt[s + 1] : -INFINITY;
        const float b2 = skip ? nxt[s + 2] : -INFINITY;
        const float v = lse3(b0, b1, b2) + e;
        cur[s] = v;
        be[(int64_t)t * Smax + s] = v;
      }
      __syncthreads();
      float* tmp = nxt; nxt = cur; cur = tmp;
    }
  }
}

// blocks [0, B): alpha (+ nll); blocks [B, 2B) when beta != nullptr: beta.  The two
// recursions are independent, so the forward runs them side by side.
__global__ void ctc_alpha_beta_kernel(int B, int T_, int Lmax, const int32_t* __restrict__ targets,
                                      const int32_t* ilen, const int32_t* tlen, const float* lp,
                                      float* alpha, float* nll, float* beta) {
  if ((int)blockIdx.x < B) ctc_alpha(blockIdx.x, T_, Lmax, targets, ilen, tlen, lp, alpha, nll);
  else ctc_beta(blockIdx.x - B, T_, Lmax, targets, ilen, tlen, lp, beta);
}
__global__ void ctc_beta_kernel(int T_, int Lmax, const int32_t* __restrict__ targets,
                                const int32_t* ilen, const int32_t* tlen, const float* lp,
                                float* beta) {
  ctc_beta(blockIdx.x, T_, Lmax, targets, ilen, tlen, lp, beta);
}

// timing ablations (tools/gemm_exp.sh with EXP_FILES=ctc; 0 in the product): bit 1 skips the
// label-gamma scan, bit 2 the whole per-row preamble (blank sum, label posteriors, scan)
#ifndef LASR_EXP
#define LASR_EXP 0
#endif
template <typename T, typename TG>
__global__ __launch_bounds__(256) void ctc_grad_kernel(const T* __restrict__ logits, int B, int T_,
                                                       int V, int64_t ld,
                                                       const int32_t* __restrict__ targets,
                                                       int Lmax, const int32_t* ilen,
                                                       const int32_t* tlen, const float* lse,
                                                       const float* lp, const float* alpha,
                                                       const float* beta, const float* nll,
                                                       TG* grad, float gscale, const float* gdev) {
  // dynamic LDS: per label position (Lmax, rounded to 4) its posterior, label, first position
  // of its label, claim slot and running sum; [(V+31)/32] label bitmap; [V] gamma per
  // vocabulary entry (read only where the bitmap is set)
  extern __shared__ float sh[];
  __shared__ float red[32];
  const int L4 = (Lmax + 3) & ~3;
  float* glab = sh;
  int* lab = (int*)(sh + L4);
  int* fpos = (int*)(sh + 2 * L4);
  int* slot = (int*)(sh + 3 * L4);
  float* lsum = sh + 4 * L4;
  uint32_t* bits = (uint32_t*)(sh + 5 * L4);
  float* gam = sh + 5 * L4 + (V + 31) / 32;
  int* gpos = (int*)gam;  // the vocabulary table holds each label's first position first
  const int row = blockIdx.x;
  const int b = row / T_, t = row - b * T_;
  TG* g = grad + (int64_t)row * ld;
  const int Tb = ilen[b];
  // 8 columns per thread with 16-B accesses when the rows allow it (ld % 8, aligned base)
  const bool vec = ld % 8 == 0 && ((uintptr_t)logits & 15) == 0 && ((uintptr_t)grad & 15) == 0;
  if (t >= Tb) {
    if (vec) {
      const float z8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int c0 = threadIdx.x * 8; c0 < V; c0 += blockDim.x * 8) {
        if (c0 + 8 <= V) stv<8>(g + c0, z8);
        else for (int c = c0; c < V; ++c) g[c] = from_f<TG>(0.f);
      }
    } else {
      for (int c = threadIdx.x; c < V; c += blockDim.x) g[c] = from_f<TG>(0.f);
    }
    return;
  }
  const int Lb = tlen[b], S = 2 * Lb + 1, Smax = 2 * Lmax + 1;
  const float nl = nll[b];
  const float* a = alpha + ((int64_t)b * T_ + t) * Smax;
  const float* be = beta + ((int64_t)b * T_ + t) * Smax;
  const float* lpt = lp + (int64_t)row * (Lmax + 1);
  const int32_t* tg = targets + (int64_t)b * Lmax;
  // blank posterior: sum over even states
  float gb = 0.f;
  if (!(LASR_EXP & 2)) {
  for (int s = threadIdx.x * 2; s < S; s += blockDim.x * 2) gb += __expf(a[s] + be[s] + nl - lpt[0]);
  gb = block_sum(gb, red);
  }
  for (int w = threadIdx.x; w < (V + 31) / 32; w += blockDim.x) bits[w] = 0u;
  __syncthreads();
  for (int j = threadIdx.x; j < Lb && !(LASR_EXP & 2); j += blockDim.x) {
    const int s = 2 * j + 1;
    glab[j] = __expf(a[s] + be[s] + nl - lpt[1 + j]);
    lab[j] = tg[j];
    atomicOr(&bits[tg[j] >> 5], 1u << (tg[j] & 31));
  }
  __syncthreads();
  // gamma of each distinct label: the posteriors of the positions carrying it summed in
  // position order from 0 (the per-column loop of r02, done once per label).  Without a serial
  // scan of the label list: the first position of each label by an LDS atomicMin (an order-
  // independent result), then rounds in which every unclaimed position bids for its label's
  // slot with atomicMin; the round's winner -- the lowest unclaimed position of that label --
  // adds its posterior to the label's sum.  So the additions happen in position order, and a
  // label list without repeats takes one round.
  if (!(LASR_EXP & 3)) {
    for (int j = threadIdx.x; j < Lb; j += blockDim.x) gpos[lab[j]] = 0x7fffffff;
    __syncthreads();
    for (int j = threadIdx.x; j < Lb; j += blockDim.x) atomicMin(&gpos[lab[j]], j);
    __syncthreads();
    for (int j = threadIdx.x; j < Lb; j += blockDim.x) {
      fpos[j] = gpos[lab[j]];
      slot[j] = 0x7fffffff;
      lsum[j] = 0.f;
    }
    __syncthreads();
    uint32_t open = 0;  // bit k: position threadIdx.x + k * blockDim.x not yet summed
    for (int k = 0, j = threadIdx.x; j < Lb && k < 32; ++k, j += blockDim.x) open |= 1u << k;
    for (;;) {
      for (int k = 0, j = threadIdx.x; j < Lb && k < 32; ++k, j += blockDim.x)
        if ((open >> k) & 1u) atomicMin(&slot[fpos[j]], j);
      __syncthreads();
      for (int k = 0, j = threadIdx.x; j < Lb && k < 32; ++k, j += blockDim.x) {
        if (!((open >> k) & 1u) || slot[fpos[j]] != j) continue;
        lsum[fpos[j]] += glab[j];
        slot[fpos[j]] = 0x7fffffff;
        open &= ~(1u << k);
      }
      if (!__syncthreads_or(open != 0u)) break;
    }
    for (int j = threadIdx.x; j < Lb; j += blockDim.x)
      if (fpos[j] == j) gam[lab[j]] = lsum[j];
  }
  __syncthreads();
  const float gs = gscale * (gdev ? gdev[0] : 1.f);
  const T* x = logits + (int64_t)row * ld;
  const float l = lse[row];
  auto gamma_of = [&](int c) {
    if (c == 0) return gb;
    return ((bits[c >> 5] >> (c & 31)) & 1u) ? gam[c] : 0.f;
  };
  if (vec) {
    for (int c0 = threadIdx.x * 8; c0 < V; c0 += blockDim.x * 8) {
      if (c0 + 8 <= V) {
        float v[8];
        ldv<8>(x + c0, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = gs * (__expf(v[q] - l) - gamma_of(c0 + q));
        stv<8>(g + c0, v);
      } else {
        for (int c = c0; c < V; ++c) g[c] = from_f<TG>(gs * (__expf(to_f(x[c]) - l) - gamma_of(c)));
      }
    }
    return;
  }
  for (int c = threadIdx.x; c < V; c += blockDim.x)
    g[c] = from_f<TG>(gs * (__expf(to_f(x[c]) - l) - gamma_of(c)));
}

// ---- the lattice with its emissions staged in LDS ---------------------------------------
// The block kernel above syncs each time step with __syncthreads(), a workgroup release fence
// that waits for every outstanding global access of the thread -- the step's alpha/beta store
// and the emission prefetch of the step CTC_PF ahead -- so each of the T' serial steps pays a
// memory round trip.  Here the emissions of CTC_CH steps are copied into LDS once per chunk
// (registers loaded at the chunk's start, written to LDS at its end, off the step chain), a
// step reads its emission from LDS, and the step barrier waits for LDS only; the alpha/beta
// stores drain in the background.  Per state the arithmetic is the block kernel's, in the same
// order: alpha, beta and nll are unchanged.
constexpr int CTC_CH = 32;   // time steps per emission chunk
constexpr int CTC_CHR = 17;  // chunk registers per thread: CTC_CH * ld / blockDim <= 17 (blockDim >= 2 ld - 1)

LASR_DEV void lds_step_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// dir = +1: alpha (t = 0 .. Tb-1), -1: beta (t = Tb-1 .. 0)
template <int DIR>
LASR_DEV void ctc_lattice_chunked(int b, int T_, int Lmax, const int32_t* __restrict__ targets, const int32_t* ilen,
                                  const int32_t* tlen, const float* lp, float* out, float* nll) {
  extern __shared__ float sh[];
  const int Tb = ilen[b], Lb = tlen[b], S = 2 * Lb + 1, Smax = 2 * Lmax + 1;
  if (Tb <= 0) {
    if (DIR > 0 && threadIdx.x == 0) nll[b] = (Lb == 0) ? 0.f : INFINITY;
    return;
  }
  const int32_t* tg = targets + (int64_t)b * Lmax;
  const int s = threadIdx.x, nt = blockDim.x;
  const bool act = s < S;
  const bool skip = DIR > 0 ? act && s >= 2 && (s & 1) && ext_label(tg, s) != ext_label(tg, s - 2)
                            : act && s + 2 < S && (s & 1) && ext_label(tg, s) != ext_label(tg, s + 2);
  const int eix = (s & 1) ? 1 + (s >> 1) : 0;
  const int ld = Lmax + 1;
  const float* lpu = lp + (int64_t)b * T_ * ld;  // the utterance's [T_][ld] emissions
  const int64_t last = (int64_t)T_ * ld - 1;
  float* o = out + (int64_t)b * T_ * Smax;
  float* buf0 = sh;
  float* buf1 = sh + Smax;
  float* chunk = sh + 2 * Smax;  // [CTC_CH][ld]: rows r0 .. r0 + CTC_CH - 1
  const int CHN = CTC_CH * ld;
  const int t_first = DIR > 0 ? 0 : Tb - 1;
  if (act) {
    const float e = lpu[(int64_t)t_first * ld + eix];
    const float v = DIR > 0 ? (s <= 1 ? e : -INFINITY) : (s >= S - 2 ? e : -INFINITY);
    buf0[s] = v;
    o[(int64_t)t_first * Smax + s] = v;
  }
  // chunk c holds the emissions of steps i = 1 + c CTC_CH .. (step i: t = t_first + DIR i);
  // its first row r0 = the lowest t of the chunk
  const int nsteps = Tb - 1;
  auto row0 = [&](int c) {
    const int i_lo = 1 + c * CTC_CH, i_hi = min(i_lo + CTC_CH - 1, nsteps);
    return DIR > 0 ? t_first + i_lo : t_first - i_hi;
  };
  float pre[CTC_CHR];
  auto load_regs = [&](int c) {
    const int64_t base = (int64_t)row0(c) * ld;
#pragma unroll
    for (int r = 0; r < CTC_CHR; ++r) {
      const int idx = r * nt + s;
      pre[r] = idx < CHN ? lpu[min(base + idx, last)] : 0.f;
    }
  };
  auto store_regs = [&]() {
#pragma unroll
    for (int r = 0; r < CTC_CHR; ++r) {
      const int idx = r * nt + s;
      if (idx < CHN) chunk[idx] = pre[r];
    }
  };
  const int nchunks = (nsteps + CTC_CH - 1) / CTC_CH;
  if (nchunks > 0) {
    load_regs(0);
    store_regs();
  }
  __syncthreads();
  float* prev = buf0;
  float* cur = buf1;
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) load_regs(c + 1);  // lands during this chunk's steps
    const int r0 = row0(c), i_lo = 1 + c * CTC_CH, i_hi = min(i_lo + CTC_CH - 1, nsteps);
    for (int i = i_lo; i <= i_hi; ++i) {
      const int t = t_first + DIR * i;
      if (act) {
        const float e = chunk[(t - r0) * ld + eix];
        float v;
        if (DIR > 0) {
          const float a0 = prev[s];
          const float a1 = s >= 1 ? prev[s - 1] : -INFINITY;
          const float a2 = skip ? prev[s - 2] : -INFINITY;
          v = lse3(a0, a1, a2) + e;
        } else {
          const float b0 = prev[s];
          const float b1 = (s + 1 < S) ? prev[s + 1] : -INFINITY;
          const float b2 = skip ? prev[s + 2] : -INFINITY;
          v = lse3(b0, b1, b2) + e;
        }
        cur[s] = v;
        o[(int64_t)t * Smax + s] = v;
      }
      lds_step_sync();
      float* tmp = prev; prev = cur; cur = tmp;
    }
    if (c + 1 < nchunks) {  // every wave is past its last read of this chunk (the step barrier)
      store_regs();
      lds_step_sync();
    }
  }
  if (DIR > 0 && threadIdx.x == 0) {
    const float ll = (S >= 2) ? lse2(prev[S - 1], prev[S - 2]) : prev[0];
    nll[b] = -ll;
  }
}

// ---- the lattice in registers, CTC_K steps per barrier ----------------------------------
// A step's state s needs s, s -/+ 1 and s -/+ 2 of the previous step: neighbouring lanes of
// one wave, read with DPP wave shifts instead of an LDS round trip and a block barrier per
// step.  Wave w owns CTC_OWN consecutive states and also computes the 2 CTC_K states beside
// them (the halo, on the side the recursion reads from): after k in-register steps the 2k
// outermost halo lanes are stale, so CTC_K steps leave every owned lane exact.  The owned
// lanes then publish their states to a double-buffered LDS vector and the block syncs once
// per CTC_K steps (the emission chunks stay staged in LDS as in ctc_lattice_chunked).  Per
// state the arithmetic is ctc_lattice_chunked's, operand for operand: alpha, beta and nll
// are unchanged.
constexpr int CTC_K = 8;
constexpr int CTC_OWN = 64 - 2 * CTC_K;
static_assert(CTC_CH % CTC_K == 0, "a step period never straddles an emission chunk");
LASR_DEV float dpp_shr1(float v) {  // lane l gets lane l - 1 (lane 0: -inf)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
LASR_DEV float dpp_shl1(float v) {  // lane l gets lane l + 1 (lane 63: -inf)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x130, 0xf, 0xf, false));
}
static int ctc_reg_waves(int Smax) { return (Smax + CTC_OWN - 1) / CTC_OWN; }
static size_t ctc_reg_lds(int Lmax) { return ((size_t)2 * (2 * Lmax + 1) + (size_t)CTC_CH * (Lmax + 1)) * sizeof(float); }

template <int DIR>
LASR_DEV void ctc_lattice_regs(int b, int T_, int Lmax, const int32_t* __restrict__ targets, const int32_t* ilen,
                               const int32_t* tlen, const float* lp, float* out, float* nll) {
  extern __shared__ float sh[];
  const int Tb = ilen[b], Lb = tlen[b], S = 2 * Lb + 1, Smax = 2 * Lmax + 1;
  if (Tb <= 0) {
    if (DIR > 0 && threadIdx.x == 0) nll[b] = (Lb == 0) ? 0.f : INFINITY;
    return;
  }
  const int32_t* tg = targets + (int64_t)b * Lmax;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nt = blockDim.x;
  // the lane's state; owned lanes publish it, halo lanes only feed their neighbours
  const int s = DIR > 0 ? w * CTC_OWN + lane - 2 * CTC_K : w * CTC_OWN + lane;
  const bool own = (DIR > 0 ? lane >= 2 * CTC_K : lane < CTC_OWN) && s < Smax;
  const bool act = s >= 0 && s < S;
  const bool skip = DIR > 0 ? act && s >= 2 && (s & 1) && ext_label(tg, s) != ext_label(tg, s - 2)
                            : act && s + 2 < S && (s & 1) && ext_label(tg, s) != ext_label(tg, s + 2);
  const bool near = DIR > 0 ? s >= 1 : s + 1 < S;  // the s -/+ 1 term exists
  const int eix = (s & 1) ? 1 + (s >> 1) : 0;
  const int ld = Lmax + 1;
  const float* lpu = lp + (int64_t)b * T_ * ld;
  const int64_t last = (int64_t)T_ * ld - 1;
  float* o = out + (int64_t)b * T_ * Smax;
  float* vec[2] = {sh, sh + Smax};
  float* chunk = sh + 2 * Smax;
  const int CHN = CTC_CH * ld;
  const int t_first = DIR > 0 ? 0 : Tb - 1;
  float v = -INFINITY;
  if (act) {
    const float e = lpu[(int64_t)t_first * ld + eix];
    v = DIR > 0 ? (s <= 1 ? e : -INFINITY) : (s >= S - 2 ? e : -INFINITY);
    if (own) o[(int64_t)t_first * Smax + s] = v;
  }
  if (own && act) vec[0][s] = v;
  const int nsteps = Tb - 1;
  auto row0 = [&](int c) {
    const int i_lo = 1 + c * CTC_CH, i_hi = min(i_lo + CTC_CH - 1, nsteps);
    return DIR > 0 ? t_first + i_lo : t_first - i_hi;
  };
  float pre[CTC_CHR];
  auto load_regs = [&](int c) {
    const int64_t base = (int64_t)row0(c) * ld;
#pragma unroll
    for (int r = 0; r < CTC_CHR; ++r) {
      const int idx = r * nt + threadIdx.x;
      pre[r] = idx < CHN ? lpu[min(base + idx, last)] : 0.f;
    }
  };
  auto store_regs = [&]() {
#pragma unroll
    for (int r = 0; r < CTC_CHR; ++r) {
      const int idx = r * nt + threadIdx.x;
      if (idx < CHN) chunk[idx] = pre[r];
    }
  };
  const int nchunks = (nsteps + CTC_CH - 1) / CTC_CH;
  if (nchunks > 0) {
    load_regs(0);
    store_regs();
  }
  __syncthreads();
  int cur = 0;
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) load_regs(c + 1);  // lands during this chunk's steps
    const int r0 = row0(c), i_lo = 1 + c * CTC_CH, i_hi = min(i_lo + CTC_CH - 1, nsteps);
    for (int p0 = i_lo; p0 <= i_hi; p0 += CTC_K) {
      // the period's start states (owned by this wave or its neighbour) and its emissions
      v = act ? vec[cur][s] : -INFINITY;
      float e[CTC_K];
#pragma unroll
      for (int k = 0; k < CTC_K; ++k) {
        const int t = t_first + DIR * (p0 + k);
        e[k] = act && p0 + k <= i_hi ? chunk[(t - r0) * ld + eix] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < CTC_K; ++k) {
        if (p0 + k > i_hi) break;  // block-uniform
        const float n1 = DIR > 0 ? dpp_shr1(v) : dpp_shl1(v);
        const float n2 = DIR > 0 ? dpp_shr1(n1) : dpp_shl1(n1);
        const float nv = lse3(v, near ? n1 : -INFINITY, skip ? n2 : -INFINITY) + e[k];
        v = act ? nv : -INFINITY;
        if (own && act) o[(int64_t)(t_first + DIR * (p0 + k)) * Smax + s] = v;
      }
      cur ^= 1;
      if (own && act) vec[cur][s] = v;
      lds_step_sync();
    }
    if (c + 1 < nchunks) {  // every wave is past its last read of this chunk (the period barrier)
      store_regs();
      lds_step_sync();
    }
  }
  if (DIR > 0 && threadIdx.x == 0) {
    const float* fin = vec[cur];
    const float ll = (S >= 2) ? lse2(fin[S - 1], fin[S - 2]) : fin[0];
    nll[b] = -ll;
  }
}

__global__ void ctc_lattice_regs_kernel(int B, int T_, int Lmax, const int32_t* __restrict__ targets,
                                        const int32_t* ilen, const int32_t* tlen, const float* lp, float* alpha,
                                        float* nll, float* beta, int beta_only) {
  if (!beta_only && (int)blockIdx.x < B)
    ctc_lattice_regs<1>(blockIdx.x, T_, Lmax, targets, ilen, tlen, lp, alpha, nll);
  else
    ctc_lattice_regs<-1>(beta_only ? blockIdx.x : blockIdx.x - B, T_, Lmax, targets, ilen, tlen, lp, beta, nullptr);
}

__global__ void ctc_lattice_chunked_kernel(int B, int T_, int Lmax, const int32_t* __restrict__ targets,
                                           const int32_t* ilen, const int32_t* tlen, const float* lp, float* alpha,
                                           float* nll, float* beta, int beta_only) {
  if (!beta_only && (int)blockIdx.x < B)
    ctc_lattice_chunked<1>(blockIdx.x, T_, Lmax, targets, ilen, tlen, lp, alpha, nll);
  else
    ctc_lattice_chunked<-1>(beta_only ? blockIdx.x : blockIdx.x - B, T_, Lmax, targets, ilen, tlen, lp, beta, nullptr);
}

static size_t ctc_chunk_lds(int Lmax) { return ((size_t)2 * (2 * Lmax + 1) + (size_t)CTC_CH * (Lmax + 1)) * sizeof(float); }

static int ctc_block(int S) {
  int nt = ((S + 63) / 64) * 64;
  return nt < 64 ? 64 : (nt > 1024 ? 1024 : nt);
}

extern "C" int lasr_ctc_fwd(const void* logits, int ldt, int B, int T, int V, int64_t ld,
                            const int32_t* targets, int Lmax, const int32_t* ilen,
                            const int32_t* tlen, float* lse, float* lp, float* alpha, float* beta,
                            float* nll, void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && V > 0 && Lmax >= 0 && ld >= V, "lasr_ctc_fwd: bad sizes");
  LASR_CHECK_ARG(ldt == LASR_F32 || ldt == LASR_BF16, "lasr_ctc_fwd: bad dtype");
  LASR_CHECK_ARG(2 * Lmax + 1 <= 1024, "lasr_ctc_fwd: Lmax=%d too large (one lattice state per thread)", Lmax);
  hipStream_t st = (hipStream_t)stream;
  if (ldt == LASR_F32)
    ctc_lse_gather_kernel<float><<<B * T, 256, 0, st>>>((const float*)logits, B, T, V, ld, targets, Lmax, ilen, tlen, lse, lp);
  else
    ctc_lse_gather_kernel<bf16_t><<<B * T, 256, 0, st>>>((const bf16_t*)logits, B, T, V, ld, targets, Lmax, ilen, tlen, lse, lp);
  int rc = lasr_check_launch("ctc_lse_gather");
  if (rc || !alpha) return rc;  // alpha == NULL: the log-softmax / gather stage only
  return lasr_ctc_lattice(B, T, Lmax, targets, ilen, tlen, lp, alpha, beta, nll, stream);
}

// the register-resident lattice when its block fits (64 lanes per CTC_OWN states);
// LASR_CTC_REGS=0 keeps the one-state-per-thread chunked kernel (same outputs)
static bool ctc_regs_ok(int Lmax) {
  static const bool on = [] { const char* e = getenv("LASR_CTC_REGS"); return !(e && e[0] == '0'); }();
  return on && 64 * ctc_reg_waves(2 * Lmax + 1) <= 1024 && ctc_reg_lds(Lmax) <= 64 * 1024;
}

extern "C" int lasr_ctc_lattice(int B, int T, int Lmax, const int32_t* targets, const int32_t* ilen,
                                const int32_t* tlen, const float* lp, float* alpha, float* beta, float* nll,
                                void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && Lmax >= 0 && 2 * Lmax + 1 <= 1024, "lasr_ctc_lattice: bad sizes");
  LASR_CHECK_ARG(lp && alpha && nll, "lasr_ctc_lattice: lp / alpha / nll");
  const int Smax = 2 * Lmax + 1;
  if (ctc_regs_ok(Lmax)) {
    ctc_lattice_regs_kernel<<<beta ? 2 * B : B, 64 * ctc_reg_waves(Smax), ctc_reg_lds(Lmax), (hipStream_t)stream>>>(
        B, T, Lmax, targets, ilen, tlen, lp, alpha, nll, beta, 0);
    return lasr_check_launch("ctc_lattice");
  }
  if (ctc_chunk_lds(Lmax) <= 64 * 1024) {
    ctc_lattice_chunked_kernel<<<beta ? 2 * B : B, ctc_block(Smax), ctc_chunk_lds(Lmax), (hipStream_t)stream>>>(
        B, T, Lmax, targets, ilen, tlen, lp, alpha, nll, beta, 0);
    return lasr_check_launch("ctc_lattice");
  }
  ctc_alpha_beta_kernel<<<beta ? 2 * B : B, ctc_block(Smax), 2 * Smax * sizeof(float), (hipStream_t)stream>>>(
      B, T, Lmax, targets, ilen, tlen, lp, alpha, nll, beta);
  return lasr_check_launch("ctc_alpha_beta");
}

extern "C" int lasr_ctc_bwd(const void* logits, int ldt, int B, int T, int V, int64_t ld,
                            const int32_t* targets, int Lmax, const int32_t* ilen,
                            const int32_t* tlen, const float* lse, const float* lp,
                            const float* alpha, const float* nll, float* beta, int beta_ready,
                            void* grad, int gdt, float gscale, const float* gdev, void* stream) {
  LASR_CHECK_ARG(B > 0 && T > 0 && V > 0 && Lmax >= 0 && ld >= V, "lasr_ctc_bwd: bad sizes");
  LASR_CHECK_ARG(2 * Lmax + 1 <= 1024, "lasr_ctc_bwd: Lmax=%d too large", Lmax);
  hipStream_t st = (hipStream_t)stream;
  const int Smax = 2 * Lmax + 1;
  if (!beta_ready && ctc_regs_ok(Lmax)) {
    ctc_lattice_regs_kernel<<<B, 64 * ctc_reg_waves(Smax), ctc_reg_lds(Lmax), st>>>(B, T, Lmax, targets, ilen, tlen, lp,
                                                                                    nullptr, nullptr, beta, 1);
    const int rc = lasr_check_launch("ctc_beta");
    if (rc) return rc;
  } else if (!beta_ready && ctc_chunk_lds(Lmax) <= 64 * 1024) {
    ctc_lattice_chunked_kernel<<<B, ctc_block(Smax), ctc_chunk_lds(Lmax), st>>>(B, T, Lmax, targets, ilen, tlen, lp,
                                                                                nullptr, nullptr, beta, 1);
    const int rc = lasr_check_launch("ctc_beta");
    if (rc) return rc;
  } else if (!beta_ready) {
    ctc_beta_kernel<<<B, ctc_block(Smax), 2 * Smax * sizeof(float), st>>>(T, Lmax, targets, ilen, tlen, lp, beta);
    const int rc = lasr_check_launch("ctc_beta");
    if (rc) return rc;
  }
  const size_t shm = ((size_t)5 * (((Lmax > 0 ? Lmax : 1) + 3) & ~3) + (V + 31) / 32 + V) * sizeof(float);
  LASR_CHECK_ARG(shm <= 64 * 1024 && Lmax <= 32 * 256, "lasr_ctc_bwd: vocab/labels too large for LDS");
#define CTC_G(TT, TGG)                                                                      \
  ctc_grad_kernel<TT, TGG><<<B * T, 256, shm, st>>>((const TT*)logits, B, T, V, ld, targets, Lmax,\
                                                    ilen, tlen, lse, lp, alpha, beta, nll,     \
                                                    (TGG*)grad, gscale, gdev)
  if (ldt == LASR_F32 && gdt == LASR_F32) CTC_G(float, float);
  else if (ldt == LASR_F32) CTC_G(float, bf16_t);
  else if (gdt == LASR_F32) CTC_G(bf16_t, float);
  else CTC_G(bf16_t, bf16_t);
#undef CTC_G
  return lasr_check_launch("ctc_grad");
}
