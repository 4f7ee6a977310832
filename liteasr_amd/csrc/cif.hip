// Continuous integrate-and-fire of the Paraformer predictor (liteasr/nets/paraformer/
// predictor.py:24-118) and the glancing sampler's mix (glancing_sampler.py:32).
//
// One wave per utterance: the scan over T' is sequential by definition (each frame's fire
// decision depends on the accumulated weight), so the parallel axis inside an utterance is
// the hidden dimension D (D / 64 values per lane); utterances run side by side.  The
// forward keeps, per frame, the accumulated weight after the frame, the fire flag and the
// output row the frame's fired state went to; the backward runs the adjoint recursion in
// reverse with those (no states are stored: the state adjoint only needs h and the
// weights).  All arithmetic fp32 with the reference's operation order (products and sums
// are separate roundings, as the reference's tensor expressions are).
#include "common.h"

#include <algorithm>

namespace {

struct CifP {
  int B, T, D, U;
  const float* z;      // [B*T] predictor logits (pre-sigmoid)
  const int* plen;     // [B] frames kept by the predictor mask (t < plen)
  const int* ylen;     // [B] target lengths (ulens)
  const float* h;      // [B, T, D] encoder output
  float* alpha;        // [B*T] out: masked sigmoid
  float* acc;          // [B*T] out: accumulated weight after frame t
  uint8_t* fired;      // [B*T] out: 1 when frame t fired
  int* row;            // [B*T] out: output row of the fired state (-1: none / past U)
  float* sum_alpha;    // [B] out
  float* mae;          // [B] out: |sum_alpha - ylen| (nullable)
  float* out;          // [B, U, D] out: fired states, fired-first, zero rows after
  // backward
  const float* gout;   // [B, U, D] gradient of out (nullable)
  const float* gsum;   // [B] gradient of sum_alpha from the loss (nullable)
  float* dz;           // [B*T] out: gradient of z
  float* dh;           // [B, T, D] out: gradient of h (written)
};

LASR_DEV float wave_sum_f(float v) { return wave_sum(v); }

template <int VPL>
__global__ __launch_bounds__(64) void cif_fwd_kernel(CifP p) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int T = p.T, D = p.D;
  const int plen = p.plen[b];
  // alpha and its sum (sequential fp32 order over t within a lane, then the wave tree)
  float part = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float zz = p.z[(int64_t)b * T + t];
    const float a = t < plen ? 1.f / (1.f + expf(-zz)) : 0.f;
    p.alpha[(int64_t)b * T + t] = a;
    part += a;
  }
  const float sum = wave_sum_f(part);
  const float beta = __fsub_rn(__fdiv_rn(sum, (float)p.ylen[b]), 1e-4f);
  if (lane == 0) {
    p.sum_alpha[b] = sum;
    if (p.mae) p.mae[b] = fabsf(sum - (float)p.ylen[b]);
  }
  float s[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) s[j] = 0.f;
  float prev = 0.f;
  int cnt = 0;
  const float* hb = p.h + (int64_t)b * T * D;
  float* ob = p.out + (int64_t)b * p.U * D;
  for (int t = 0; t < T; ++t) {
    // every lane recomputes alpha_t (same expression as above: same value)
    const float a = t < plen ? 1.f / (1.f + expf(-p.z[(int64_t)b * T + t])) : 0.f;
    const float nw = __fadd_rn(prev, a);
    const bool fire = nw >= beta;
    const float left = __fsub_rn(beta, prev), right = __fsub_rn(nw, beta);
    float hv[VPL], o[VPL];
    bool nz = false;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      hv[j] = hb[(int64_t)t * D + j * 64 + lane];
      o[j] = __fadd_rn(s[j], __fmul_rn(left, hv[j]));
      nz |= o[j] != 0.f;
    }
    int r = -1;
    if (fire) {
      if (__any(nz)) {  // rows whose |.|-sum is 0 count as not fired (predictor.py:105)
        if (cnt < p.U) {
          r = cnt;
#pragma unroll
          for (int j = 0; j < VPL; ++j) ob[(int64_t)cnt * D + j * 64 + lane] = o[j];
        }
        ++cnt;
      }
#pragma unroll
      for (int j = 0; j < VPL; ++j) s[j] = __fmul_rn(right, hv[j]);
      prev = right;
    } else {
#pragma unroll
      for (int j = 0; j < VPL; ++j) s[j] = o[j];
      prev = nw;
    }
    if (lane == 0) {
      p.acc[(int64_t)b * T + t] = prev;
      p.fired[(int64_t)b * T + t] = fire ? 1 : 0;
      p.row[(int64_t)b * T + t] = r;
    }
  }
  for (int u = cnt < p.U ? cnt : p.U; u < p.U; ++u)
#pragma unroll
    for (int j = 0; j < VPL; ++j) ob[(int64_t)u * D + j * 64 + lane] = 0.f;
}

template <int VPL>
__global__ __launch_bounds__(64) void cif_bwd_kernel(CifP p) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int T = p.T, D = p.D;
  const int plen = p.plen[b];
  const float sum = p.sum_alpha[b];
  const float yl = (float)p.ylen[b];
  const float beta = __fsub_rn(__fdiv_rn(sum, yl), 1e-4f);
  const float* hb = p.h + (int64_t)b * T * D;
  const float* gb = p.gout ? p.gout + (int64_t)b * p.U * D : nullptr;
  float* dhb = p.dh + (int64_t)b * T * D;
  float dS[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) dS[j] = 0.f;
  float dA = 0.f, dbeta = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const int64_t bt = (int64_t)b * T + t;
    const float a = p.alpha[bt];
    const float prev = t > 0 ? p.acc[bt - 1] : 0.f;
    const float nw = __fadd_rn(prev, a);
    const float left = __fsub_rn(beta, prev), right = __fsub_rn(nw, beta);
    const bool fire = p.fired[bt] != 0;
    const int r = p.row[bt];
    float hv[VPL], G[VPL];
    float ds_h = 0.f, g_h = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      hv[j] = hb[(int64_t)t * D + j * 64 + lane];
      G[j] = (r >= 0 && gb) ? gb[(int64_t)r * D + j * 64 + lane] : 0.f;
      ds_h += dS[j] * hv[j];
      g_h += G[j] * hv[j];
    }
    ds_h = wave_sum_f(ds_h);
    float da;
    if (fire) {
      g_h = wave_sum_f(g_h);
      const float dr = dA + ds_h;  // A_t = r, S_t = r h
#pragma unroll
      for (int j = 0; j < VPL; ++j) {
        dhb[(int64_t)t * D + j * 64 + lane] = right * dS[j] + left * G[j];
        dS[j] = G[j];  // F_t = S_{t-1} + l h
      }
      da = dr;
      dA = dr - g_h;
      dbeta += g_h - dr;
    } else {
#pragma unroll
      for (int j = 0; j < VPL; ++j) dhb[(int64_t)t * D + j * 64 + lane] = left * dS[j];  // S_t = S_{t-1} + l h
      da = dA;
      dA = dA - ds_h;
      dbeta += ds_h;
    }
    if (lane == 0) p.dz[bt] = da;  // scan part; the sum_alpha term is added below
  }
  const float dsum = dbeta / yl + (p.gsum ? p.gsum[b] : 0.f);  // beta = sum / ylen - 1e-4
  __syncthreads();
  for (int t = lane; t < T; t += 64) {
    const int64_t bt = (int64_t)b * T + t;
    const float a = p.alpha[bt];
    p.dz[bt] = t < plen ? (p.dz[bt] + dsum) * a * (1.f - a) : 0.f;
  }
}

// out[r, :] = replace[r] ? emb[r, :] : cif[r, :] (fwd); g_emb / g_cif split (bwd)
__global__ void glancing_mix_kernel(int64_t rows, int D, const uint8_t* rep, const float* a, const float* b,
                                    float* out, float* out2, int bwd) {
  const int64_t n = rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool r = rep[i / D] != 0;
    if (!bwd) {
      out[i] = r ? a[i] : b[i];
    } else {
      const float g = a[i];
      out[i] = r ? g : 0.f;   // -> embedding branch
      out2[i] = r ? 0.f : g;  // -> CIF branch
    }
  }
}

template <int VPL>
void launch_cif(const CifP& p, bool bwd, hipStream_t st) {
  if (bwd) cif_bwd_kernel<VPL><<<p.B, 64, 0, st>>>(p);
  else cif_fwd_kernel<VPL><<<p.B, 64, 0, st>>>(p);
}

int cif_dispatch(const CifP& p, bool bwd, hipStream_t st) {
  switch (p.D / 64) {
    case 1: launch_cif<1>(p, bwd, st); break;
    case 2: launch_cif<2>(p, bwd, st); break;
    case 4: launch_cif<4>(p, bwd, st); break;
    case 8: launch_cif<8>(p, bwd, st); break;
    case 16: launch_cif<16>(p, bwd, st); break;
    default: return LASR_ERR_INVALID;
  }
  return lasr_check_launch(bwd ? "lasr_cif_bwd" : "lasr_cif_fwd");
}

bool cif_shape_ok(int B, int T, int D, int U) {
  const int v = D / 64;
  return B > 0 && T > 0 && U > 0 && D % 64 == 0 && (v == 1 || v == 2 || v == 4 || v == 8 || v == 16);
}

}  // namespace

extern "C" int lasr_cif_fwd(const lasr_cif_args* a, void* stream) {
  LASR_CHECK_ARG(a && cif_shape_ok(a->B, a->T, a->D, a->U), "lasr_cif_fwd: bad shape (D in 64,128,256,512,1024)");
  LASR_CHECK_ARG(a->z && a->plen && a->ylen && a->h && a->alpha && a->acc && a->fired && a->row && a->sum_alpha &&
                     a->out, "lasr_cif_fwd: null pointer");
  CifP p{};
  p.B = a->B; p.T = a->T; p.D = a->D; p.U = a->U;
  p.z = a->z; p.plen = a->plen; p.ylen = a->ylen; p.h = a->h;
  p.alpha = a->alpha; p.acc = a->acc; p.fired = a->fired; p.row = a->row; p.sum_alpha = a->sum_alpha;
  p.mae = a->mae; p.out = a->out;
  return cif_dispatch(p, false, (hipStream_t)stream);
}

extern "C" int lasr_cif_bwd(const lasr_cif_args* a, void* stream) {
  LASR_CHECK_ARG(a && cif_shape_ok(a->B, a->T, a->D, a->U), "lasr_cif_bwd: bad shape");
  LASR_CHECK_ARG(a->plen && a->ylen && a->h && a->alpha && a->acc && a->fired && a->row && a->sum_alpha && a->dz &&
                     a->dh, "lasr_cif_bwd: null pointer");
  CifP p{};
  p.B = a->B; p.T = a->T; p.D = a->D; p.U = a->U;
  p.plen = a->plen; p.ylen = a->ylen; p.h = a->h;
  p.alpha = a->alpha; p.acc = a->acc; p.fired = a->fired; p.row = a->row; p.sum_alpha = a->sum_alpha;
  p.gout = a->gout; p.gsum = a->gsum; p.dz = a->dz; p.dh = a->dh;
  return cif_dispatch(p, true, (hipStream_t)stream);
}

extern "C" int lasr_glancing_mix(int64_t rows, int D, const uint8_t* replace, const float* a, const float* b,
                                 float* out, float* out2, int backward, void* stream) {
  LASR_CHECK_ARG(rows >= 0 && D > 0 && replace && a && out && (backward ? out2 != nullptr : b != nullptr),
                 "lasr_glancing_mix: bad arguments");
  if (rows == 0) return LASR_OK;
  const int64_t n = rows * D;
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 4096);
  glancing_mix_kernel<<<nb, 256, 0, (hipStream_t)stream>>>(rows, D, replace, a, b, out, out2, backward);
  return lasr_check_launch("lasr_glancing_mix");
}
